#!/bin/bash
# r03t: GPU suite on the final tree, secondary bench lines (C4 / C2 / C5 shard /
# C5 two-rank rehearsal), and a rocprofv3 kernel trace of the driver's bench shape.
# Usage (repo root, on the box): bash tools/gpu_r03t.sh TAG
set -u
TAG=${1:-r03t}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
bash tools/gpu_lines_r03.sh "$TAG" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/s20_traced.json" 2> "$OUT/s20_traced.err" \
  || { tail -20 "$OUT/s20_traced.err"; exit 1; }
cut -c1-200 "$OUT/s20_traced.json"
