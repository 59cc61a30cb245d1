#!/bin/bash
# Quick GPU-box check after a change: the GPU test suite, then one C3 bench
# line under rocprofv3 --kernel-trace --stats.
# Usage (from the repo root, on the box): bash tools/gpu_check.sh TAG
set -u
TAG=${1:-check}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 200 --warmup 2 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
cut -c1-200 "$OUT/bench.json"
cut -c1-150 "$OUT/prof/run_kernel_stats.csv"
