#!/bin/bash
# GPU suite, smoke(), 20/200-epoch bench lines and a kernel trace of the 20-epoch line.
# Usage (repo root, on the box): bash tools/gpu_check2.sh TAG
set -u
TAG=${1:-chk}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
for S in 20 200; do
  timeout -k 10 300 python bench.py --steps $S --warmup 5 > "$OUT/bench_s$S.json" 2> "$OUT/bench_s$S.err" || { tail -20 "$OUT/bench_s$S.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_s$S.json'));print($S, d['value']/1e6, d['timing'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_s20_traced.json" 2> "$OUT/trace_s20.err" || { tail -20 "$OUT/trace_s20.err"; exit 1; }
echo done
