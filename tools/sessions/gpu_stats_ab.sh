#!/bin/bash
# Statistics-path check: the ensemble/timer GPU tests, then the 20-epoch bench
# line under a kernel trace (k_pose_stats / k_pose_stats_sum durations).
# Usage (repo root, on the box): bash tools/gpu_stats_ab.sh TAG
set -u
TAG=${1:-stats}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_distributed.py tests/test_gpu_edges.py -q -m gpu -x --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_s20_traced.json" 2> "$OUT/trace_s20.err" || { tail -20 "$OUT/trace_s20.err"; exit 1; }
grep -i stats "$OUT/trace_s20/run_kernel_stats.csv" | cut -c1-150
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_s20_$i.json" 2> "$OUT/bench_s20_$i.err" || { tail -20 "$OUT/bench_s20_$i.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_s20_$i.json'));print(d['value']/1e6, d['timing'])"
done
echo done
