#!/bin/bash
# After a kernel change: full GPU suite (stop at first failure), bench at the
# driver's shape and at 200 epochs, and the per-wave timeline of a 20-epoch launch.
set -u
TAG=${1:-quick}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { grep -E "FAILED|^E " "$OUT/pytest_gpu.log" | head -30; tail -3 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for s in 20 200; do
  timeout -k 10 300 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline > "$OUT/bench_s$s.json" 2> "$OUT/bench_s$s.err" || { tail -20 "$OUT/bench_s$s.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_s$s.json')); t=d['timing']; print('s$s', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'], 'outside %.3f ms' % t['outside_kernel_ms'])"
done
if [ -f slam-uwv_kalman_filters_amd/libuwvk_timeline.so ]; then
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_timeline.so timeout -k 10 200 python tools/timeline.py --steps 20 --out "$OUT/tl_s20.npz"
fi
