#!/bin/bash
# r06zb: the statistics warm-up ahead of the untimed epochs and the remainder
# launch first (the launch before the window is a full-length one): the GPU
# suite, the driver-shaped line with its CPU baseline, the rocprofv3 trace /
# stats of the same command, and two more 20-epoch lines.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'kernel_ms', t.get('kernel_ms'), 'frac', (d.get('roofline') or {}).get('frac'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'))"; }
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_traced.json" 2> "$OUT/c3_s20_traced.err" || { tail -5 "$OUT/c3_s20_traced.err"; exit 1; }
line "$OUT/c3_s20_traced.json" c3_s20_traced
cut -c1-200 "$OUT/trace_s20/run_kernel_stats.csv" | head -3
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_r$r.json" 2> "$OUT/c3_s20_r$r.err" || { tail -5 "$OUT/c3_s20_r$r.err"; exit 1; }
  line "$OUT/c3_s20_r$r.json" c3_s20_r$r
done
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c3_s200.json" 2> "$OUT/c3_s200.err" || { tail -5 "$OUT/c3_s200.err"; exit 1; }
line "$OUT/c3_s200.json" c3_s200
echo "r06zb $TAG done"
