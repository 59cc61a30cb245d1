#!/bin/bash
# r06w: no tail spreading for pair launches by default: the GPU suite, then the
# driver-shaped C3 line with its CPU baseline and its rocprofv3 trace, 200
# epochs, the 26-DOF handles, C4's cycle and the C5 shard.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'kernel_ms', t.get('kernel_ms'), 'frac', (d.get('roofline') or {}).get('frac'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'))"; }
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_traced.json" 2> "$OUT/c3_s20_traced.err" || { tail -5 "$OUT/c3_s20_traced.err"; exit 1; }
line "$OUT/c3_s20_traced.json" c3_s20_traced
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_r$r.json" 2> "$OUT/c3_s20_r$r.err" || { tail -5 "$OUT/c3_s20_r$r.err"; exit 1; }
  line "$OUT/c3_s20_r$r.json" c3_s20_r$r
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c3_s200_r$r.json" 2> "$OUT/c3_s200_r$r.err" || { tail -5 "$OUT/c3_s200_r$r.err"; exit 1; }
  line "$OUT/c3_s200_r$r.json" c3_s200_r$r
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dof 26 > "$OUT/c3_dof26_s20.json" 2> "$OUT/c3_dof26.err" || { tail -5 "$OUT/c3_dof26.err"; exit 1; }
line "$OUT/c3_dof26_s20.json" c3_dof26_s20
timeout -k 10 300 python3 bench.py --mode C5 --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c5_shard.json" 2> "$OUT/c5.err" || { tail -5 "$OUT/c5.err"; exit 1; }
line "$OUT/c5_shard.json" c5_shard
timeout -k 10 600 python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c4_cycle.json" 2> "$OUT/c4_cycle.err" || { tail -20 "$OUT/c4_cycle.err"; exit 1; }
line "$OUT/c4_cycle.json" c4_cycle
echo "r06w $TAG done"
