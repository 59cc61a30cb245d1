#!/bin/bash
# r06r: the pair kernel for 26-DOF handles too (k_psp_epoch_pair<SR, EVS, 0>):
# the GPU suite, then interleaved A/B of 26-DOF C3 with the pair kernel
# (default) against --pair 0 (one-instance kernel at 4 waves), two rounds,
# 20 / 200 epochs, and the 53-DOF driver shape.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'kernel_ms', t.get('kernel_ms'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'), d['config']['kernel'][:90])"; }
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
for r in 1 2; do
  for v in pair single; do
    args=""; [ "$v" = single ] && args="--pair 0"
    for st in 20 200; do
      timeout -k 10 300 python3 bench.py --dof 26 --steps $st --warmup 5 --no-cpu-baseline $args > "$OUT/d26_$v-s$st-r$r.json" 2> "$OUT/d26_$v-s$st-r$r.err" || { tail -20 "$OUT/d26_$v-s$st-r$r.err"; exit 1; }
      line "$OUT/d26_$v-s$st-r$r.json" d26_$v-s$st-r$r
    done
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
echo "r06r $TAG done"
