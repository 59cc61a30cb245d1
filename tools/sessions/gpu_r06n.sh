#!/bin/bash
# r06n: run_log splits launches around the pressure epochs so that the runs
# between them take the pair kernel (ADCP update compiled into
# k_psp_epoch_pair<SR, 0>): the GPU suite, then C4 over the full drop-out cycle
# with the split (default) against --pair 0 (one-instance PD kernel), two
# rounds, and the C3 driver shape.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'kernel_ms', t.get('kernel_ms'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'), d['config']['kernel'][:120])"; }
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
for r in 1 2; do
  for v in split single; do
    args=""; [ "$v" = single ] && args="--pair 0"
    timeout -k 10 600 python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline $args > "$OUT/c4_$v-r$r.json" 2> "$OUT/c4_$v-r$r.err" || { tail -20 "$OUT/c4_$v-r$r.err"; exit 1; }
    line "$OUT/c4_$v-r$r.json" c4_$v-r$r
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
  python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c4_cycle_traced.json" 2> "$OUT/c4_cycle_traced.err" \
  || { tail -20 "$OUT/c4_cycle_traced.err"; exit 1; }
line "$OUT/c4_cycle_traced.json" c4_cycle_traced
cut -c1-160 "$OUT/c4prof/run_kernel_stats.csv" | head -8
echo "r06n $TAG done"
