#!/bin/bash
# r06zh: what a live RCCL communicator costs the pair kernel (VERDICT r05 weak
# #9), on one GPU: no communicator, a one-rank communicator through the timed
# region (UWVK_BENCH_COLL=rccl1, the N > 1 lifetime) and one made around each
# statistics all-reduce (=scoped); C5 (200 epochs) and C3 at the driver shape,
# interleaved, two rounds.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in none rccl1 scoped; do
    for m in "C5 200" "C3 20"; do
      set -- $m
      f="$OUT/$v-$1-s$2-r$r"
      UWVK_BENCH_COLL=$v timeout -k 10 300 python3 bench.py --mode $1 --no-cpu-baseline --steps $2 --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v $m failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v $1 s$2 r$r', '%.2fM' % (d['value']/1e6), 'wall', round(d['timing']['wall_ms'], 3), 'kernel', round(d['timing']['kernel_ms'], 3), d['config'].get('collective'), 'nees %.9f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
echo "r06zh $TAG done"
