#!/bin/bash
# r06zd: the pair unit with the issue-priority raise also over the manifold
# mean and the update's gain chain (libuwvk_moreprio.so) against the default
# (libuwvk.so): interleaved, three rounds,
# 20 / 200 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for v in base moreprio; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], 'nees %.9f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
echo "r06zd $TAG done"
