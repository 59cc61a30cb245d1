#!/bin/bash
# Interleaved A/B of variant libraries (libuwvk_<v>.so; base = libuwvk.so) on the
# C3 bench: ROUNDS passes over the variants, each at every window length.
# Usage (repo root, on the box): bash tools/ab_r03.sh TAG ROUNDS "20 200" base v1 v2 ...
set -u
TAG=$1; ROUNDS=$2; STEPS=$3; shift 3
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for s in $STEPS; do
      f="$OUT/$v-s$s-r$r"
      UWVK_LIB=$lib timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "$v $s failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d['timing']; print('$v', $s, 'r$r', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'], 'nees %.2f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
