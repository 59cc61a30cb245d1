#!/bin/bash
# A/B of variant libraries at several window lengths: kernel ms per launch (HIP events)
# Usage: bash tools/ab_steps.sh "20 200" base noload ...   (base = libuwvk.so)
set -u
OUT=$PWD/gpurun_out/ab_steps
mkdir -p "$OUT"
STEPS=$1; shift
for v in "$@"; do
  lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
  [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
  for s in $STEPS; do
    UWVK_LIB=$lib timeout -k 10 200 python bench.py --steps $s --warmup 5 --no-cpu-baseline > "$OUT/$v-$s.json" 2> "$OUT/$v-$s.err" || { echo "$v $s failed"; tail -5 "$OUT/$v-$s.err"; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$v-$s.json')); t=d['timing']; print('$v', $s, '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'], 'outside %.3f ms' % t['outside_kernel_ms'])"
  done
done
