#!/bin/bash
# A/B timing of PSP variants (libuwvk_<V>.so built by `make variant`): kernel ms per launch of the C3 bench.
# usage: tools/ablate.sh V1 V2 ...   (base = libuwvk.so)
set -e
mkdir -p gpurun_out
out=gpurun_out/ablate.txt
: > $out
for v in base "$@"; do
  if [ "$v" = base ]; then lib=slam-uwv_kalman_filters_amd/libuwvk.so; else lib=slam-uwv_kalman_filters_amd/libuwvk_$v.so; fi
  UWVK_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']; print('%-10s %8.3f ms/launch  %7.1f M steps/s' % ('$v', r['kernel_ms_per_launch'], d['value']/1e6))" >> $out
done
cat $out
