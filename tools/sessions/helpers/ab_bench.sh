#!/bin/bash
# A/B: bench.py against each variant library given on the command line.
set -u
OUT=$PWD/gpurun_out/ab
mkdir -p "$OUT"
for v in "$@"; do
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/$v.json')); print('$v', '%.2fM steps/s' % (d['value']/1e6), '%.3f ms/epoch' % d['ms_per_step'])"
done
