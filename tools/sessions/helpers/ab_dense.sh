#!/bin/bash
# A/B of the literal (dense) C3 bench line against variant libraries.
set -u
OUT=$PWD/gpurun_out/abdense
mkdir -p "$OUT"
for v in "$@"; do
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so timeout -k 10 300 python bench.py --dense --steps 50 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', '%.3fM steps/s' % (d['value']/1e6), d['ensemble'])"
done
