#!/bin/bash
# A/B of the C4 bench (2,000 epochs, compressed drop-out cycle) against variant libraries.
set -u
OUT=$PWD/gpurun_out/abc4
mkdir -p "$OUT"
for v in "$@"; do
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so timeout -k 10 300 python bench.py --mode C4 --steps 2000 --c4-cycle 0.3,0.1 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$v.json')); print('$v', '%.2fM steps/s' % (d['value']/1e6), d['ensemble'])"
done
