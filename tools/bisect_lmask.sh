#!/bin/bash
# r04 bisect of the lane-mask experiment: the facade (300 single-call epochs)
# and the parity file against variant libraries copied over libuwvk.so on the
# box (the facade test links -luwvk).  Usage: bash tools/bisect_lmask.sh TAG v1 v2 ...
set -u
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
cp "$LIB" "$OUT/libuwvk_head.so"
for v in "$@"; do
  cp "$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so" "$LIB"
  timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_facade.py tests/test_gpu_parity.py -m gpu -p no:cacheprovider > "$OUT/$v.txt" 2>&1
  echo "$v: $(tail -1 $OUT/$v.txt) | $(grep -h 'worst' $OUT/$v.txt | head -1)"
  grep FAILED "$OUT/$v.txt" | head -8
done
cp "$OUT/libuwvk_head.so" "$LIB"
