#!/bin/bash
# Parity tests of variant libraries (libuwvk_<v>.so) before an A/B: the GPU
# parity file against the oracle, one pytest process per variant.
# Usage (repo root, on the box): bash tools/ab_parity.sh TAG v1 v2 ...
set -u
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tail.py -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/parity_$v.log" 2>&1 || { echo "$v parity failed"; tail -30 "$OUT/parity_$v.log"; exit 1; }
  echo "$v $(tail -1 "$OUT/parity_$v.log")"
done
