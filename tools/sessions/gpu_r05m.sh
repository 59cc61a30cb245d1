#!/bin/bash
# r05m: PSP_PSEL alone against + PSP_HVGPR (the measurement Jacobian
# in VGPRs), + PSP_QMB (staged-row slot by v_mbcnt) and both; four interleaved
# C3 rounds against the shipped build; parity of the ph and pqh variants first.

set -u
OUT=$PWD/gpurun_out/r05m
mkdir -p "$OUT"
PKGD=$PWD/slam-uwv_kalman_filters_amd
for v in ph pqh; do UWVK_LIB=$PKGD/libuwvk_$v.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_efforts.py tests/test_gpu_so3_side.py \
  -q -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { tail -30 "$OUT/pytest_$v.txt"; exit 1; }
echo "$v: $(tail -1 $OUT/pytest_$v.txt)"; done
bash tools/ab_variants.sh r05m 4 psel ph pq pqh | tee "$OUT/summary.txt"
