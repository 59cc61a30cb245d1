#!/bin/bash
# r05o: small VALU cuts as A/B variants of the PSP unit (the shipped build
# already reads the update's Gr entries with constant lane masks):
#   q1  the uniform quaternion stored by one lane (no lane-indexed select chain) (PSP_Q1)
#   zs  the rank-M K padding read from a zero slot instead of selected (PSP_ZSLOT)
#   qz  both
#   qzd both + the 4-lane window sums of wave_sum_dpp by doubling (PSP_DPP2)
# Parity of qz under UWVK_LIB, then four interleaved C3 rounds.
set -u
OUT=$PWD/gpurun_out/r05o
mkdir -p "$OUT"
PKGD=$PWD/slam-uwv_kalman_filters_amd
for v in qz qzd; do UWVK_LIB=$PKGD/libuwvk_$v.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_efforts.py tests/test_gpu_so3_side.py \
  -q -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { tail -30 "$OUT/pytest_$v.txt"; exit 1; }
echo "$v: $(tail -1 $OUT/pytest_$v.txt)"; done
bash tools/ab_variants.sh r05o 4 q1 zs qz qzd | tee "$OUT/summary.txt"
