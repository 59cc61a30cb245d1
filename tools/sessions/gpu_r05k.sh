#!/bin/bash
# r05k: rank-M tile loads / stores through per-row LDS pointers (PSP_RANKM_VOL,
# libuwvk_rvol.so): parity of the variant (the GPU parity and efforts tests
# under UWVK_LIB), then an interleaved C3 A/B against the shipped build.
set -u
OUT=$PWD/gpurun_out/r05k
mkdir -p "$OUT"
PKGD=$PWD/slam-uwv_kalman_filters_amd
UWVK_LIB=$PKGD/libuwvk_rvol.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_efforts.py tests/test_gpu_so3_side.py \
  -q -m gpu -x --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_rvol.txt" 2>&1 || { tail -30 "$OUT/pytest_rvol.txt"; exit 1; }
tail -1 "$OUT/pytest_rvol.txt"
bash tools/ab_variants.sh r05k 3 rvol | tee "$OUT/summary.txt"
