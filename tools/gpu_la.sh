#!/bin/bash
# r04: look-ahead two-wave Cholesky (UWVK_CHOL_LA) in the literal kernels:
# bitwise comparison against the previous build, the efforts A/B, the GPU suite.
set -o pipefail
O=gpurun_out/effla; mkdir -p $O
P=$PWD/slam-uwv_kalman_filters_amd
timeout -k 10 300 python3 -u tools/diag_lib_bitwise.py $P/libuwvk_b0.so $P/libuwvk_la.so > $O/bitwise.txt 2>&1 || { tail -20 $O/bitwise.txt; exit 1; }
tail -5 $O/bitwise.txt
bash tools/ab_eff.sh effla 2 b0 la > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
