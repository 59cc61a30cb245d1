#!/bin/bash
# r04: the model-change VelocityUKF test (now with W != B and general centres)
# on the shipped library and on the VEL_GLIN variant.
set -o pipefail
O=gpurun_out/gl2; mkdir -p $O
for v in ${GL2_VARIANTS:-base gl}; do
  lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
  [ $v != base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
  UWVK_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -k "velocity" -x -v --timeout 120 --timeout-method thread \
    > $O/pytest_vel_$v.txt 2>&1 || { tail -30 $O/pytest_vel_$v.txt; exit 1; }
  tail -1 $O/pytest_vel_$v.txt
done
