#!/bin/bash
# r06d: the parameter-decoupled kernel at 4 waves per SIMD (libuwvk_w4.so:
# amdgpu_waves_per_eu(4, 4) on the epoch kernels; the 53-DOF layout stays at 3,
# LDS-bound) against the shipped 3-wave build, interleaved, 20 and 200 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/ab_lib_args.sh $TAG/s200 3 "--steps 200 --warmup 5" base w4 || exit 1
bash tools/ab_lib_args.sh $TAG/s20 3 "--steps 20 --warmup 5" base w4 || exit 1
echo "r06d $TAG done"
