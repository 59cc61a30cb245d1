#!/bin/bash
# r04: the fixed lane-mask variant: full GPU suite with libuwvk_lmfix.so copied
# over libuwvk.so (the facade test links -luwvk), then the C3 A/B against the
# committed library.  Usage (repo root, on the box): bash tools/ab_lmfix.sh TAG [VARIANT (default lmfix)]
set -u
TAG=$1; V=${2:-lmfix}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
D=$PWD/slam-uwv_kalman_filters_amd
cp "$D/libuwvk.so" "$D/libuwvk_head.so"
cp "$D/libuwvk_${V}.so" "$D/libuwvk.so"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1
rc=$?
cp "$D/libuwvk_head.so" "$D/libuwvk.so"
tail -2 "$OUT/pytest_gpu.txt"
[ $rc -eq 0 ] || exit 1
bash tools/ab_r04.sh "$TAG" 3 head "$V"
