#!/bin/bash
# r03v: BodyEfforts one-wave Cholesky A/B (w1) against the shipped kernel (new),
# two interleaved rounds, then the self-launch tests (2 and 4 ranks on one GPU).
set -u
TAG=${1:-r03v}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/ab_eff.sh "$TAG/abeff3" 2 w1 new || exit 1
unset UWVK_LIB
timeout -k 10 900 python -u -m pytest tests/test_distributed.py -q -m gpu -x -k self_launches --timeout 600 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_self_launch.txt" 2>&1 || { tail -30 "$OUT/pytest_self_launch.txt"; exit 1; }
tail -1 "$OUT/pytest_self_launch.txt"
