#!/bin/bash
# GPU suite, then the C4 kernel split (tools/gpu_c4_prof.sh).  Usage: bash tools/gpu_check_c4.sh TAG
set -u
TAG=${1:-checkc4}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
bash tools/gpu_c4_prof.sh "$TAG"
