#!/bin/bash
# Round-end record of the committed tree: the GPU suite, then the bench lines
# and smoke() of tools/gpu_lines.sh.  Usage (repo root, on the box): bash tools/gpu_round_end.sh TAG
set -u
TAG=${1:-end}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
bash tools/gpu_lines.sh "$TAG"
