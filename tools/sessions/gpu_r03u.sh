#!/bin/bash
# r03u: second BodyEfforts A/B round (reversed order) and the C5 eight-rank
# rehearsal on one GPU (8 x 131,072 = 1,048,576 instances, gloo sum: RCCL refuses
# two ranks on one device).  Usage (repo root, on the box): bash tools/gpu_r03u.sh TAG
set -u
TAG=${1:-r03u}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/ab_eff.sh "$TAG/abeff2" 2 c3 new base || exit 1
unset UWVK_LIB
for K in 20 200; do
  timeout -k 10 600 env UWVK_BENCH_SAME_DEVICE=1 python3 bench.py --gpus 8 --mode C5 --steps $K --warmup 5 \
    > "$OUT/c5_gpus8_same_s$K.json" 2> "$OUT/c5_gpus8_same_s$K.err" || { tail -30 "$OUT/c5_gpus8_same_s$K.err"; exit 1; }
  cut -c1-400 "$OUT/c5_gpus8_same_s$K.json"
done
