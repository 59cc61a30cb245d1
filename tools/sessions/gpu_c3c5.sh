#!/bin/bash
# C3 over a 2,000-epoch window and the C5 shard size (131,072 instances on one GPU).
set -u
TAG=${1:-c3c5}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python bench.py --steps 2000 --no-cpu-baseline > "$OUT/c3_2000.json" 2> "$OUT/c3.err" || { tail -20 "$OUT/c3.err"; exit 1; }
cut -c1-160 "$OUT/c3_2000.json"
timeout -k 10 400 python bench.py --batch-per-gpu 131072 --no-cpu-baseline > "$OUT/c5shard.json" 2> "$OUT/c5.err" || { tail -20 "$OUT/c5.err"; exit 1; }
cut -c1-160 "$OUT/c5shard.json"
