#!/bin/bash
# rocprofv3 kernel trace of the C4 bench (2,000-epoch window, compressed drop-out
# cycle): splits the time between the PSP launches and the literal BodyEfforts
# launches.  Usage (repo root, on the box): bash tools/gpu_c4_prof.sh TAG
set -u
TAG=${1:-c4prof}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --mode C4 --steps 2000 --c4-cycle 0.3,0.1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { tail -30 "$OUT/bench.err"; exit 1; }
cut -c1-200 "$OUT/bench.json"
cut -c1-170 "$OUT/prof/run_kernel_stats.csv"
