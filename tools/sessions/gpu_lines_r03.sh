#!/bin/bash
# Secondary bench lines of round 3: C4 (2,000 epochs, compressed drop-out
# cycle), C2 (VelocityUKF batch 4,096), C5's shard on one GPU (131,072 x 200
# epochs), the C5 two-rank rehearsal on one GPU.
# Usage (repo root, on the box): bash tools/gpu_lines_r03.sh TAG
set -u
TAG=${1:-r03}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', '%.2fM' % (d['value']/1e6), d.get('n_gpus'), d.get('timing'), (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'))"
}
run c4 400 python3 bench.py --mode C4 --steps 2000 --warmup 5 --c4-cycle 0.3,0.1 --no-cpu-baseline
run c2 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline
run c5shard 300 python3 bench.py --mode C5 --steps 200 --warmup 5 --no-cpu-baseline
run c5_gpus2_same 400 env UWVK_BENCH_SAME_DEVICE=1 python3 bench.py --gpus 2 --mode C5 --steps 200 --warmup 5
