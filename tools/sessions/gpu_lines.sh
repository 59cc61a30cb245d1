#!/bin/bash
# Bench lines of the current tree: the driver's shape (with the CPU baseline),
# 200 epochs, a world-size-1 torchrun (engine RCCL communicator), C4 over a
# 2,000-epoch window with the compressed drop-out cycle, C2, and smoke().
set -u
TAG=${1:-lines}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', '%.2fM' % (d['value']/1e6), d.get('timing'), (d.get('cpu_baseline') or {}).get('value'))"
}
run s20 400 python3 bench.py --steps 20 --warmup 5
run s200 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline
run torchrun1 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --steps 20 --warmup 5 --no-cpu-baseline
run c4 400 python3 bench.py --mode C4 --steps 2000 --warmup 5 --c4-cycle 0.3,0.1 --no-cpu-baseline
run c2 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
