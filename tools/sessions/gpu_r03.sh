#!/bin/bash
# Round-3 GPU session: the GPU suite, the driver's bench shape, 200 epochs, the
# self-launched two-rank rehearsal (one GPU), and smoke().
# Usage (repo root, on the box): bash tools/gpu_r03.sh TAG [suite|nosuite]
set -u
TAG=${1:-r03}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-suite}" = suite ]; then
  timeout -k 10 1000 python -u -m pytest tests -q -m gpu -x --timeout 900 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -20 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', '%.2fM' % (d['value']/1e6), d.get('n_gpus'), d.get('timing'), (d.get('cpu_baseline') or {}).get('value'))"
}
run s20 400 python3 bench.py --steps 20 --warmup 5
run s200 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline
run gpus2_same 400 env UWVK_BENCH_SAME_DEVICE=1 python3 bench.py --gpus 2 --steps 20 --warmup 5
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
