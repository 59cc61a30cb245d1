#!/bin/bash
# Kernel time per launch against epochs per launch (C3, batch 65,536): the
# intercept of the linear fit is the per-launch fixed cost (Sigma~ load / store
# per instance, the end-of-launch ramp).  ARGS: extra bench arguments.
# Usage (repo root, on the box): bash tools/epochs_sweep.sh TAG LABEL "ARGS"
set -u
TAG=$1; LABEL=$2; ARGS=${3:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
for s in 1 2 5 10 20 50; do
  timeout -k 10 200 python3 bench.py --steps $s --warmup 3 --no-cpu-baseline $ARGS > "$OUT/${LABEL}_s$s.json" 2> "$OUT/${LABEL}_s$s.err" || { tail -5 "$OUT/${LABEL}_s$s.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.4f ms' % d['roofline']['kernel_ms_per_launch'], '%.1f M' % (d['value']/1e6))" "$OUT/${LABEL}_s$s.json" "$LABEL" "$s"
done
