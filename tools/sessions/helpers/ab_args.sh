#!/bin/bash
# Interleaved A/B of bench.py argument sets on one library (C3 by default):
# ROUNDS passes, each running every argument set once.
# Usage (repo root, on the box): bash tools/ab_args.sh TAG ROUNDS "name1:args1" "name2:args2" ...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    n=${spec%%:*}; args=${spec#*:}
    f="$OUT/$n-r$r"
    timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > "$f.json" 2> "$f.err" || { echo "$n failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d.get('timing') or {}; print('$n', 'r$r', '%.2fM' % (d['value']/1e6), 'kernel %s ms' % t.get('kernel_ms'), 'ms_per_step %.5f' % d['ms_per_step'])"
  done
done
