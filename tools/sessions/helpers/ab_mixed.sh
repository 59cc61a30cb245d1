#!/bin/bash
# Interleaved A/B over (library, bench.py arguments) pairs: ROUNDS passes.
# Usage (repo root, on the box): bash tools/ab_mixed.sh TAG ROUNDS "name:lib:args" ...
#   lib = base (libuwvk.so) or a variant name (libuwvk_<name>.so)
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    n=${spec%%:*}; rest=${spec#*:}; v=${rest%%:*}; args=${rest#*:}
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    f="$OUT/$n-r$r"
    UWVK_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline $args > "$f.json" 2> "$f.err" || { echo "$n failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d.get('timing') or {}; print('$n', 'r$r', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t.get('kernel_ms'))"
  done
done
