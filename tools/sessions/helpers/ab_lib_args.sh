#!/bin/bash
# Interleaved A/B of whole-library builds (libuwvk_<v>.so; base = libuwvk.so)
# on one bench.py argument set.
# Usage (repo root, on the box): bash tools/ab_lib_args.sh TAG ROUNDS "ARGS" base v1 ...
set -u
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    f="$OUT/$v-r$r"
    UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline $ARGS > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v', 'r$r', '%.2fM' % (d['value']/1e6), 'ms_per_step %.5f' % d['ms_per_step'])"
  done
done
