#!/bin/bash
# Interleaved C3 A/B of libuwvk variants (UWVK_LIB) against the shipped build:
# ROUNDS rounds x {20, 200} epochs x {base, variants...}.
# Usage (repo root, on the box): bash tools/ab_variants.sh TAG ROUNDS V1 [V2 ...]
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
PKGD=$PWD/slam-uwv_kalman_filters_amd
for rep in $(seq 1 $ROUNDS); do
  for s in 20 200; do
    for v in base "$@"; do
      n="${v}-s${s}-r${rep}"
      if [ "$v" = base ]; then LIBV=$PKGD/libuwvk.so; else LIBV=$PKGD/libuwvk_$v.so; fi
      UWVK_LIB=$LIBV timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
    done
  done
done
echo "ab $TAG done"
