#!/bin/bash
# r05: occupancy sweep of the C3 epoch kernel (UWVK_OPT_LDS_PAD): unused dynamic
# LDS per workgroup lowers the resident instances per CU from 12 (3 waves per
# SIMD) to 11 / 10 / 9 / 8 / 6 (1.5 per SIMD) / 4 (1 per SIMD); tail spreading off
# in every arm.  200-epoch launches, 2 interleaved rounds.  This prices the
# occupancy that two instances per wave would give up.
# Usage (repo root, on the box): bash tools/gpu_r05c.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for rep in 1 2; do
  for pad in 0 2000 3500 5300 7600 14400 28000; do
    n="pad${pad}-r${rep}"
    timeout -k 10 200 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --tail-slots -1 --lds-pad $pad \
      > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
  done
done
echo "r05c $TAG done"
