#!/bin/bash
# Interleaved A/B of variant libraries on the C2 bench (VelocityUKF, batch 4,096,
# 2,000 epochs).  Variants: names of slam-uwv_kalman_filters_amd/libuwvk_<name>.so,
# "base" = libuwvk.so.  Usage (repo root, on the box): bash tools/ab_c2.sh TAG ROUNDS v1 v2 ...
set -u
TAG=$1; ROUNDS=$2; shift 2
SFX=${C2_SFX:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
vs=("$@")
n=${#vs[@]}
for r in $(seq 1 "$ROUNDS"); do
  for i in $(seq 0 $((n - 1))); do
    v=${vs[$(( (i + r - 1) % n ))]}
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    [ "$v" != base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    UWVK_LIB=$lib timeout -k 10 200 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline ${C2_ARGS:-} \
      > "$OUT/c2${SFX}_${v}_r$r.json" 2> "$OUT/c2${SFX}_${v}_r$r.err" || { echo "$v failed"; tail -5 "$OUT/c2${SFX}_${v}_r$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-8s r%d %7.2f M %8.3f ms' % (sys.argv[2], int(sys.argv[3]), d['value']/1e6, d['ms_per_step']*d['steps']))" \
      "$OUT/c2${SFX}_${v}_r$r.json" "$v" "$r"
  done
done
