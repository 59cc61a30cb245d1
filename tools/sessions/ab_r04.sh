#!/bin/bash
# r04 interleaved A/B of variant libraries on the C3 bench, both launch shapes
# (the driver's 20 epochs and 200), ROUNDS rounds in rotating order so that
# box drift does not favour one variant.  Variants: names of
# slam-uwv_kalman_filters_amd/libuwvk_<name>.so, "base" = libuwvk.so.
# Usage (repo root, on the box): bash tools/ab_r04.sh TAG ROUNDS v1 v2 ...
set -u
TAG=$1; ROUNDS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
vs=("$@")
n=${#vs[@]}
for r in $(seq 1 "$ROUNDS"); do
  for i in $(seq 0 $((n - 1))); do
    v=${vs[$(( (i + r - 1) % n ))]}
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    [ "$v" != base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    for s in 20 200; do
      UWVK_LIB=$lib timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline \
        > "$OUT/${v}_s${s}_r$r.json" 2> "$OUT/${v}_s${s}_r$r.err" || { echo "$v failed"; tail -5 "$OUT/${v}_s${s}_r$r.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('%-10s s%-3d r%d %7.2f M %8.3f ms' % (sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), d['value']/1e6, d['timing']['kernel_ms']))" \
        "$OUT/${v}_s${s}_r$r.json" "$v" "$s" "$r"
    done
  done
done
