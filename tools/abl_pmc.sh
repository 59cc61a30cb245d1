#!/bin/bash
# Dynamic instruction budget per phase of k_psp_epoch<53>: one rocprofv3 --pmc
# pass per ablation build (libuwvk_a<N>.so from `make variant V=a<N>
# VFLAGS=-DPSP_ABL=<N>`; results of an ablated build are invalid, only its
# counters and time are used).  The difference to base is the phase's count.
# r04: the fp64 mix (FMA / MUL / ADD / TRANS) as well, 20-epoch launches (the
# driver's shape), into gpurun_out/TAG/.
# usage (on the GPU box, repo root): bash tools/abl_pmc.sh TAG base a1 a2 ...
set -u
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=slam-uwv_kalman_filters_amd/libuwvk.so; else lib=slam-uwv_kalman_filters_amd/libuwvk_$v.so; fi
  UWVK_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 \
    SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv \
    -d "$OUT/$v" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" \
    || { echo "$v failed"; tail -5 "$OUT/$v.err"; exit 1; }
  echo "$v done"
done
