#!/bin/bash
# Counter passes of the C2 bench (VelocityUKF, batch 4,096, k_vel_epoch_g):
# how busy the VALU is at one wave per SIMD (is the
# lane-group kernel latency-bound?), plus the kernel-trace summary.
# Usage (repo root, on the box): bash tools/pmc_c2.sh TAG [STEPS]
set -u
TAG=$1; STEPS=${2:-2000}
OUT=$PWD/gpurun_out/$TAG/c2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --mode C2 --steps $STEPS --warmup 5 --no-cpu-baseline"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 1; }
pass() {
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- $CMD > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "pass $1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
}
pass busy "SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
pass wait "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
echo "pmc c2 $TAG done"
