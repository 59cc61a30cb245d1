#!/bin/bash
# Counter passes of the C3 bench at one launch shape (one rocprofv3 --pmc run
# per pass: FETCH_SIZE and WRITE_SIZE cannot share one; SQ <= 8, GRBM <= 2),
# plus the kernel-trace --stats summary of the same command and (r03) an f64
# MFMA pass.
# Usage (repo root, on the box): bash tools/pmc_r03.sh TAG STEPS [WARMUP]
set -u
TAG=$1; STEPS=$2; WARM=${3:-5}
OUT=$PWD/gpurun_out/$TAG/s$STEPS
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline ${BENCH_EXTRA:-}"  # BENCH_EXTRA: e.g. --pair
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 1; }
pass() {
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- $CMD > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "pass $1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
}
pass sq_mix "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
pass sq_busy "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE GRBM_COUNT"
pass fetch "FETCH_SIZE"
pass write "WRITE_SIZE"
pass mfma "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
echo "pmc $TAG s$STEPS done"
