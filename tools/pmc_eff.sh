#!/bin/bash
# Counter passes of the C4 bench with a compressed drop-out cycle (7 BodyEfforts
# epochs in 2,000), for the literal k_pose_efforts_epoch (tools/pmc_eff_fold.py
# extracts its dispatches).  One rocprofv3 --pmc run per pass.
# Usage (repo root, on the box): bash tools/pmc_eff.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG/eff
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 bench.py --mode C4 --steps 2000 --warmup 5 --c4-cycle 0.3,0.1 --no-cpu-baseline"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $CMD > "$OUT/trace.json" 2> "$OUT/trace.err" || { tail -5 "$OUT/trace.err"; exit 1; }
pass() {
  timeout -s KILL 200 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- $CMD > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "pass $1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
}
pass sq_mix "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"
pass sq_busy "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 GRBM_GUI_ACTIVE GRBM_COUNT"
pass mfma "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
pass lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
echo "pmc eff $TAG done"
