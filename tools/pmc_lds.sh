#!/bin/bash
# LDS counter passes of the C3 bench at one launch shape (VERDICT r03 next #3:
# measure the LDS side before fusing the Sigma~ sweeps).  One rocprofv3 --pmc
# run per pass, each under its own time limit; the available-counter listing
# first, so that a name this ROCm does not know shows up in the log.
# Usage (repo root, on the box): bash tools/pmc_lds.sh TAG STEPS [WARMUP]
set -u
TAG=$1; STEPS=$2; WARM=${3:-5}
OUT=$PWD/gpurun_out/$TAG/s$STEPS
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
CMD="python3 bench.py --steps $STEPS --warmup $WARM --no-cpu-baseline ${BENCH_EXTRA:-}"  # BENCH_EXTRA: e.g. --pair
pass() {
  timeout -s KILL 150 rocprofv3 --pmc $2 --output-format csv -d "$OUT/$1" -o run -- $CMD > "$OUT/$1.json" 2> "$OUT/$1.err" || { echo "pass $1 failed"; tail -5 "$OUT/$1.err"; exit 1; }
}
pass lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
pass lds2 "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES"
echo "pmc lds $TAG s$STEPS done"
