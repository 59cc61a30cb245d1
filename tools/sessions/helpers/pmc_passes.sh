#!/bin/bash
# SQ counter passes over the C3 bench (one rocprofv3 --pmc run per pass; summaries with tools/rocpd_summary.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
run() {
  timeout -s KILL 150 rocprofv3 --pmc $2 -d gpurun_out/pmc/$1 -o $1 -- python3 bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/pmc/$1.json 2> gpurun_out/pmc/$1.err
}
run A "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS"
run B "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
run C "SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
