#!/bin/bash
# One GPU-box session: parity tests, bench line, rocprofv3 kernel stats and
# the two HBM PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Usage (from the repo root, on the box): bash tools/gpu_round.sh TAG [STEPS_PROF]
set -u
TAG=${1:-run}
SP=${2:-20}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { cat "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --dense --no-cpu-baseline --steps 50 > "$OUT/bench_dense.json" 2>> "$OUT/bench.err" || { cat "$OUT/bench.err"; exit 1; }
cat "$OUT/bench_dense.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps $SP --warmup 2 --no-cpu-baseline > "$OUT/prof.log" 2>&1 || { tail -30 "$OUT/prof.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps $SP --warmup 2 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1 || { tail -30 "$OUT/pmc_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps $SP --warmup 2 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1 || { tail -30 "$OUT/pmc_write.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 SQ_WAVES --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py --steps $SP --warmup 2 --no-cpu-baseline > "$OUT/pmc_sq.log" 2>&1 || { tail -30 "$OUT/pmc_sq.log"; exit 1; }
find "$OUT" -name "*.csv" | head -20
