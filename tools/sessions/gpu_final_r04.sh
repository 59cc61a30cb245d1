#!/bin/bash
# r04 closing session on one MI355X: GPU suite, smoke(), the default C3 bench
# line (with the CPU baseline), counter passes of the current kernel at the
# driver's 20 epochs and at 200 (tools/pmc_r03.sh, pmc_lds.sh: kernel trace +
# stats, VALU / fp64 mix, busy, HBM traffic, MFMA, LDS), and the C4 / C5-shard /
# C2 lines.  Every step has its own time limit; the first failure ends it.
# Usage (repo root, on the box): bash tools/gpu_final_r04.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || { tail -5 "$OUT/bench_c3.err"; exit 1; }
tail -c 400 "$OUT/bench_c3.json"; echo
if [ -z "${SKIP_PMC:-}" ]; then  # SKIP_PMC=1: the PSP kernel unchanged since the last counter passes
  bash tools/pmc_r03.sh "$TAG" 20 || exit 1
  bash tools/pmc_r03.sh "$TAG" 200 || exit 1
  bash tools/pmc_lds.sh "$TAG" 20 || exit 1
  bash tools/pmc_lds.sh "$TAG" 200 || exit 1
fi
timeout -k 10 300 python3 bench.py --mode C4 --steps 2000 --warmup 5 --no-cpu-baseline > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -5 "$OUT/c4.err"; exit 1; }
timeout -k 10 300 python3 bench.py --mode C5 --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c5shard.json" 2> "$OUT/c5shard.err" || { tail -5 "$OUT/c5shard.err"; exit 1; }
timeout -k 10 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -5 "$OUT/c2.err"; exit 1; }
for f in c4 c5shard c2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.2f M' % (d['value']/1e6))" "$OUT/$f.json" $f; done
echo "final $TAG done"
