#!/bin/bash
# r05 second GPU session: GPU suite (constrainVelocity on PSP), single-update
# timings, counter passes of the default (right-side) C3 kernel at the driver's
# 20 epochs and at 200 (tools/pmc_r03.sh, pmc_lds.sh), and the interleaved tail
# spreading A/B: --tail-slots -1 (off) against 0 (on), 20
# and 200 epochs, 3 rounds.  Every step has its own time limit; the first
# failure ends the script.  Usage (repo root, on the box): bash tools/gpu_r05b.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 tools/time_single_update.py > "$OUT/single_update.txt" 2>&1 || { tail -5 "$OUT/single_update.txt"; exit 1; }
cat "$OUT/single_update.txt"
for rep in 1 2 3; do
  for s in 20 200; do
    for t in -1 0; do
      n="t${t}-s${s}-r${rep}"
      timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline --tail-slots $t > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
    done
  done
done
bash tools/pmc_r03.sh "$TAG" 20 || exit 1
bash tools/pmc_r03.sh "$TAG" 200 || exit 1
bash tools/pmc_lds.sh "$TAG" 20 || exit 1
bash tools/pmc_lds.sh "$TAG" 200 || exit 1
echo "r05b $TAG done"
