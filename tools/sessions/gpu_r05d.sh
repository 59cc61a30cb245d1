#!/bin/bash
# r05: two instances per wavefront (UWVK_OPT_PAIR, k_psp2_epoch; VERDICT r04
# next #3).  Parity first (tests/test_gpu_pair.py), then the interleaved C3 A/B
# at the driver's 20 epochs and at 200: default (tail spreading on), unpaired
# with spreading off, paired (no spreading); 3 rounds.  Then the paired
# kernel's trace + counter passes at 20 / 200 epochs (its VALU per instance-
# epoch against k_psp_epoch's 2417 / 2342 per wave-epoch, r05b), and the
# occupancy sweep (tools/gpu_r05c.sh) that prices the paired kernel's 1.5
# waves per SIMD.  Every step has its own time limit; the first failure ends
# the script.  Usage (repo root, on the box): bash tools/gpu_r05d.sh TAG
# (The pair kernel, --pair and tests/test_gpu_pair.py were removed after this
# session's measurement; commit 582df31 is the tree it ran on.)
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pair.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_pair.txt" 2>&1 || { tail -40 "$OUT/pytest_pair.txt"; exit 1; }
tail -3 "$OUT/pytest_pair.txt"
for rep in 1 2 3; do
  for s in 20 200; do
    for arm in def off pair; do
      case $arm in
        def) X="--tail-slots 0" ;;
        off) X="--tail-slots -1" ;;
        pair) X="--pair" ;;
      esac
      n="${arm}-s${s}-r${rep}"
      timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline $X > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'], d['config']['kernel'])"
    done
  done
done
BENCH_EXTRA=--pair bash tools/pmc_r03.sh "$TAG" 20 || exit 1
BENCH_EXTRA=--pair bash tools/pmc_r03.sh "$TAG" 200 || exit 1
BENCH_EXTRA=--pair bash tools/pmc_lds.sh "$TAG" 200 || exit 1
bash tools/gpu_r05c.sh "$TAG-occ" || exit 1
echo "r05d $TAG done"
