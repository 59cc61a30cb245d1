#!/bin/bash
# r06l: the GPU suite on the round's kernel (pair default, no fusion), counter
# passes of the pair kernel at 20 and 200 epochs (VALU mix, busy, FETCH/WRITE,
# MFMA, LDS), then an interleaved C2 A/B: the low-rate sensor arguments staged
# in LDS (libuwvk.so, 0 B/lane scratch) against the r05 private copy
# (libuwvk_velold.so), 2,000 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
bash tools/pmc_r03.sh $TAG 20 5 || exit 1
bash tools/pmc_lds.sh $TAG 20 5 || exit 1
bash tools/pmc_r03.sh $TAG 200 5 || exit 1
for r in 1 2 3; do
  for v in velnew velold; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = velnew ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    f="$OUT/c2-$v-r$r"
    UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('c2 $v r$r', '%.2fM' % (d['value']/1e6), d['roofline']['kernel_ms_per_launch'])"
  done
done
echo "r06l $TAG done"
