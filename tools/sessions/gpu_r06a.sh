#!/bin/bash
# r06a: first session of round 6 — GPU suite + smoke on the round's starting tree,
# the driver-shaped C3 line, then two interleaved A/Bs:
#   (1) 26-DOF k_psp_epoch at 4 waves/SIMD (libuwvk_w4.so, amdgpu_waves_per_eu(4,4))
#       against the shipped 3-wave build;
#   (2) the persistent scheduler (--persist 1) against static tail spreading on the
#       53-DOF headline kernel.
# Every step has its own time limit; the first failure ends the script.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
tail -1 "$OUT/c3_s20.json" | cut -c1-300
bash tools/ab_lib_args.sh $TAG/w4_s200 3 "--dof 26 --steps 200 --warmup 5" base w4 || exit 1
bash tools/ab_lib_args.sh $TAG/w4_s20 3 "--dof 26 --steps 20 --warmup 5" base w4 || exit 1
bash tools/ab_args.sh $TAG/persist 4 "static20:--steps 20 --warmup 5 --persist 0" "persist20:--steps 20 --warmup 5 --persist 1" \
  "static200:--steps 200 --warmup 5 --persist 0" "persist200:--steps 200 --warmup 5 --persist 1" || exit 1
echo "r06a $TAG done"
