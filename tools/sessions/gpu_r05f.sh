#!/bin/bash
# r05: the full BodyEfforts update on PSP (k_psp_efforts<DOF, 0, SR>,
# psp_update_eff).  GPU suite first (every efforts test
# now runs the new kernel on the default path), the single-call timings of the
# shipped build (2 waves per SIMD, 0 scratch) and of the 3-waves variant
# (libuwvk_effw3.so, -DEFFWPE=3: 168 VGPRs, 12 B/lane scratch), the C4 full
# cycle under rocprofv3 (the efforts kernel's per-launch time), and two C3
# rounds (the apply_delta refactor must not move the hot kernel).
# Usage (repo root, on the box): bash tools/gpu_r05f.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 tools/time_single_update.py > "$OUT/single_update.txt" 2>&1 || { tail -5 "$OUT/single_update.txt"; exit 1; }
cat "$OUT/single_update.txt"
UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_effw3.so timeout -k 10 300 python3 tools/time_single_update.py > "$OUT/single_update_effw3.txt" 2>&1 || { tail -5 "$OUT/single_update_effw3.txt"; exit 1; }
echo "effw3: $(cat $OUT/single_update_effw3.txt)"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
  python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c4_cycle.json" 2> "$OUT/c4_cycle.err" \
  || { tail -20 "$OUT/c4_cycle.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c4_cycle.json').read().strip().splitlines()[-1]); print('c4', '%.2fM' % (d['value']/1e6))"
cut -c1-200 "$OUT/c4prof/run_kernel_stats.csv"
for rep in 1 2; do
  for s in 20 200; do
    n="c3-s${s}-r${rep}"
    timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing']; print('$n', '%.2fM' % (d['value']/1e6), 'kernel %.3f ms' % t['kernel_ms'])"
  done
done
echo "r05f $TAG done"
