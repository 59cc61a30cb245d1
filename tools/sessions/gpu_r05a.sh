#!/bin/bash
# r05 first GPU session: the right SO3 side as the default.  GPU suite (both
# sides parametrised), smoke(), the C3 line on the default (right) side and on
# the left option, the C1 CPU line, the C2 line, and the C4 line over one full
# 30 s / 10 s drop-out cycle (40,000 epochs, segmented log) under rocprofv3
# --kernel-trace --stats (splits k_psp_epoch from k_pose_efforts_epoch).
# Every step has its own time limit; the first failure ends the script.
# Usage (repo root, on the box): bash tools/gpu_r05a.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.4g' % d['value'], d.get('ms_per_step'))" "$1" "$2"; }
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_right_s20_r$r.json" 2> "$OUT/c3_right_s20_r$r.err" || { tail -5 "$OUT/c3_right_s20_r$r.err"; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --so3-left > "$OUT/c3_left_s20_r$r.json" 2> "$OUT/c3_left_s20_r$r.err" || { tail -5 "$OUT/c3_left_s20_r$r.err"; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c3_right_s200_r$r.json" 2> "$OUT/c3_right_s200_r$r.err" || { tail -5 "$OUT/c3_right_s200_r$r.err"; exit 1; }
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline --so3-left > "$OUT/c3_left_s200_r$r.json" 2> "$OUT/c3_left_s200_r$r.err" || { tail -5 "$OUT/c3_left_s200_r$r.err"; exit 1; }
  for f in c3_right_s20 c3_left_s20 c3_right_s200 c3_left_s200; do line "$OUT/${f}_r$r.json" "$f r$r"; done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_cpu.json" 2> "$OUT/c3_cpu.err" || { tail -5 "$OUT/c3_cpu.err"; exit 1; }
line "$OUT/c3_cpu.json" c3_with_cpu_baseline
timeout -k 10 300 python3 bench.py --mode C1 > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -5 "$OUT/c1.err"; exit 1; }
line "$OUT/c1.json" c1
timeout -k 10 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -5 "$OUT/c2.err"; exit 1; }
line "$OUT/c2.json" c2
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
  python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c4_cycle.json" 2> "$OUT/c4_cycle.err" \
  || { tail -20 "$OUT/c4_cycle.err"; exit 1; }
line "$OUT/c4_cycle.json" c4_cycle
cut -c1-200 "$OUT/c4prof/run_kernel_stats.csv"
echo "r05a $TAG done"
