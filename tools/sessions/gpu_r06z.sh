#!/bin/bash
# r06z: the closing-measurement session on the final r06 tree (pair kernel with
# the DPP broadcasts and masked rank-M stores, no tail spreading of pair launches;
# 26-DOF handles paired too): counter
# passes of the timed launch at 20 and 200 epochs first, then:
# GPU suite, smoke, the driver-shaped C3 line with its CPU
# baseline and rocprofv3 trace/stats, 200-epoch lines, the left SO3 side,
# n = 26, the C5 shard, C2, the C4 full cycle under rocprofv3, and C3 over
# 40,000 epochs (the ensemble NEES of a long window).  Every step has its own
# time limit; the first failure ends the script.
# Usage (repo root, on the box): bash tools/sessions/gpu_r06z.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_r03.sh $TAG 20 5 || exit 1
bash tools/pmc_lds.sh $TAG 20 5 || exit 1
bash tools/pmc_r03.sh $TAG 200 5 || exit 1
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'kernel_ms', t.get('kernel_ms'), 'frac', (d.get('roofline') or {}).get('frac'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'))"; }
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_traced.json" 2> "$OUT/c3_s20_traced.err" || { tail -5 "$OUT/c3_s20_traced.err"; exit 1; }
line "$OUT/c3_s20_traced.json" c3_s20_traced
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c3_s200_r$r.json" 2> "$OUT/c3_s200_r$r.err" || { tail -5 "$OUT/c3_s200_r$r.err"; exit 1; }
  line "$OUT/c3_s200_r$r.json" c3_s200_r$r
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --so3-left > "$OUT/c3_left_s20.json" 2> "$OUT/c3_left.err" || { tail -5 "$OUT/c3_left.err"; exit 1; }
line "$OUT/c3_left_s20.json" c3_left_s20
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --dof 26 > "$OUT/c3_dof26_s20.json" 2> "$OUT/c3_dof26.err" || { tail -5 "$OUT/c3_dof26.err"; exit 1; }
line "$OUT/c3_dof26_s20.json" c3_dof26_s20
timeout -k 10 300 python3 bench.py --mode C5 --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c5_shard.json" 2> "$OUT/c5.err" || { tail -5 "$OUT/c5.err"; exit 1; }
line "$OUT/c5_shard.json" c5_shard
timeout -k 10 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 > "$OUT/c2.json" 2> "$OUT/c2.err" || { tail -5 "$OUT/c2.err"; exit 1; }
line "$OUT/c2.json" c2
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
  python3 -u bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c4_cycle.json" 2> "$OUT/c4_cycle.err" \
  || { tail -20 "$OUT/c4_cycle.err"; exit 1; }
line "$OUT/c4_cycle.json" c4_cycle
cut -c1-160 "$OUT/c4prof/run_kernel_stats.csv" | head -5
timeout -k 10 400 python3 -u bench.py --mode C3 --steps 40000 --warmup 5 --no-cpu-baseline > "$OUT/c3_e40000.json" 2> "$OUT/c3_e40000.err" \
  || { tail -20 "$OUT/c3_e40000.err"; exit 1; }
line "$OUT/c3_e40000.json" c3_e40000
echo "r06z $TAG done"
