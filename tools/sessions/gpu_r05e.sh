#!/bin/bash
# r05: the C2 32-lane question.  k_vel_epoch_g<32> runs
# every filter twice in a 32-lane group (second row stores nothing): the
# 16-lane kernel's per-wave instruction stream at twice the waves, capped at
# 256 registers for 2 waves per SIMD.  Interleaved A/B against the shipped
# 16-lane kernel (3 rounds), then one counter pass of each (VALU issue and
# wave cycles).  Usage (repo root, on the box): bash tools/gpu_r05e.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for g in 1 2; do
    n="c2g${g}-r${rep}"
    timeout -k 10 200 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline --vel-groups $g > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); t=d['timing'] if 'timing' in d else {}; print('$n', '%.2fM' % (d['value']/1e6), d['config']['kernel'], d['roofline']['kernel_ms_per_launch'])"
  done
done
for g in 1 2; do
  CMD="python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline --vel-groups $g"
  timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g$g/trace" -o run -- $CMD > "$OUT/g$g.trace.json" 2> "$OUT/g$g.trace.err" || { echo "trace g$g failed"; tail -5 "$OUT/g$g.trace.err"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE --output-format csv -d "$OUT/g$g/busy" -o run -- $CMD > "$OUT/g$g.busy.json" 2> "$OUT/g$g.busy.err" || { echo "pmc g$g failed"; tail -5 "$OUT/g$g.busy.err"; exit 1; }
done
echo "r05e $TAG done"
