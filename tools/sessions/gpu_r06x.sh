#!/bin/bash
# r06x: per-unit cost or launch ramp? C3 at 20 / 200 epochs for 5, 10 and 20
# generations of pair units over the 3,072 resident slots (30,720 / 61,440 /
# 122,880 instances), the 20-epoch runs twice.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 30720 61440 122880; do
  for st in 20 20 200; do
    f="$OUT/b$b-s$st-$RANDOM"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 --batch-per-gpu $b > "$f.json" 2> "$f.err" || { echo "failed $f"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('b$b s$st', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'])"
  done
done
echo "r06x $TAG done"
