#!/bin/bash
# r06v: tail spreading of the pair kernel's persistent launch at C3: the
# planner's choice (2 chunks at 20 epochs, 4 at 200) against no spreading
# (--tail-slots -1) and forced 3 / 4 chunks, interleaved, two rounds.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for v in plan off c3 c4; do
    case $v in plan) a="";; off) a="--tail-slots -1";; c3) a="--tail-chunks 3";; c4) a="--tail-chunks 4";; esac
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 $a > "$f.json" 2> "$f.err" || { echo "failed $f"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'])"
    done
  done
done
echo "r06v $TAG done"
