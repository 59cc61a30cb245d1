#!/bin/bash
# r06u: where the 20-epoch launch's fixed ~0.5 ms goes: C3 at 20 and 200 epochs
# for batches that fill the pair kernel's 3,072 resident slots with 10 / 10.67 /
# 11 generations of pair units (61,440 / 65,536 / 67,584), and 65,536 without
# tail spreading (--tail-slots -1).
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in "61440 0" "65536 0" "67584 0" "65536 -1"; do
  set -- $cfg
  for st in 20 200; do
    f="$OUT/b$1-t$2-s$st"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 --batch-per-gpu $1 --tail-slots $2 > "$f.json" 2> "$f.err" || { echo "failed $f"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('b$1 t$2 s$st', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'])"
  done
done
echo "r06u $TAG done"
