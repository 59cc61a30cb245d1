#!/bin/bash
# r05i: where the C4 full-cycle ensemble NEES (125) comes from — the same
# 40,000-epoch window without drop-outs (C4, cycle 100 s / 0 s) and as C3, and
# C3's NEES at 2,000 and 10,000 epochs.  Ran on the r05 final tree.
set -u
O=gpurun_out/r05i
mkdir -p $O
run() {  # LABEL ARGS...
  local lab=$1; shift
  timeout -k 10 400 python3 -u bench.py --no-cpu-baseline "$@" > $O/$lab.json 2> $O/$lab.err || { tail -20 $O/$lab.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f M' % (d['value']/1e6), d['ensemble'])" $O/$lab.json $lab
}
run c4_nodrop --mode C4 --steps 40000 --c4-cycle 100,0
run c3_e40000 --mode C3 --steps 40000
run c3_e10000 --mode C3 --steps 10000
run c3_e2000 --mode C3 --steps 2000
