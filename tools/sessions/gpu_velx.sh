#!/bin/bash
# r04: VelocityUKF lane-group kernel against lane-per-filter across batch sizes
# (the automatic choice switches at kVelGroupsMaxBatch).
set -o pipefail
O=gpurun_out/velx; mkdir -p $O
for B in 8192 16384 32768 65536; do
  for g in 0 1; do
    timeout -k 10 200 python3 bench.py --mode C2 --batch $B --vel-groups $g --steps 2000 --warmup 5 --no-cpu-baseline \
      > $O/c2_b${B}_g$g.json 2> $O/c2_b${B}_g$g.err || { tail -5 $O/c2_b${B}_g$g.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], '%.1f M' % (d['value']/1e6))" $O/c2_b${B}_g$g.json $B $g
  done
done
