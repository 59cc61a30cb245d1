#!/bin/bash
# r04: the automatic lane-group choice at batch 28,672 (inside the moved threshold)
set -o pipefail
O=gpurun_out/velx2; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests -m gpu -k "vel or Vel" -x -q --timeout 120 --timeout-method thread > $O/pytest_vel.txt 2>&1 || { tail -20 $O/pytest_vel.txt; exit 1; }
tail -1 $O/pytest_vel.txt
for g in -1 0; do
  timeout -k 10 200 python3 bench.py --mode C2 --batch 28672 --vel-groups $g --steps 2000 --warmup 5 --no-cpu-baseline \
    > $O/c2_b28672_g$g.json 2> $O/c2_g$g.err || { tail -5 $O/c2_g$g.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f M' % (d['value']/1e6), d['roofline'].get('kernel', ''))" $O/c2_b28672_g$g.json $g
done
