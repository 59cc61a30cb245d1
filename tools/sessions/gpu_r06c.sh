#!/bin/bash
# r06c: the parameter-decoupled epoch kernel (UWVK_OPT_PARAM_BLOCK): its bitwise
# tests first, then the GPU suite, smoke, and an interleaved A/B of the kernel
# against the general 53-DOF one (--param-block 0) at 20 and 200 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pd.py -v -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_pd.txt" 2>&1 || { tail -60 "$OUT/pytest_pd.txt"; exit 1; }
tail -3 "$OUT/pytest_pd.txt"
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
bash tools/ab_args.sh $TAG/pd 3 "pd20:--steps 20 --warmup 5" "gen20:--steps 20 --warmup 5 --param-block 0" \
  "pd200:--steps 200 --warmup 5" "gen200:--steps 200 --warmup 5 --param-block 0" || exit 1
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3_s20.json').read().strip().splitlines()[-1]); print('c3_s20', d['value']/1e6, d['timing'], d['roofline']['kernel'], d['roofline']['frac'])"
echo "r06c $TAG done"
