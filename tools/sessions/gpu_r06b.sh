#!/bin/bash
# r06b: the tree after the ABI-3 changes (persistent scheduler default, host-mapped
# hand-off fault word, reference call-form facade): GPU suite (incl.
# test_reference_call_forms_match_oracle, test_headline_shape_sampled,
# test_handoff_timeout_is_an_error), smoke, the driver-shaped C3 line, the
# 200-epoch line, and the 20-epoch line under rocprofv3 (kernel trace / stats).
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), t, 'frac', (d.get('roofline') or {}).get('frac'))"; }
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
line "$OUT/c3_s20.json" c3_s20
timeout -k 10 300 python3 bench.py --steps 200 --warmup 5 --no-cpu-baseline > "$OUT/c3_s200.json" 2> "$OUT/c3_s200.err" || { tail -5 "$OUT/c3_s200.err"; exit 1; }
line "$OUT/c3_s200.json" c3_s200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_s20" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20_traced.json" 2> "$OUT/c3_s20_traced.err" || { tail -5 "$OUT/c3_s20_traced.err"; exit 1; }
line "$OUT/c3_s20_traced.json" c3_s20_traced
echo "r06b $TAG done"
