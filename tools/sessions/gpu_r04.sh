#!/bin/bash
# r04 GPU session: the right-side parity tests first, then the whole GPU suite,
# smoke, and same-box A/B lines of the driver's bench shape (C3, 20 epochs):
# left and right SO3 side, interleaved.  Every GPU step under its own limit;
# the first failure ends the script.
# Usage (repo root, on the box): bash tools/gpu_r04.sh TAG [ROUNDS]
set -u
TAG=${1:-r04}; ROUNDS=${2:-2}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_so3_right.py -v -m gpu -x --timeout 200 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_right.txt" 2>&1 || { tail -40 "$OUT/pytest_right.txt"; exit 1; }
tail -1 "$OUT/pytest_right.txt"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.txt" 2>&1 \
  || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
for r in $(seq 1 "$ROUNDS"); do
  for side in left right; do
    extra=""; [ "$side" = right ] && extra="--so3-right"
    for s in 20 200; do
      timeout -k 10 200 python3 bench.py --steps $s --warmup 5 --no-cpu-baseline $extra > "$OUT/b_${side}_s${s}_r$r.json" \
        2> "$OUT/b_${side}_s${s}_r$r.err" || { tail -20 "$OUT/b_${side}_s${s}_r$r.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'M', d['roofline']['kernel'], round(d['timing']['kernel_ms'],3), 'ms')" "$OUT/b_${side}_s${s}_r$r.json"
    done
  done
done
