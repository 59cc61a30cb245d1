#!/bin/bash
# r04d: fp64 rsq/rcp accuracy probe, phase stamps of the C3 kernel, the GPU
# suite, and an interleaved C2 A/B (libuwvk.so vs the variants given).
# Usage (repo root, on the box): bash tools/gpu_r04d.sh TAG v1 v2 ...
set -u
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./tools/probe_rsq > "$OUT/probe_rsq.txt" 2>&1 || { cat "$OUT/probe_rsq.txt"; exit 1; }
cat "$OUT/probe_rsq.txt"
timeout -k 10 200 python3 tools/phase_stamps.py > "$OUT/stamps.txt" 2>&1 || { tail -5 "$OUT/stamps.txt"; exit 1; }
cat "$OUT/stamps.txt"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.txt" 2>&1 || { tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for r in 1 2 3; do
  for v in base "$@"; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    [ "$v" != base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    UWVK_LIB=$lib timeout -k 10 200 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline \
      > "$OUT/c2_${v}_r$r.json" 2> "$OUT/c2_${v}_r$r.err" || { tail -5 "$OUT/c2_${v}_r$r.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], '%.1f M' % (d['value']/1e6), '%.3f ms' % d['roofline']['kernel_ms_per_launch'])" "$OUT/c2_${v}_r$r.json" "$v" "$r"
  done
done
