#!/bin/bash
# r05 checkpoint: the GPU suite (with tests/test_gpu_efforts.py), smoke(), the
# driver-shaped bench line with the CPU baseline, and its rocprofv3 kernel
# trace + stats.  Usage (repo root, on the box): bash tools/gpu_r05g.sh TAG
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -2 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print('bench', '%.2fM' % (d['value']/1e6), 'frac', d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_traced.json" 2> "$OUT/bench_traced.err" || { tail -5 "$OUT/bench_traced.err"; exit 1; }
cut -c1-160 "$OUT/trace/run_kernel_stats.csv" | head -5
echo "r05g $TAG done"
