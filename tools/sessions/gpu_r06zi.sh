#!/bin/bash
# r06zi: the closing check of the final r06 tree as the driver runs it: the GPU
# suite, smoke(), the default bench line (driver shape, with its CPU baseline),
# and the N-rank path rehearsed on one GPU (UWVK_BENCH_SAME_DEVICE: every rank
# on device 0, statistics summed over gloo) at N = 2 and 4 through
# torch.distributed.run, as the driver launches the scaling runs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
line() { python3 -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); t=d.get('timing',{}); print('$2', '%.2fM' % (d['value']/1e6), 'n_gpus', d['n_gpus'], 'kernel_ms', t.get('kernel_ms'), 'kernel', d['config'].get('kernel'), 'coll', d['config'].get('collective'), 'check', d.get('collective_check'), 'nees', (d.get('ensemble') or {}).get('nees_mean_pos_ori_vel'))"; }
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -20 "$OUT/smoke.txt"; exit 1; }
tail -1 "$OUT/smoke.txt"
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
line "$OUT/bench.json" bench_default
for n in 2 4; do
  UWVK_BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus $n --steps 20 --warmup 5 > "$OUT/same_n$n.json" 2> "$OUT/same_n$n.err" || { tail -20 "$OUT/same_n$n.err"; exit 1; }
  line "$OUT/same_n$n.json" same_n$n
done
echo "r06zi $TAG done"
