#!/bin/bash
# r06i: the GPU suite on the pair-default tree (fused rank-M + apply_delta in
# the pair kernel), one C3 line under rocprofv3, then an interleaved A/B of the
# fusion (libuwvk.so) against the unfused pair kernel (libuwvk_nofuse.so).
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -q -m gpu -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.txt" 2>&1 || { tail -40 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" \
  || { tail -30 "$OUT/bench_prof.err"; exit 1; }
cut -c1-300 "$OUT/bench_prof.json"
for r in 1 2 3; do
  for v in fuse nofuse; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = fuse ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], d['config']['kernel'][:40], 'nees %.3f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
echo "r06i $TAG done"
