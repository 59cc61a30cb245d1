#!/bin/bash
# r06k: the pair tests, then interleaved A/Bs: the pair kernel's per-half
# broadcasts by ds_bpermute (libuwvk.so) against v_readlane + select
# (libuwvk_hrl.so); C2 with the DVL covariance by indexed kernel-argument loads
# (libuwvk.so) against the private copy (libuwvk_velold.so), 2,000 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pd.py tests/test_gpu_tail.py -q -x --timeout 500 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_pair.txt" 2>&1 || { tail -40 "$OUT/pytest_pair.txt"; exit 1; }
tail -2 "$OUT/pytest_pair.txt"
for r in 1 2 3; do
  for v in bp hrl; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = bp ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], d['config']['kernel'][:40], 'nees %.6f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
for r in 1 2 3; do
  for v in velnew velold; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = velnew ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    f="$OUT/c2-$v-r$r"
    UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('c2 $v r$r', '%.2fM' % (d['value']/1e6), d['roofline']['kernel_ms_per_launch'])"
  done
done
echo "r06k $TAG done"
