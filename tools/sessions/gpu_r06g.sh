#!/bin/bash
# r06g: the two-instances-per-wave PD kernel (UWVK_OPT_PAIR): its tests, then an
# interleaved A/B of the pair kernel at 4 / 3 / 2 waves per SIMD (libuwvk.so,
# libuwvk_pw3.so, libuwvk_pw2.so) against the one-instance PD kernel (--pair 0).
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_pd.py -v -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_pd.txt" 2>&1 || { tail -60 "$OUT/pytest_pd.txt"; exit 1; }
tail -3 "$OUT/pytest_pd.txt"
for r in 1 2; do
  for v in single base pw3 pw2; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so; args="--pair 1"
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    [ "$v" = single ] && { lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so; args="--pair 0"; }
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 $args > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], d['config']['kernel'][:40], 'nees %.3f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
echo "r06g $TAG done"
