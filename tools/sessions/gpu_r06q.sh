#!/bin/bash
# r06q: the pair kernel's rank-M sweep with its stores under constant lane masks
# (EXEC by scalar instructions; libuwvk.so) against two address selects per entry
# (libuwvk_rm0.so): the pair tests, then an interleaved A/B, three
# rounds, 20 / 200 epochs, and C4's cycle once each.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pd.py tests/test_gpu_tail.py tests/test_gpu_surface.py -q -x --timeout 500 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_pair.txt" 2>&1 || { tail -40 "$OUT/pytest_pair.txt"; exit 1; }
tail -1 "$OUT/pytest_pair.txt"
for r in 1 2 3; do
  for v in mask rm0; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = mask ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], 'nees %.9f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
for v in mask rm0; do
  lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
  [ "$v" = mask ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
  f="$OUT/c4-$v"
  UWVK_LIB=$lib timeout -k 10 600 python3 bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('c4 $v', '%.2fM' % (d['value']/1e6), 'nees %.12f' % d['ensemble']['nees_mean_pos_ori_vel'])"
done
echo "r06q $TAG done"
