#!/bin/bash
# r06zf: the pair kernel's H Gl products with Gl staged through LDS and read as
# broadcasts (libuwvk_gl.so) against the per-(t, j) half-wave broadcasts
# (libuwvk.so): the pair / surface / parity tests on the variant, then an
# interleaved A/B, three rounds, 20 / 200 epochs.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_gl.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_pd.py tests/test_gpu_surface.py tests/test_gpu_parity.py -q -x --timeout 500 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gl.txt" 2>&1 || { tail -40 "$OUT/pytest_gl.txt"; exit 1; }
tail -1 "$OUT/pytest_gl.txt"
for r in 1 2 3; do
  for v in base gl; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = base ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    for st in 20 200; do
      f="$OUT/$v-s$st-r$r"
      UWVK_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps $st --warmup 5 > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('$v s$st r$r', '%.2fM' % (d['value']/1e6), d['timing']['kernel_ms'], 'nees %.9f' % d['ensemble']['nees_mean_pos_ori_vel'])"
    done
  done
done
echo "r06zf $TAG done"
