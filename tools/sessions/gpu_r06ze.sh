#!/bin/bash
# r06ze: the pressure update inside the pair kernel (two sigma points per lane,
# libuwvk.so) against r06n's split of the launches around the pressure epochs
# (libuwvk_split.so): the pair / surface / parity tests on the new default,
# then C4's full cycle interleaved, two rounds, and the C3 driver shape.
set -u
TAG=$1
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_pd.py tests/test_gpu_surface.py tests/test_gpu_parity.py tests/test_gpu_tail.py tests/test_golden.py -q -x --timeout 600 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.txt" 2>&1 || { tail -40 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
for r in 1 2; do
  for v in inpair split; do
    lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$v.so
    [ "$v" = inpair ] && lib=$PWD/slam-uwv_kalman_filters_amd/libuwvk.so
    f="$OUT/c4-$v-r$r"
    UWVK_LIB=$lib timeout -k 10 600 python3 bench.py --mode C4 --steps 40000 --warmup 5 --no-cpu-baseline > "$f.json" 2> "$f.err" || { echo "$v failed"; tail -5 "$f.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); print('c4 $v r$r', '%.2fM' % (d['value']/1e6), 'nees %.12f' % d['ensemble']['nees_mean_pos_ori_vel'], d['config']['kernel'][:100])"
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_s20.json" 2> "$OUT/c3_s20.err" || { tail -5 "$OUT/c3_s20.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/c3_s20.json').read().strip().splitlines()[-1]); print('c3 s20', '%.2fM' % (d['value']/1e6))"
echo "r06ze $TAG done"
