#!/bin/bash
# r04: VelocityUKF model pointer laundered per matrix (VEL_LAUNDER_MAT):
# velocity GPU tests on the variant, interleaved C2 A/B, C2 busy-counter pass.
set -o pipefail
O=gpurun_out/lm; mkdir -p $O
V=$PWD/slam-uwv_kalman_filters_amd/libuwvk_lm.so
UWVK_LIB=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "vel or Vel" -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_vel_lm.txt 2>&1 || { tail -20 $O/pytest_vel_lm.txt; exit 1; }
tail -1 $O/pytest_vel_lm.txt
bash tools/ab_c2.sh lm 3 base lm || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
UWVK_LIB=$V timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES \
  --output-format csv -d $O/c2pmc -o run -- python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline \
  > $O/c2pmc.log 2>&1 || { tail -20 $O/c2pmc.log; exit 1; }
find $O/c2pmc -name "*counter_collection*" -exec cp {} $O/c2_pmc_busy_lm.csv \;
echo done
