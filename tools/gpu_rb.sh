#!/bin/bash
# r04: VelocityUKF row broadcast by DPP row_newbcast (VEL_ROW_DPP):
# velocity GPU tests on the variant, interleaved C2 A/B, C2 busy-counter pass.
set -o pipefail
O=gpurun_out/rb; mkdir -p $O
V=$PWD/slam-uwv_kalman_filters_amd/libuwvk_rb.so
UWVK_LIB=$V timeout -k 10 600 python3 -u -m pytest tests -m gpu -k "vel or Vel" -x -v --timeout 120 --timeout-method thread \
  > $O/pytest_vel_rb.txt 2>&1 || { tail -20 $O/pytest_vel_rb.txt; exit 1; }
tail -1 $O/pytest_vel_rb.txt
bash tools/ab_c2.sh rb 3 base rb || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
UWVK_LIB=$V timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES \
  --output-format csv -d $O/c2pmc -o run -- python3 bench.py --mode C2 --steps 2000 --warmup 5 --no-cpu-baseline \
  > $O/c2pmc.log 2>&1 || { tail -20 $O/c2pmc.log; exit 1; }
find $O/c2pmc -name "*counter_collection*" -exec cp {} $O/c2_pmc_busy_rb.csv \;
echo done
