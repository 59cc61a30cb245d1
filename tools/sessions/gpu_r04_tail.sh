#!/bin/bash
# r04 tail session: phase stamps of the current PSP / efforts kernels and a
# C2 busy-counter pass of the current k_vel_epoch_g.
set -o pipefail
O=gpurun_out/tail; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 240 python3 -u tools/phase_stamps.py > $O/stamps_r04z.txt 2>&1 || exit 1
timeout -k 10 240 python3 -u tools/efforts_stamps.py > $O/eff_stamps_r04z.txt 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES \
  --output-format csv -d $O/c2pmc -o run -- python3 bench.py --mode C2 --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/c2pmc.log 2>&1 || { tail -20 $O/c2pmc.log; exit 1; }
find $O/c2pmc -name "*counter_collection*" -exec cp {} $O/c2_pmc_busy.csv \;
echo done
