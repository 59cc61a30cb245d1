#!/bin/bash
# r06f: counter passes of the parameter-decoupled kernel at the driver's 20-epoch
# launch and at 200 (VALU mix, busy, FETCH/WRITE, f64 MFMA, LDS), each pass its
# own rocprofv3 run under its own time limit.
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_r03.sh $TAG 20 5 || exit 1
bash tools/pmc_lds.sh $TAG 20 5 || exit 1
bash tools/pmc_r03.sh $TAG 200 5 || exit 1
echo "r06f $TAG done"
