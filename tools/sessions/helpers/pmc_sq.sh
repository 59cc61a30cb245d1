#!/bin/bash
# SQ instruction-mix / stall counters of the PSP epoch kernel (one --pmc pass each).
set -u
OUT=$PWD/gpurun_out/pmc_sq
mkdir -p "$OUT"
export TMPDIR=/tmp
LIBV=${1:-}
[ -n "$LIBV" ] && export UWVK_LIB=$PWD/slam-uwv_kalman_filters_amd/libuwvk_$LIBV.so
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$OUT/p1" -o run -- python3 bench.py --steps 50 --warmup 2 --no-cpu-baseline > "$OUT/p1.log" 2>&1 || { tail -20 "$OUT/p1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD --output-format csv -d "$OUT/p2" -o run -- python3 bench.py --steps 50 --warmup 2 --no-cpu-baseline > "$OUT/p2.log" 2>&1 || { tail -20 "$OUT/p2.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, sys, glob
out = sys.argv[1]
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    best = {}
    for r in rows:
        if "psp_epoch" not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Counter_Name"])
        best[key] = float(r["Counter_Value"])
    # largest dispatch (the timed one)
    disp = {}
    for (d, c), v in best.items():
        disp.setdefault(d, {})[c] = v
    d = max(disp, key=lambda k: max(disp[k].values()))
    for c, v in sorted(disp[d].items()):
        print("%-24s %16.4g" % (c, v))
PY
