#!/usr/bin/env python3
"""Fold tools/pmc_eff.sh passes: per-dispatch counters of k_pose_efforts_epoch
(the literal BodyEfforts update, 65,536 instances per dispatch) averaged over
its dispatches, normalised per instance-update, into
profiles/pmc_traffic.json["C4-efforts-dof53-b65536"], and the summaries copied
to profiles/ROUND_DIR/.

usage: tools/pmc_eff_fold.py TAG [ROUND_DIR (default r04)]"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rdir = sys.argv[2] if len(sys.argv) > 2 else "r04"
base = os.path.join(ROOT, "gpurun_out", tag, "eff")
KERNEL = "k_pose_efforts_epoch<53"
N_SIMD, B = 1024, 65536


def passc(name):
    rows = [r for r in csv.DictReader(open(os.path.join(base, name, "run_counter_collection.csv")))
            if KERNEL in r["Kernel_Name"]]
    per = {}
    for r in rows:
        d = per.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    n = len(per)
    avg = {}
    for d in per.values():
        for k, v in d.items():
            avg[k] = avg.get(k, 0.0) + v / n
    return avg, n, rows


mix, n1, r1 = passc("sq_mix")
busy, n2, r2 = passc("sq_busy")
mfma, n3, r3 = passc("mfma")
lds, n4, r4 = passc("lds")
stats = [r for r in csv.DictReader(open(os.path.join(base, "trace", "run_kernel_stats.csv"))) if KERNEL in r["Name"]]
avg_ms = float(stats[0]["AverageNs"]) / 1e6
xcd = busy["GRBM_GUI_ACTIVE"] / 8.0
f64 = mix["SQ_INSTS_VALU_FMA_F64"] + mix["SQ_INSTS_VALU_MUL_F64"] + mix["SQ_INSTS_VALU_ADD_F64"] + mix["SQ_INSTS_VALU_TRANS_F64"]
e = {
    "kernel": "k_pose_efforts_epoch<53, 0, 0>", "dispatches": n1, "instances_per_dispatch": B,
    "avg_ms": avg_ms,
    "per_instance_update": {k.replace("SQ_INSTS_", "").lower(): v / B for k, v in mix.items() if k.startswith("SQ_INSTS_")},
    "waves_per_dispatch": mix["SQ_WAVES"],
    "issued_fp64_lane_flops_per_instance": 64 * (2 * mix["SQ_INSTS_VALU_FMA_F64"] + mix["SQ_INSTS_VALU_MUL_F64"]
                                                 + mix["SQ_INSTS_VALU_ADD_F64"]) / B
                                            + mfma["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512.0 / B,
    "frac_issued_fp64": (64 * (2 * mix["SQ_INSTS_VALU_FMA_F64"] + mix["SQ_INSTS_VALU_MUL_F64"] + mix["SQ_INSTS_VALU_ADD_F64"])
                         + mfma["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512.0) / (avg_ms * 1e-3) / 78.6e12,
    "valu_busy": busy["SQ_ACTIVE_INST_VALU"] * 4.0 / (N_SIMD * xcd),
    "valu_busy_model": (4.0 * f64 + 2.0 * (mix["SQ_INSTS_VALU"] - f64)) / (N_SIMD * xcd),
    "mfma_busy": mfma["SQ_VALU_MFMA_BUSY_CYCLES"] / mfma["SQ_BUSY_CU_CYCLES"],
    "lds_array_busy": lds["SQ_LDS_IDX_ACTIVE"] / (256.0 * lds["GRBM_GUI_ACTIVE"] / 8.0),
    "lds_bank_conflict_frac": lds["SQ_LDS_BANK_CONFLICT"] / max(1.0, lds["SQ_LDS_IDX_ACTIVE"]),
    "counters": {"sq_mix": mix, "sq_busy": busy, "mfma": mfma, "lds": lds},
    "source": "profiles/%s/pmc_eff_%s.csv (rocprofv3 --pmc, C4 --c4-cycle 0.3,0.1, averaged over the %d dispatches)"
              % (rdir, tag, n1),
}
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
d = json.load(open(path))
d["C4-efforts-dof53-b65536"] = e
json.dump(d, open(path, "w"), indent=1)
keep = ("Dispatch_Id", "Kernel_Name", "Grid_Size", "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Counter_Name",
        "Counter_Value", "Start_Timestamp", "End_Timestamp")
os.makedirs(os.path.join(ROOT, "profiles", rdir), exist_ok=True)
with open(os.path.join(ROOT, "profiles", rdir, "pmc_eff_%s.csv" % tag), "w") as f:
    w = csv.DictWriter(f, fieldnames=list(keep))
    w.writeheader()
    for rows in (r1, r2, r3, r4):
        for r in rows:
            w.writerow({k: r[k] for k in keep})
shutil.copy(os.path.join(base, "trace", "run_kernel_stats.csv"),
            os.path.join(ROOT, "profiles", rdir, "kernel_stats_eff_%s.csv" % tag))
print(json.dumps({k: v for k, v in e.items() if k != "counters"}, indent=1))
