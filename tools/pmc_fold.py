#!/usr/bin/env python3
"""Fold one tools/pmc_r02.sh run into profiles/pmc_traffic.json (key
WORKLOAD-eSTEPS) and copy the summaries bench.py's roofline is computed from
into profiles/ROUND_DIR/.  The timed launch is the LAST k_psp_epoch<53> dispatch of
the bench (the alignment shift and the warm-up launches come first).

usage: tools/pmc_fold.py TAG STEPS [WORKLOAD] [ROUND_DIR (default r05)] [KERNEL]
An optional "mfma" pass (tools/pmc_r03.sh) adds the f64 MFMA counters.
KERNEL: a substring of the timed kernel's name (default from WORKLOAD: the
parameter-decoupled k_psp_epoch_p<26, 1, 1, 1, 1> for "-pd", k_psp_epoch_pair<1 for
"-pdpair", else k_psp_epoch<53,
which also matches the persistent k_psp_epoch_p<53)."""
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag, steps = sys.argv[1], int(sys.argv[2])
workload = sys.argv[3] if len(sys.argv) > 3 else "C3-dof53-b65536"
rdir = sys.argv[4] if len(sys.argv) > 4 else "r05"
base = os.path.join(ROOT, "gpurun_out", tag, "s%d" % steps)
# k_psp_epoch<53, QM, ...> (r03: instantiated per process-noise shape); a
# WORKLOAD ending in "-pair" folds the two-instances-per-wave k_psp2_epoch<53, SR>
KERNEL = "k_psp2_epoch<53" if workload.endswith("-pair") else "k_psp_epoch<53"
if workload.endswith("-pdpair"):  # r06: the two-instances-per-wave PD kernel (the default since r06)
    KERNEL = "k_psp_epoch_pair<%d" % (0 if "-left" in workload else 1)
if workload.endswith("-pd"):
    KERNEL = "k_psp_epoch_p<26, 1, 1, %d, 1>" % (0 if "-left" in workload else 1)
if len(sys.argv) > 5:
    KERNEL = sys.argv[5]
N_SIMD = 1024


def last(pass_name):
    rows = [r for r in csv.DictReader(open(os.path.join(base, pass_name, "run_counter_collection.csv")))
            if KERNEL in r["Kernel_Name"]]
    did = max(int(r["Dispatch_Id"]) for r in rows)
    sel = [r for r in rows if int(r["Dispatch_Id"]) == did]
    c = {}
    for r in sel:  # rocprofv3 may list a counter once per agent/dimension: sum
        c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return c, did, sel


mix, d1, rows_mix = last("sq_mix")
busy, d2, rows_busy = last("sq_busy")
fetch, d3, rows_f = last("fetch")
write, d4, rows_w = last("write")
has_mfma = os.path.exists(os.path.join(base, "mfma", "run_counter_collection.csv"))
mfma, d5, rows_m = last("mfma") if has_mfma else ({}, None, [])
waves = mix["SQ_WAVES"]
# normalised per instance-epoch: one wave per instance, except that the tail
# instances of a spread launch (UWVK_OPT_TAIL_SLOTS) run as several chunk
# waves, so SQ_WAVES exceeds the batch; "per_wave_epoch" keeps its r02 name
instances = int(re.search(r"-b(\d+)", workload).group(1))
we = instances * steps
e = {
    "kernel": "k_psp2_epoch<53, 1>" if workload.endswith("-pair") else (
              KERNEL + "> (53-DOF state, parameter-decoupled, two instances per wave)"
              if workload.endswith("-pdpair") else (
              KERNEL + " (53-DOF state, parameter-decoupled)" if workload.endswith("-pd") else
              "k_psp_epoch<53, 1, 1, %d>" % (0 if workload.endswith("-left") else 1))),
    "epochs_per_launch": steps, "waves": waves, "instances": instances,
    "fetch_size_kib_raw": fetch["FETCH_SIZE"], "write_size_kib_raw": write["WRITE_SIZE"],
    "fetch_bytes": fetch["FETCH_SIZE"] * 1024 * 2, "write_bytes": write["WRITE_SIZE"] * 1024,
}
e["bytes_per_launch"] = e["fetch_bytes"] + e["write_bytes"]
e["per_wave_epoch"] = {k.replace("SQ_INSTS_", "").lower(): v / we for k, v in mix.items() if k.startswith("SQ_INSTS_")}
# VALU busy from the measured issue counter: SQ_ACTIVE_INST_VALU counts quad-cycles
# (SQ_WAVE_CYCLES x 4 = a wave's lifetime in clocks, cross-checked against the
# wall-clock timeline); GRBM_GUI_ACTIVE is summed over the 8 XCDs
xcd_cycles = busy["GRBM_GUI_ACTIVE"] / 8.0
e["valu_busy"] = {
    "frac": busy["SQ_ACTIVE_INST_VALU"] * 4.0 / (N_SIMD * xcd_cycles),
    "definition": "SQ_ACTIVE_INST_VALU x 4 cycles / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs); the counter's "
                  "quad-cycle granularity rounds a 2-cycle wave64 32-bit VALU op up to 4, so this is an upper bound",
    "model_frac": (4.0 * (mix["SQ_INSTS_VALU_FMA_F64"] + mix["SQ_INSTS_VALU_MUL_F64"] + mix["SQ_INSTS_VALU_ADD_F64"]
                          + mix["SQ_INSTS_VALU_TRANS_F64"])
                   + 2.0 * (mix["SQ_INSTS_VALU"] - mix["SQ_INSTS_VALU_FMA_F64"] - mix["SQ_INSTS_VALU_MUL_F64"]
                            - mix["SQ_INSTS_VALU_ADD_F64"] - mix["SQ_INSTS_VALU_TRANS_F64"])) / (N_SIMD * xcd_cycles),
    "model_definition": "issue-cycle model: 4 cycles per wave64 fp64 instruction (78.6 TFLOP/s = 1024 x 2.4 GHz x 32), "
                        "2 per other wave64 VALU instruction (MI355X_MICROARCH.md), over the same SIMD-cycles (lower bound)",
    "counters": busy,
}
e["active_lanes"] = {
    "thread_cycles_per_valu_quad_cycle": busy["SQ_THREAD_CYCLES_VALU"] / busy["SQ_ACTIVE_INST_VALU"],
    "note": "SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU; 64 would be every lane of every VALU cycle",
}
if has_mfma:
    # SQ_INSTS_VALU_MFMA_MOPS_F64 counts f64 MFMA work in units of 512 flops
    # (v_mfma_f64_16x16x4: 16*16*4*2 = 2,048 flops = 4 units per wave instruction)
    e["mfma"] = {
        "insts_f64_per_wave_epoch": mfma["SQ_INSTS_VALU_MFMA_F64"] / we,
        "mops_f64_per_wave_epoch": mfma["SQ_INSTS_VALU_MFMA_MOPS_F64"] / we,
        "flop_per_wave_epoch": mfma["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512.0 / we,
        "busy_frac": mfma["SQ_VALU_MFMA_BUSY_CYCLES"] / mfma["SQ_BUSY_CU_CYCLES"],
        "busy_definition": "SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CU_CYCLES",
        "counters": mfma,
    }
# LDS passes (tools/pmc_lds.sh, r04), when present: LDS-array occupancy next to the VALU
rows_l = []
if os.path.exists(os.path.join(base, "lds", "run_counter_collection.csv")):
    lds, _, rows_l1 = last("lds")
    lds2, _, rows_l2 = last("lds2") if os.path.exists(os.path.join(base, "lds2", "run_counter_collection.csv")) else ({}, None, [])
    rows_l = rows_l1 + rows_l2
    cu_cycles = 256.0 * lds["GRBM_GUI_ACTIVE"] / 8.0
    e["lds"] = {
        "insts_per_wave_epoch": lds["SQ_INSTS_LDS"] / we,
        "array_cycles_per_wave_epoch": lds["SQ_LDS_IDX_ACTIVE"] / we,
        "bank_conflict_cycles_per_wave_epoch": lds["SQ_LDS_BANK_CONFLICT"] / we,
        "array_busy_frac": lds["SQ_LDS_IDX_ACTIVE"] / cu_cycles,
        "array_busy_definition": "SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM_GUI_ACTIVE / 8 XCDs)",
        "counters": dict(lds, **lds2),
    }
    if lds2:
        e["lds"]["wait_inst_lds_frac_of_wave_cycles"] = lds2["SQ_WAIT_INST_LDS"] / lds2["SQ_WAVE_CYCLES"]
e["source"] = ("profiles/%s/pmc_%s_s%d.csv (rocprofv3 --pmc, one pass per counter group; dispatch %d = the %d-epoch "
               "timed launch; FETCH_SIZE doubled per MI355X_MICROARCH.md)" % (rdir, tag, steps, d3, steps))
e["valu_source"] = "profiles/%s/pmc_%s_s%d.csv (dispatch %d)" % (rdir, tag, steps, d1)
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
d = json.load(open(path)) if os.path.exists(path) else {}
d["%s-e%d" % (workload, steps)] = e
json.dump(d, open(path, "w"), indent=1)
os.makedirs(os.path.join(ROOT, "profiles", rdir), exist_ok=True)
keep = ("Dispatch_Id", "Kernel_Name", "Grid_Size", "VGPR_Count", "SGPR_Count", "LDS_Block_Size", "Counter_Name",
        "Counter_Value", "Start_Timestamp", "End_Timestamp")
with open(os.path.join(ROOT, "profiles", rdir, "pmc_%s_s%d.csv" % (tag, steps)), "w") as f:
    w = csv.DictWriter(f, fieldnames=list(keep))
    w.writeheader()
    for rows in (rows_mix, rows_busy, rows_f, rows_w, rows_m, rows_l):
        for r in rows:
            w.writerow({k: r[k] for k in keep})
shutil.copy(os.path.join(base, "trace", "run_kernel_stats.csv"),
            os.path.join(ROOT, "profiles", rdir, "kernel_stats_%s_s%d.csv" % (tag, steps)))
if os.path.exists(os.path.join(base, "trace", "run_kernel_trace.csv")):
    shutil.copy(os.path.join(base, "trace", "run_kernel_trace.csv"),
                os.path.join(ROOT, "profiles", rdir, "kernel_trace_%s_s%d.csv" % (tag, steps)))
shutil.copy(os.path.join(base, "trace.json"), os.path.join(ROOT, "profiles", rdir, "bench_%s_s%d_traced.json" % (tag, steps)))
print(json.dumps({k: v for k, v in e.items() if k != "valu_busy"}, indent=1))
print("valu_busy", e["valu_busy"]["frac"], "model", e["valu_busy"]["model_frac"])
