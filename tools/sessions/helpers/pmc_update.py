#!/usr/bin/env python3
"""Fold the PMC passes of one tools/gpu_round.sh run into profiles/pmc_traffic.json.

usage: tools/pmc_update.py TAG [EPOCHS]   (reads gpurun_out/TAG/pmc_{fetch,write,sq})
The timed launch is the longest k_psp_epoch<53> dispatch (EPOCHS epochs, default 200).
FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B reads at 64 B)."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 200
base = os.path.join(ROOT, "gpurun_out", tag)
KERNEL = "k_psp_epoch<53"  # k_psp_epoch<53, QM> (r03: instantiated per process-noise shape)


def longest(pass_name):
    rows = [r for r in csv.DictReader(open(os.path.join(base, pass_name, "run_counter_collection.csv")))
            if KERNEL in r["Kernel_Name"]]
    did = max(rows, key=lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))["Dispatch_Id"]
    return {r["Counter_Name"]: float(r["Counter_Value"]) for r in rows if r["Dispatch_Id"] == did}, did


fetch, d1 = longest("pmc_fetch")
write, d2 = longest("pmc_write")
sq, d3 = longest("pmc_sq")
waves = sq.get("SQ_WAVES", 65536.0)
path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
d = json.load(open(path))
e = d["C3-dof53-b65536"]
e["epochs_per_launch"] = epochs
e["fetch_size_kib_raw"] = fetch["FETCH_SIZE"]
e["write_size_kib_raw"] = write["WRITE_SIZE"]
e["fetch_bytes"] = fetch["FETCH_SIZE"] * 1024 * 2
e["write_bytes"] = write["WRITE_SIZE"] * 1024
e["bytes_per_launch"] = e["fetch_bytes"] + e["write_bytes"]
e["valu_insts_per_epoch"] = sq["SQ_INSTS_VALU"] / epochs
e["valu_insts_per_wave_epoch"] = sq["SQ_INSTS_VALU"] / (waves * epochs)
e["per_wave_epoch"] = {k.replace("SQ_INSTS_", "").lower(): v / (waves * epochs) for k, v in sq.items()
                       if k.startswith("SQ_INSTS_")}
e["source"] = ("profiles/r01/pmc_%s.csv (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; dispatches "
               "%s / %s = the %d-epoch timed launch)" % (tag, d1, d2, epochs))
e["valu_source"] = "profiles/r01/pmc_%s.csv (rocprofv3 --pmc SQ_INSTS_VALU ..., dispatch %s)" % (tag, d3)
json.dump(d, open(path, "w"), indent=1)
rows = []
for p in ("pmc_fetch", "pmc_write", "pmc_sq"):
    for r in csv.DictReader(open(os.path.join(base, p, "run_counter_collection.csv"))):
        if "psp" in r["Kernel_Name"]:
            rows.append({k: r[k] for k in ("Dispatch_Id", "Kernel_Name", "Grid_Size", "VGPR_Count", "SGPR_Count",
                                           "LDS_Block_Size", "Counter_Name", "Counter_Value", "Start_Timestamp",
                                           "End_Timestamp")})
with open(os.path.join(ROOT, "profiles", "r01", "pmc_%s.csv" % tag), "w") as f:
    w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)
print(json.dumps(e, indent=1))
