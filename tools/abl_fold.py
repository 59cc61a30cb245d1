#!/usr/bin/env python3
"""Per-phase budget of k_psp_epoch<53> from the ablation counter passes of
tools/abl_pmc.sh (gpurun_out/TAG/<variant>/): for each ablation, the counters
per instance-epoch of the timed (last, 20-epoch) launch and the kernel time,
and the difference to base = the phase's share.  Writes the table to stdout
and, with --json PATH, the numbers.
usage: tools/abl_fold.py TAG [--json PATH]"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
base = os.path.join(ROOT, "gpurun_out", tag)
PHASE = {"base": "(all)", "a1": "manifold mean beyond 1 iteration", "a2": "Sigma -= C K^T (rank-M)",
         "a4": "L Delta / X (ori x lin)", "a8": "predict partial Cholesky (15 columns)",
         "a16": "predict sigma points (orientation model)", "a32": "update partial Cholesky (6 columns)",
         "a64": "A-coupled rows (pos / vel)", "a128": "flat pass (Q band)", "a256": "apply_delta"}


def counters(v):
    rows = [r for r in csv.DictReader(open(os.path.join(base, v, "run_counter_collection.csv")))
            if "k_psp_epoch<53" in r["Kernel_Name"]]
    did = max(int(r["Dispatch_Id"]) for r in rows)
    c = {}
    for r in rows:
        if int(r["Dispatch_Id"]) == did:
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return c


out = {}
for v in PHASE:
    p = os.path.join(base, v, "run_counter_collection.csv")
    if not os.path.exists(p):
        continue
    c = counters(v)
    line = json.loads(open(os.path.join(base, v + ".json")).read().strip().splitlines()[-1])
    ie = line["config"]["batch_per_gpu"] * line["steps"]
    e = {k.replace("SQ_INSTS_", "").lower(): c[k] / ie for k in c if k.startswith("SQ_INSTS_")}
    e["fp64_lane_flop"] = 64 * (2 * e["valu_fma_f64"] + e["valu_mul_f64"] + e["valu_add_f64"] + e["valu_trans_f64"])
    e["kernel_ms"] = line["timing"]["kernel_ms"]
    out[v] = e
b = out["base"]
keys = ["valu", "valu_fma_f64", "valu_mul_f64", "valu_add_f64", "valu_trans_f64", "salu", "lds", "fp64_lane_flop", "kernel_ms"]
print("%-44s " % "phase removed" + " ".join("%9s" % k.replace("valu_", "")[:9] for k in keys))
for v, e in out.items():
    row = [e[k] if v == "base" else b[k] - e[k] for k in keys]
    print("%-44s " % PHASE[v] + " ".join("%9.1f" % x if k != "kernel_ms" else "%9.3f" % x for k, x in zip(keys, row)))
if "--json" in sys.argv:
    json.dump({"tag": tag, "per_instance_epoch": out, "phases": PHASE}, open(sys.argv[sys.argv.index("--json") + 1], "w"),
              indent=1)
