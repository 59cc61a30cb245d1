#!/usr/bin/env python3
"""Static LDS instruction mix and LDS-array cycle estimate per phase of the C3
epoch kernel (diagnostic; run tools/isa_phases.py first, it writes
/tmp/psp_phases.s).  Cycles per wave-instruction from MI355X_MICROARCH.md's LDS
table (ds_read_b64 2, ds_read2_b64 8, ds_read_b128 4, ds_write_b64 4 array
cycles, ...); loops counted once.  The measured total to compare with is
SQ_LDS_IDX_ACTIVE per instance-epoch (profiles/pmc_traffic.json "lds")."""
import collections
import sys

dof = sys.argv[1] if len(sys.argv) > 1 else "53"
s = open("/tmp/psp_phases.s").read().split("\n")
name = "_ZN4uwvk3psp11k_psp_epochILi%sELi1ELi1ELi0EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % dof
st = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
en = [i for i, l in enumerate(s) if i > st and l.startswith(".Lfunc_end")][0]
COST = {"ds_read_b32": 2, "ds_read_b64": 2, "ds_read_b128": 4, "ds_read2_b64": 8, "ds_read2_b32": 4,
        "ds_read2st64_b64": 8, "ds_write_b32": 2, "ds_write_b64": 4, "ds_write2_b64": 8, "ds_write2st64_b64": 8,
        "ds_write_b128": 8, "ds_bpermute_b32": 2}
NAMES = ["prologue", "load", "epoch inputs", "predict pchol", "predict points", "manifold mean", "ori + L Delta",
         "A-coupled rows", "flat pass", "mean update", "update pchol", "points + zbar + S", "H, P, G", "C, S, gain",
         "Sigma -= C K^T", "apply_delta", "loop end"]
segs = [collections.Counter()]
for l in s[st:en + 1]:
    t = l.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op == "s_memtime":
        segs.append(collections.Counter())
    elif op.startswith("ds_"):
        segs[-1][op] += 1
tot = 0
for i, c in enumerate(segs):
    cyc = sum(COST.get(k, 4) * v for k, v in c.items())
    tot += cyc
    print("%-2d %-18s %4d instr %5d cycles  %s" % (i, NAMES[i] if i < len(NAMES) else "", sum(c.values()), cyc,
                                                  " ".join("%s:%d" % kv for kv in sorted(c.items()))))
print("total (static) %d LDS-array cycles" % tot)
