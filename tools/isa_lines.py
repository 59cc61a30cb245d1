#!/usr/bin/env python3
"""Static VALU per source line inside the epoch loop of k_psp_epoch<53, 1, 1, SR>
(diagnostic): the production flags plus -gline-tables-only, the loop body found
as in tools/isa_loop.py, every instruction charged to the last .loc before it
(inlined code is charged to the innermost source line).  Static counts: blocks
that are skipped at run time (library fallbacks, NaN paths, rare events) count
as much as the hot ones, so read the list with the source beside it.

usage: tools/isa_lines.py [N] [extra hipcc flags...]"""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_hash import BASE, HIPCC, psp_flags  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
SR = os.environ.get("UWVK_SR", "1")
N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
out = "/tmp/psp_lines.s"
tu = "uwvk_psp_k_r.hip" if SR == "1" else "uwvk_psp_k.hip"
subprocess.run([HIPCC] + BASE + psp_flags() + ["-gline-tables-only", "--cuda-device-only", "-S", "-o", out,
                                                "csrc/" + tu] + sys.argv[2:], cwd=PKG, check=True)
s = open(out).read().split("\n")
files = {}
for l in s:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m:
        files[m.group(1)] = os.path.basename(m.group(3) or m.group(2))
name = "_ZN4uwvk3psp11k_psp_epochILi53ELi1ELi1ELi%sEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % SR
st = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
en = [i for i, l in enumerate(s) if i > st and l.startswith(".Lfunc_end")][0]
L = [l.strip() for l in s[st:en]]
best = None
for hdr, t in enumerate(L):
    if "Loop Header: Depth=1" in t:
        lab = t.split(":")[0]
        bs = [i for i, x in enumerate(L) if x.startswith(("s_branch", "s_cbranch")) and x.endswith(" " + lab)]
        if bs and (best is None or max(bs) - hdr > best[1] - best[0]):
            best = (hdr, max(bs))
# the last .loc before the loop header
loc = None
for t in L[:best[0]]:
    if t.startswith(".loc"):
        loc = t
c, kinds = collections.Counter(), collections.defaultdict(collections.Counter)
for t in L[best[0]:best[1] + 1]:
    if t.startswith(".loc"):
        p = t.split()
        loc = "%s:%s" % (files.get(p[1], p[1]), p[2])
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op.startswith("v_"):
        c[loc] += 1
        k = "f64" if ("f64" in op and not op.startswith("v_cmp")) else op.split("_e32")[0].split("_e64")[0]
        kinds[loc][k] += 1
tot = sum(c.values())
print("loop body: %d static VALU" % tot)
for k, v in c.most_common(N):
    print("%5d  %-28s %s" % (v, k, ", ".join("%s %d" % kv for kv in kinds[k].most_common(4))))
