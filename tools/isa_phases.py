#!/usr/bin/env python3
"""Static VALU mix per phase of k_psp_epoch<DOF> (diagnostic): compiles the PSP
translation unit with -DUWVK_STAMPS to gfx950 assembly and splits the kernel at
the s_memtime of every UWVK_STAMP (sched_barrier keeps phases apart).  Loops are
counted once (the rank-M blocks, the manifold-mean iterations).

usage: tools/isa_phases.py [DOF] [extra hipcc flags...]"""
import collections
import os
import re
import subprocess
import sys

# UWVK_SR=0: the left-side instantiation (uwvk_psp_k.hip); default the right side
SR = os.environ.get("UWVK_SR", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
dof = sys.argv[1] if len(sys.argv) > 1 else "53"
extra = sys.argv[2:]
out = "/tmp/psp_phases.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-mfma-vgpr-form", "-DUWVK_STAMPS", *extra, "-S", "-o", out,
                os.path.join(PKG, "csrc", "uwvk_psp_k_r.hip" if SR == "1" else "uwvk_psp_k.hip")], check=True, stderr=subprocess.DEVNULL)
s = open(out).read().split("\n")
name = "_ZN4uwvk3psp11k_psp_epochILi%sELi1ELi1ELi%sEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % (dof, SR)
st = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
en = [i for i, l in enumerate(s) if i > st and l.startswith(".Lfunc_end")][0]
INT = re.compile(r"v_(add|sub|subrev|mul_lo|mul_hi|mad|lshl|lshr|ashr|and|or|xor|bfe|bfi|max|min|cvt|mul_u32|"
                 r"lshlrev|lshrrev|ashrrev|not|perm|alignbit|add3|lshl_add|lshl_or|and_or|or3|xad)_")
segs, cur = [], collections.Counter()
for l in s[st:en + 1]:
    t = l.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    if op == "s_memtime":
        segs.append(cur)
        cur = collections.Counter()
        continue
    if op.startswith("v_"):
        cur["valu"] += 1
        if "f64" in op and not op.startswith("v_cmp"):
            cur["f64"] += 1
        elif op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            cur["lane"] += 1
        elif "dpp" in op or "dpp" in t:
            cur["dpp"] += 1
        elif op.startswith("v_cndmask"):
            cur["cnd"] += 1
        elif op.startswith("v_mov"):
            cur["mov"] += 1
        elif op.startswith("v_cmp"):
            cur["cmp"] += 1
        elif INT.match(op):
            cur["int"] += 1
        else:
            cur["other"] += 1
    elif op.startswith("ds_"):
        cur["lds"] += 1
    elif op.startswith("s_"):
        cur["salu"] += 1
segs.append(cur)
keys = ["valu", "f64", "int", "mov", "cnd", "lane", "dpp", "cmp", "other", "lds", "salu"]
print("%-4s " % "seg" + " ".join("%6s" % k for k in keys))
for i, c in enumerate(segs):
    print("%-4d " % i + " ".join("%6d" % c[k] for k in keys))
