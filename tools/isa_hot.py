#!/usr/bin/env python3
"""Static instruction mix of the C3 epoch loop of k_psp_epoch<53> (diagnostic):
compiles the PSP translation unit (r05: PSP_HOT_ONLY is gone; the epoch loop keeps the
predict and the acceleration update only) plus any extra flags, finds the epoch
loop (the outermost loop of the kernel) and counts its instructions by class.
Inner loops (rank-M blocks, manifold-mean iterations) are counted once.

usage: tools/isa_hot.py [extra hipcc flags...]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")


def mix(extra=(), dof=53):
    out = "/tmp/psp_hot_%d.s" % os.getpid()
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                    "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-mfma-vgpr-form", *extra, "-S", "-o", out,
                    os.path.join(PKG, "csrc", "uwvk_psp_k.hip")], check=True, stderr=subprocess.DEVNULL)
    s = open(out).read().split("\n")
    os.unlink(out)
    name = "_ZN4uwvk3psp11k_psp_epochILi%dELi1ELi1ELi0EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % dof
    st = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
    en = [i for i, l in enumerate(s) if i > st and l.startswith(".Lfunc_end")][0]
    body = s[st:en + 1]
    hdr = [l for l in body if "This Loop Header: Depth=1" in l]
    lab = hdr[0].split(":")[0] if hdr else None
    key = "Header=%s " % lab.lstrip(".L") if lab else None
    idx = [i for i, l in enumerate(body) if key and key in l + " "]
    lo, hi = (idx[0], idx[-1]) if idx else (0, len(body))
    # extend hi to the back-edge branch
    for j in range(hi, len(body)):
        if lab and re.search(r"s_(cbranch_\w+|branch)\s+%s\b" % re.escape(lab), body[j]):
            hi = j
            break
    c = collections.Counter()
    for l in body[lo:hi + 1]:
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if "f64" in op and not op.startswith("v_cmp"):
                c["f64"] += 1
            elif op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
                c["lane"] += 1
                if re.search(r"v(14[5-9]|15\d)\b", t):
                    c["spill_lane"] += 1
            elif op.startswith("v_mov") or "dpp" in t:
                c["mov"] += 1
            elif op.startswith("v_cndmask"):
                c["cnd"] += 1
            elif op.startswith("v_cmp"):
                c["cmp"] += 1
            else:
                c["int/other"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
            if op == "s_nop":
                c["s_nop"] += 1
            if op == "s_waitcnt":
                c["waitcnt"] += 1
        elif op.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
    return c


KEYS = ["valu", "f64", "int/other", "mov", "cnd", "cmp", "lane", "spill_lane", "lds", "salu", "s_nop", "waitcnt", "vmem"]

if __name__ == "__main__":
    c = mix(sys.argv[1:])
    print(" ".join("%s=%d" % (k, c[k]) for k in KEYS))
