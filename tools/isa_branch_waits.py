#!/usr/bin/env python3
"""Exec-masked branches of the C3 epoch loop that wait for LDS (diagnostic):
compiles the shipped PSP translation unit (production flags, C3 hot path) to
gfx950 assembly and lists each s_and_saveexec ... s_cbranch_execz region that
contains an LDS load and an s_waitcnt lgkmcnt inside it: such a branch exposes
the load's latency once per lane group instead of overlapping it (r04: the
A-coupled rows' 12 such branches cost 2.2%, profiles/r04/ab_cpl/).
usage: tools/isa_branch_waits.py [extra hipcc flags...]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
out = "/tmp/psp_branch.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-mfma-vgpr-form",
                *sys.argv[1:], "-S", "-o", out, os.path.join(PKG, "csrc", "uwvk_psp_k.hip")],
               check=True, stderr=subprocess.DEVNULL)
s = open(out).read().split("\n")
name = "_ZN4uwvk3psp11k_psp_epochILi53ELi1ELi1ELi0EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE"
a = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
b = [i for i, l in enumerate(s) if i > a and l.startswith(".Lfunc_end")][0]
L = s[a:b + 1]
n = 0
i = 0
while i < len(L):
    t = L[i].strip()
    if t.startswith("s_cbranch_execz"):
        target = t.split()[1]
        j = i + 1
        body = []
        while j < len(L) and not L[j].startswith(target + ":"):
            body.append(L[j].strip())
            j += 1
        loads = [x for x in body if x.startswith("ds_read")]
        waits = [x for x in body if x.startswith("s_waitcnt") and "lgkmcnt" in x]
        if loads and waits and len(body) < 60:
            n += 1
            print("--- %s (line %d): %d LDS loads, %d waits, %d instructions" % (target, i, len(loads), len(waits), len(body)))
            for x in body[:14]:
                print("    " + x)
    i += 1
print("%d branch regions with an LDS load and an lgkmcnt wait" % n)
