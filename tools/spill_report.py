#!/usr/bin/env python3
"""SGPR spill traffic of the C3 epoch loop of k_psp_epoch<53> (diagnostic):
compiles the PSP translation unit (+ extra flags; r05: the hot-path-only diagnostic defines are gone, the whole kernel is analysed), finds the VGPRs
used as SGPR spill lanes, and lists the spill slots by the number of reloads
(v_readlane from a spill VGPR) inside the epoch loop, with the instruction that
defined the spilled SGPR before the loop (a kernarg s_load offset names the
kernel argument) or "loop" when the slot is rewritten inside the loop.

usage: tools/spill_report.py [extra hipcc flags...]   (FULL=1: the shipped build, cold paths included)"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
out = "/tmp/spill_%d.s" % os.getpid()
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-mfma-vgpr-form", *sys.argv[1:], "-S", "-o", out,
                os.path.join(PKG, "csrc", "uwvk_psp_k.hip")], check=True, stderr=subprocess.DEVNULL)
s = open(out).read().split("\n")
os.unlink(out)
name = "_ZN4uwvk3psp11k_psp_epochILi53ELi1ELi1ELi0EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE"
a = [i for i, l in enumerate(s) if l.startswith(name + ":")][0]
b = [i for i, l in enumerate(s) if i > a and l.startswith(".Lfunc_end")][0]
L = s[a:b + 1]
hdr = [i for i, l in enumerate(L) if "This Loop Header: Depth=1" in l][0]
lab = L[hdr].split(":")[0]
en = max(i for i, l in enumerate(L) if re.search(r"s_(cbranch_\w+|branch)\s+%s\b" % re.escape(lab), l))
spill_v = collections.Counter(m.group(1) for l in L for m in [re.match(r"\s*v_writelane_b32\s+(v\d+)", l)] if m)
spill_v = {v for v, n in spill_v.items() if n >= 4}
rel, wr_loop, src = collections.Counter(), set(), {}
for i, l in enumerate(L):
    m = re.match(r"\s*v_writelane_b32\s+(v\d+),\s*(s\d+),\s*(\d+)", l)
    if m and m.group(1) in spill_v:
        key = (m.group(1), int(m.group(3)))
        if hdr <= i <= en:
            wr_loop.add(key)
        elif i < hdr:
            n = int(m.group(2)[1:])
            for j in range(i - 1, max(0, i - 80), -1):
                mm = re.match(r"\s*(s_\w+|v_readfirstlane_b32|v_readlane_b32)\s+(s\[(\d+):(\d+)\]|s(\d+))", L[j])
                if not mm:
                    continue
                lo = int(mm.group(3) or mm.group(5))
                hi = int(mm.group(4) or mm.group(5))
                if lo <= n <= hi:
                    src[key] = L[j].strip()
                    break
    m = re.match(r"\s*v_readlane_b32\s+s\d+,\s*(v\d+),\s*(\d+)", l)
    if m and m.group(1) in spill_v and hdr <= i <= en:
        rel[(m.group(1), int(m.group(2)))] += 1
print("spill VGPRs %s; loop reloads %d over %d slots; loop spill writes %d" %
      (sorted(spill_v), sum(rel.values()), len(rel),
       sum(1 for i in range(hdr, en + 1) if re.match(r"\s*v_writelane_b32\s+(v\d+)", L[i]) and
           re.match(r"\s*v_writelane_b32\s+(v\d+)", L[i]).group(1) in spill_v)))
for k, n in sorted(rel.items(), key=lambda kv: -kv[1])[:int(os.environ.get("TOP", "40"))]:
    print("%3d %-12s %s" % (n, "%s:%d" % k, "loop" if k in wr_loop else src.get(k, "?")[:100]))
