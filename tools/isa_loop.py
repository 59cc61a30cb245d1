#!/usr/bin/env python3
"""Instruction mix of the epoch loop body of k_psp_epoch<53, 1, 1, 0> in the
production build (no stamps): VALU, v_cmp, lane (readlane / writelane, incl.
SGPR-spill traffic), fp64, v_cndmask, SALU, LDS.  The stamped build of
tools/isa_phases.py has more SGPR pressure and can mislead on spill traffic.

usage: tools/isa_loop.py [extra hipcc flags...]"""
import collections
import os
import subprocess
import sys

# UWVK_SR=0: the left-side instantiation (uwvk_psp_k.hip); default the right side
SR = os.environ.get("UWVK_SR", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
out = "/tmp/psp_loop.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
                "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-mfma-vgpr-form",
                *sys.argv[1:], "-I", os.path.join(PKG, "csrc"), "-I", os.path.join(ROOT, "include"),
                "-S", "-o", out, os.path.join(PKG, "csrc", "uwvk_psp_k_r.hip" if SR == "1" else "uwvk_psp_k.hip")], check=True, stderr=subprocess.DEVNULL)
s = open(out).read().split("\n")
name="_ZN4uwvk3psp11k_psp_epochILi53ELi1ELi1ELi%sEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % SR
st=[i for i,l in enumerate(s) if l.startswith(name+":")][0]
en=[i for i,l in enumerate(s) if i>st and l.startswith(".Lfunc_end")][0]
L=[l.strip() for l in s[st:en] if l.strip() and not l.strip().startswith(';')]
best=None
for hdr,t in enumerate(L):
    if 'Loop Header: Depth=1' in t:
        lab=t.split(':')[0]
        bs=[i for i,x in enumerate(L) if x.startswith(('s_branch','s_cbranch')) and x.endswith(' '+lab)]
        if bs and (best is None or max(bs)-hdr>best[1]-best[0]): best=(hdr,max(bs),lab)
hdr,back,lab=best
c=collections.Counter()
for t in L[hdr:back+1]:
    op=t.split()[0]
    if op.startswith('v_'):
        c['valu']+=1
        if op.startswith('v_cmp'): c['cmp']+=1
        if op.startswith(('v_readlane','v_writelane')): c['lane']+=1
        if 'f64' in op and not op.startswith('v_cmp'): c['f64']+=1
        if op.startswith('v_cndmask'): c['cnd']+=1
    elif op.startswith('s_'): c['salu']+=1
    elif op.startswith('ds_'): c['lds']+=1
print(' '.join(sys.argv[1:]) or '(default)', dict(c))
