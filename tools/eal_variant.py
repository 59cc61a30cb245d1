#!/usr/bin/env python3
"""Rebuild the r04o `PSP_EA_LAUNDER` variant (EpochArgs read through its
kernel-argument address, re-laundered in the constant address space every
epoch) from the current source, compile it and the shipped
PSP unit to gfx950 assembly, and report how each forms the address of the
laundered object: the shipped kernel launders `b.shared` (a hipMalloc'ed
global pointer), the variant `&ea` (the address of a by-value kernel
parameter).  The variant's source is a textual patch of csrc/uwvk_psp_k.hip
written to a temporary directory; nothing in the package changes.

usage: tools/eal_variant.py OUTDIR
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
sys.path.insert(0, os.path.join(ROOT, "tools"))
from isa_hash import BASE, HIPCC, psp_flags  # noqa: E402

LAUNDER = '''
// r04o variant (PSP_EA_LAUNDER): EpochArgs through its own address, laundered
// as a constant-address-space pointer once per epoch
UWVK_DEV const EpochArgs& launder_ea(const EpochArgs& ea) {
  using CP = const __attribute__((address_space(4))) EpochArgs*;
  CP p = (CP)&ea;
  asm volatile("" : "+s"(p));
  return *(const EpochArgs*)p;
}
'''


def make_variant(out):
    src = open(os.path.join(PKG, "csrc", "uwvk_psp_k.hip")).read()
    anchor = "UWVK_DEV const PoseShared& shared_for_epoch(const PoseBufs& b) {"
    assert anchor in src
    src = src.replace(anchor, LAUNDER + "\n" + anchor, 1)
    loop = "  for (int64_t e = e_begin; e < e_end; e++) {\n"
    assert src.count(loop) == 1
    i0 = src.index(loop) + len(loop)
    depth, i = 1, i0
    while depth:  # the loop body: uses of ea inside it read the laundered reference
        depth += {"{": 1, "}": -1}.get(src[i], 0)
        i += 1
    body = re.sub(r"\bea\b", "eal", src[i0:i])
    src = src[:i0] + "    const EpochArgs& eal = launder_ea(ea);\n" + body + src[i:]
    d = os.path.join(out, "csrc")
    os.makedirs(d, exist_ok=True)
    for f in os.listdir(os.path.join(PKG, "csrc")):
        if f.endswith(".hpp"):
            shutil.copy(os.path.join(PKG, "csrc", f), d)
    open(os.path.join(d, "uwvk_psp_k.hip"), "w").write(src)
    os.makedirs(os.path.join(out, "..", "include"), exist_ok=True)
    return os.path.join(d, "uwvk_psp_k.hip")


def asm(src, out):
    cmd = [HIPCC] + BASE + psp_flags() + ["-I", os.path.join(ROOT, "include"), "--cuda-device-only", "-S", src,
                                         "-o", out]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    return open(out).read()


def kernel_body(text, name_re):
    lines = text.split("\n")
    st = [i for i, l in enumerate(lines) if re.match(r"^%s\w*:" % name_re, l)]
    assert st, name_re
    i = st[0]
    en = [k for k in range(i, len(lines)) if lines[k].startswith(".Lfunc_end")][0]
    return lines[i:en]


def report(body, tag):
    scratch_st = [l.strip() for l in body if "scratch_store" in l or "buffer_store" in l and "off, s[0:3]" in l]
    aperture = [l.strip() for l in body if "src_private_base" in l or "SH_MEM_BASES" in l or "private_base" in l]
    sload = [l.strip() for l in body if re.match(r"\s*s_load_dword", l)]
    print("== %s: %d lines, %d scratch stores, %d s_load, private-aperture refs: %d" %
          (tag, len(body), len(scratch_st), len(sload), len(aperture)))
    for l in aperture[:6]:
        print("   aperture:", l)
    for l in scratch_st[:6]:
        print("   scratch :", l)
    return scratch_st, aperture


def main():
    out = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else "/tmp/eal")
    os.makedirs(out, exist_ok=True)
    vsrc = make_variant(os.path.join(out, "variant"))
    shipped = asm(os.path.join(PKG, "csrc", "uwvk_psp_k.hip"), os.path.join(out, "shipped.s"))
    # the variant includes "../../include/uwvk.h" relative to its csrc/: mirror it
    inc = os.path.join(out, "include")
    os.makedirs(inc, exist_ok=True)
    shutil.copy(os.path.join(ROOT, "include", "uwvk.h"), inc)
    variant = asm(vsrc, os.path.join(out, "variant.s"))
    k = r"_ZN4uwvk3psp11k_psp_epochILi53ELi1ELi1ELi0EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE"
    report(kernel_body(shipped, k), "shipped k_psp_epoch<53,1,1,0>")
    report(kernel_body(variant, k), "variant k_psp_epoch<53,1,1,0>")


if __name__ == "__main__":
    main()
