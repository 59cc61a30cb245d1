#!/usr/bin/env python3
"""Hash the gfx950 device assembly of every translation unit of libuwvk.so,
compiled with the Makefile's flags (`hipcc --cuda-device-only -S`), so that a
source-only refactor (e.g. pruning compile-time knobs) can be shown to leave
the shipped kernels unchanged.  Lines that name source files or the compiler
(`.file`, `.ident`, debug-line directives, comments) are dropped before hashing.

usage: tools/isa_hash.py [OUT.json] [--keep DIR]   (prints TU -> sha256)
"""
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
HIPCC = "/opt/rocm/bin/hipcc"
BASE = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function",
        "-Wno-unused-result"]


def psp_flags():
    """PSP_FLAGS of the Makefile (the PSP translation units only)."""
    for line in open(os.path.join(PKG, "Makefile")):
        if line.startswith("PSP_FLAGS :="):
            return line.split(":=", 1)[1].split()
    raise RuntimeError("PSP_FLAGS not found in the Makefile")


def norm(asm):
    out = []
    for line in asm.splitlines():
        s = line.strip()
        if not s or s.startswith(";") or s.startswith("//"):
            continue
        if re.match(r"\.(file|ident|loc|cfi_)", s):
            continue
        out.append(re.sub(r"\s*;.*$", "", line.rstrip()))
    return "\n".join(out) + "\n"


def one(src, keep):
    name = os.path.basename(src)[:-4]
    flags = list(BASE)
    if name in ("uwvk_psp_k", "uwvk_psp_k_r"):
        flags += psp_flags()
    cmd = [HIPCC] + flags + ["--cuda-device-only", "-S", src, "-o", "-"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("%s: %s" % (name, r.stderr[-2000:]))
    asm = norm(r.stdout)
    if keep:
        os.makedirs(keep, exist_ok=True)
        open(os.path.join(keep, name + ".s"), "w").write(asm)
    return name, hashlib.sha256(asm.encode()).hexdigest()


def main():
    args = [a for a in sys.argv[1:]]
    keep = None
    if "--keep" in args:
        i = args.index("--keep")
        keep = args[i + 1]
        del args[i:i + 2]
    srcs = sorted(glob.glob(os.path.join(PKG, "csrc", "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = dict(ex.map(lambda s: one(s, keep), srcs))
    for k in sorted(res):
        print("%-28s %s" % (k, res[k]))
    if args:
        json.dump(res, open(args[0], "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
