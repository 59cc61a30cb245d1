#!/usr/bin/env python3
"""Per-kernel ISA comparison of one translation unit between the working tree
and a git revision: both are compiled to gfx950 assembly with the Makefile's
flags (tools/isa_hash.py), split into functions (label .. .Lfunc_end) and
hashed per mangled name (and their opcode sequences compared, which a
register renaming leaves equal), so that a refactor that also ADDS kernels to a unit
can be shown to leave the existing kernels' code unchanged.

usage: tools/kernel_isa_diff.py REV [TU ...]   (default TU: uwvk_psp_k uwvk_psp_k_r)
"""
import hashlib
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_hash import BASE, HIPCC, norm, psp_flags  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(pkg, tu):
    flags = list(BASE) + (psp_flags() if tu.startswith("uwvk_psp_k") else [])
    r = subprocess.run([HIPCC] + flags + ["--cuda-device-only", "-S", "csrc/%s.hip" % tu, "-o", "-"], cwd=pkg,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-2000:])
    out, ops, cur, body = {}, {}, None, []
    for line in norm(r.stdout).splitlines():
        m = re.match(r"^(_Z\w+):\s*$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.startswith(".Lfunc_end"):
            out[cur] = hashlib.sha256("\n".join(body).encode()).hexdigest()
            ops[cur] = [b.split()[0] for b in body if b.strip() and not b.strip().endswith(":")]
            cur = None
            continue
        if cur:
            body.append(line)
    return out, ops


def main():
    rev = sys.argv[1]
    tus = sys.argv[2:] or ["uwvk_psp_k", "uwvk_psp_k_r"]
    with tempfile.TemporaryDirectory() as wt:
        subprocess.run(["git", "worktree", "add", "--detach", wt, rev], cwd=ROOT, check=True, capture_output=True)
        try:
            for tu in tus:
                old, oops = kernels(os.path.join(wt, "slam-uwv_kalman_filters_amd"), tu)
                new, nops = kernels(os.path.join(ROOT, "slam-uwv_kalman_filters_amd"), tu)
                same = sorted(k for k in old if new.get(k) == old[k])
                diff = sorted(k for k in old if k in new and new[k] != old[k])
                print("%s: %d kernels identical, %d changed, %d removed, %d added" %
                      (tu, len(same), len(diff), len([k for k in old if k not in new]),
                       len([k for k in new if k not in old])))
                for k in diff:  # register renaming only, or other instructions
                    print("  changed (%s):" % ("same opcode sequence" if oops[k] == nops[k] else
                                               "opcodes %d -> %d" % (len(oops[k]), len(nops[k]))), k)
                for k in sorted(set(new) - set(old)):
                    print("  added:  ", k)
        finally:
            subprocess.run(["git", "worktree", "remove", "--force", wt], cwd=ROOT, capture_output=True)


if __name__ == "__main__":
    main()
