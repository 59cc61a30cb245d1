"""Register / scratch budget of the hot kernel (CPU: hipcc cross-compile only).

k_psp_epoch<53> must keep 3 waves per SIMD (<= 168 VGPRs, no scratch): with
12 instances per CU from the LDS budget every wave slot is used (DESIGN.md
section 5).  A harmless-looking change once took it to 173 VGPRs, 800 B/lane
of scratch and 2 waves per SIMD (a noinline helper taking the EpochArgs
reference); this test catches that class of regression before a GPU run."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
HIPCC = "/opt/rocm/bin/hipcc"


def psp_flags():
    """The PSP translation unit's extra flags, from the Makefile's PSP_FLAGS line."""
    for line in open(os.path.join(PKG, "Makefile")):
        if line.startswith("PSP_FLAGS :="):
            return line.split(":=", 1)[1].split()
    raise AssertionError("PSP_FLAGS not found in the Makefile")


def kernel_usage(src, mangled_prefix, extra=()):
    cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
           *psp_flags(), *extra, "-c", src, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            continue
        if cur and cur.startswith(mangled_prefix):
            for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"\bAGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                             ("occupancy", r"Occupancy \[waves/SIMD\]: (\d+)")):
                m = re.search(pat, line)
                if m:
                    out[key] = int(m.group(1))
    return out


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="no hipcc")
def test_psp_epoch_kernel_keeps_three_waves_per_simd():
    u = kernel_usage("csrc/uwvk_psp_k.hip", "_ZN4uwvk3psp11k_psp_epochILi53E")
    assert u, "k_psp_epoch<53> not found in the resource report"
    # VGPRs and AGPRs share one 512-entry file per SIMD lane: 3 waves need <= 168 together
    assert u["vgpr"] + u.get("agpr", 0) <= 168 and u["scratch"] == 0 and u["occupancy"] >= 3, u
