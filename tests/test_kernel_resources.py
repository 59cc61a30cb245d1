"""Register / scratch budget of the hot kernels (CPU: hipcc cross-compile only).

Every k_psp_epoch / k_psp_epoch_p instantiation (DOF 53 / 26, process-noise
shape QM, event set EVS, SO3 side SR) must keep 3 waves per SIMD (<= 168
VGPRs + AGPRs, no scratch): with 12 instances per CU from the LDS budget every
wave slot is used, and psp_epoch_slots sizes the
persistent grid from <DOF, 1, 0, 0> on the assumption that all of them fit the
same budget.  A harmless-looking change once took the kernel to 173 VGPRs,
800 B/lane of scratch and 2 waves per SIMD (a noinline helper taking the
EpochArgs reference); this test catches that class of regression before a GPU
run.  Usage is collected per mangled name, so no instantiation hides another."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
HIPCC = "/opt/rocm/bin/hipcc"


def psp_flags():
    """The PSP translation units' extra flags, from the Makefile's PSP_FLAGS line."""
    for line in open(os.path.join(PKG, "Makefile")):
        if line.startswith("PSP_FLAGS :="):
            return line.split(":=", 1)[1].split()
    raise AssertionError("PSP_FLAGS not found in the Makefile")


def kernel_usage(src, mangled_prefixes, extra=()):
    """{mangled name: {vgpr, agpr, scratch, occupancy}} for every kernel whose
    mangled name starts with one of mangled_prefixes."""
    cmd = [HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only",
           *psp_flags(), *extra, "-c", src, "-o", os.devnull,
           "-Rpass-analysis=kernel-resource-usage"]
    r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    out, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            if cur.startswith(tuple(mangled_prefixes)):
                out[cur] = {}
            continue
        if cur in out:
            for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"\bAGPRs: (\d+)"),
                             ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                             ("occupancy", r"Occupancy \[waves/SIMD\]: (\d+)")):
                m = re.search(pat, line)
                if m:
                    out[cur][key] = int(m.group(1))
    return out


PREFIXES = ("_ZN4uwvk3psp11k_psp_epochILi", "_ZN4uwvk3psp13k_psp_epoch_pILi")


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("src,side", [("csrc/uwvk_psp_k.hip", 0), ("csrc/uwvk_psp_k_r.hip", 1)])
def test_psp_epoch_kernels_keep_three_waves_per_simd(src, side):
    u = kernel_usage(src, PREFIXES)
    # 2 DOFs x 3 (QM, EVS) sets x {static, persistent}, all of this unit's side
    assert len(u) == 12, sorted(u)
    for name, r in u.items():
        assert name.endswith("ELi%dEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % side), name
        # VGPRs and AGPRs share one 512-entry file per SIMD lane: 3 waves need <= 168 together
        assert r["vgpr"] + r.get("agpr", 0) <= 168 and r["scratch"] == 0 and r["occupancy"] >= 3, (name, r)
