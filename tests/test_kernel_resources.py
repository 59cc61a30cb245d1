"""Register / scratch budget of the hot kernels (CPU: hipcc cross-compile only).

Every k_psp_epoch / k_psp_epoch_p instantiation (DOF 53 / 26, process-noise
shape QM, event set EVS, SO3 side SR) must keep 3 waves per SIMD (<= 168
VGPRs + AGPRs, no scratch): with 12 instances per CU from the LDS budget every
wave slot is used, and psp_epoch_slots sizes the
persistent grid from <DOF, 1, 0, 0> on the assumption that all of them fit the
same budget.  A harmless-looking change once took the kernel to 173 VGPRs,
800 B/lane of scratch and 2 waves per SIMD (a noinline helper taking the
EpochArgs reference); this test catches that class of regression before a GPU
run.  Usage is collected per mangled name, so no instantiation hides another.

Each translation unit is compiled once per flag set (assembly and the
resource remarks from one hipcc run, the IR from another), all of them in
parallel on first use, and shared by the tests below."""
import concurrent.futures as cf
import functools
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "slam-uwv_kalman_filters_amd")
HIPCC = "/opt/rocm/bin/hipcc"
BASE = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "--cuda-device-only"]
HAVE_HIPCC = bool(shutil.which(HIPCC) or os.path.exists(HIPCC))


def psp_flags():
    """The PSP translation units' extra flags, from the Makefile's PSP_FLAGS line."""
    for line in open(os.path.join(PKG, "Makefile")):
        if line.startswith("PSP_FLAGS :="):
            return line.split(":=", 1)[1].split()
    raise AssertionError("PSP_FLAGS not found in the Makefile")


def tu_flags(src):
    """A translation unit's extra Makefile flags."""
    return tuple(psp_flags()) if os.path.basename(src)[:-4] in ("uwvk_psp_k", "uwvk_psp_k_r", "uwvk_psp_pair") else ()


@functools.lru_cache(maxsize=None)
def compile_asm(src, flags):
    """(gfx950 assembly, resource-usage remarks) of one translation unit."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "tu.s")
        cmd = [HIPCC, *BASE, *flags, "-S", src, "-o", out, "-Rpass-analysis=kernel-resource-usage"]
        r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        return open(out).read(), r.stderr


@functools.lru_cache(maxsize=None)
def compile_ir(src, flags):
    """The optimised LLVM IR of one translation unit."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "tu.ll")
        cmd = [HIPCC, *BASE, *flags, "-S", "-emit-llvm", src, "-o", out]
        r = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-2000:]
        return open(out).read()


ALL_TUS = sorted(os.path.join("csrc", f) for f in os.listdir(os.path.join(PKG, "csrc")) if f.endswith(".hip"))


@pytest.fixture(scope="module", autouse=True)
def _prewarm():
    """Every compile the module needs, in parallel, before its first test."""
    if not HAVE_HIPCC:
        return
    jobs = [(compile_asm, src, tu_flags(src)) for src in ALL_TUS] + [(compile_ir, src, tu_flags(src)) for src in ALL_TUS]
    with cf.ThreadPoolExecutor(max_workers=max(1, min(8, os.cpu_count() or 1))) as ex:
        for f in [ex.submit(fn, src, fl) for fn, src, fl in jobs]:
            f.result()


def kernel_usage(src, mangled_prefixes, extra=(), flags=None):
    """{mangled name: {vgpr, agpr, scratch, occupancy}} for every kernel whose
    mangled name starts with one of mangled_prefixes (flags: the unit's extra
    Makefile flags by default; extra: more flags, for experiments)."""
    fl = tuple(tu_flags(src) if flags is None else flags) + tuple(extra)
    _, remarks = compile_asm(src, fl)
    out, cur = {}, None
    for line in remarks.splitlines():
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


@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
@pytest.mark.parametrize("src,side", [("csrc/uwvk_psp_k.hip", 0), ("csrc/uwvk_psp_k_r.hip", 1)])
def test_psp_epoch_kernels_keep_their_occupancy(src, side):
    """53-DOF layout: 3 waves per SIMD, no scratch (LDS-bound at 12 per CU).
    26-DOF layout (the kinematic handles and, PD = 1, the parameter-decoupled
    kernel of 53-DOF handles, r06): 4 waves per SIMD (<= 128 VGPRs) with a
    bounded spill area (uwvk_psp_k.hip PSP_EPOCH_ATTR)."""
    u = kernel_usage(src, PREFIXES)
    # (2 DOFs x 3 (QM, EVS) sets + PD x 2 EVS) x {static, persistent}, all of this unit's side
    assert len(u) == 16, sorted(u)
    for name, r in u.items():
        assert name.endswith("ELi%dELi%dEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % (side, 0)) or \
            name.endswith("ELi%dELi%dEEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE" % (side, 1)), name
        regs = r["vgpr"] + r.get("agpr", 0)  # one 512-entry file per SIMD lane
        if "ILi53E" in name:
            assert regs <= 168 and r["scratch"] == 0 and r["occupancy"] >= 3, (name, r)
        else:
            assert regs <= 128 and r["occupancy"] >= 4 and r["scratch"] <= 160, (name, r)
    pd = [n for n in u if n.endswith("ELi1EEEvNS_8PoseBufsENS_10PoseSharedENS_9EpochArgsE") and "ILi26ELi1E" in n]
    assert len(pd) == 4, sorted(u)  # QM 1 x EVS {0, 1} x {static, persistent}


# The two-instances-per-wave kernel (k_psp_epoch_pair<SR, EVS, PD>, r06, the
# default of run_log's launches without pressure epochs, 53-DOF decoupled and
# 26-DOF handles): 3 waves per SIMD (<= 168
# registers; the r06g A/B measured 3 > 2 > 4 waves: 347.6 / 299.6 / 278.8 M
# steps/s at C3, 200 epochs) with a bounded spill area (180 B/lane without the
# ADCP update, 272 with it, at r06).
@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
def test_pair_kernel_keeps_three_waves_per_simd():
    u = kernel_usage("csrc/uwvk_psp_pair.hip", ("_ZN4uwvk4psp216k_psp_epoch_pairILi",))
    # SR 0 / 1 x EVS (ADCP compiled in or not) x PD (53-DOF decoupled / 26-DOF handles), persistent
    assert len(u) == 8, sorted(u)
    for name, r in u.items():
        sr, evs, pd = map(int, re.search(r"pairILi(\d)ELi(\d)ELi(\d)E", name).groups())
        regs = r["vgpr"] + r.get("agpr", 0)
        assert regs <= 168 and r["occupancy"] >= 3 and r["scratch"] <= (256 if evs else 320), (name, r)


# The BodyEfforts kernels (k_psp_efforts<DOF, VO, SR>, r05): no scratch, at
# least 2 waves per SIMD (one instance per wave, so 8 instances per CU; the
# literal two-wave kernel held 4).  Their register peak is the model
# evaluation: so3_exp_psp's library fallback inside an evaluation, or the two
# evaluations of a lane overlapped by the scheduler, took the full update to
# 512 registers with spills (psp_update_eff's comments).
@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
@pytest.mark.parametrize("src,side", [("csrc/uwvk_psp_k.hip", 0), ("csrc/uwvk_psp_k_r.hip", 1)])
def test_efforts_kernels_fit_two_waves_per_simd(src, side):
    u = kernel_usage(src, ("_ZN4uwvk3psp13k_psp_effortsILi",))
    assert len(u) == 4, sorted(u)  # DOF 53 / 26 x {full, velocity-only}
    for name, r in u.items():
        assert r["vgpr"] + r.get("agpr", 0) <= 256 and r["scratch"] == 0 and r["occupancy"] >= 2, (name, r)


# The VelocityUKF kernels: no scratch round trip per epoch.  k_vel_epoch_g (C2)
# had 272 B/lane until r04: vg_point's select chain over L[k][0..3] by the
# lane's column was turned into one lane-indexed load from a private copy of L,
# i.e. L stored to scratch and reloaded in every predict and update
# (the r04 point selection keeps the selects; C2 633-635 -> 741-745 M steps/s,
# profiles/r04/vpt/).  Since the r04 no-hoist change (+3%, profiles/r04/nh/) the kernel
# keeps 168 B/lane of loop-invariant values written once before the epoch
# loop and only read inside it; a scratch store inside the loop fails here.
@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
def test_velocity_kernels_have_no_scratch_round_trip():
    u = kernel_usage("csrc/uwvk_vel.hip", ("_ZN12_GLOBAL__N_1", "_ZN4uwvk"), flags=[])
    names = [n for n in u if "k_vel_" in n]
    assert any("k_vel_epoch_g" in n for n in names) and len(names) >= 6, sorted(u)
    for n in names:
        assert "k_vel_epoch_g" in n or u[n]["scratch"] == 0, (n, u[n])
    lines = compile_asm("csrc/uwvk_vel.hip", ())[0].split("\n")
    # the shipped k_vel_epoch_g<16>; the <32> diagnostic (UWVK_VEL_OPT_LANE_GROUPS 2)
    # is capped at 256 registers for 2 waves per SIMD and spills inside the loop
    starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\w*k_vel_epoch_gILi16E\w*:", l)]
    assert len(starts) == 1, starts
    for st in starts:
        en = [i for i, l in enumerate(lines) if i > st and l.startswith(".Lfunc_end")][0]
        body = lines[st:en]
        head = [i for i, l in enumerate(body) if "Loop Header: Depth=1" in l]
        assert len(head) == 1, head
        in_loop = [l.strip() for l in body[head[0]:] if "scratch_store" in l]
        assert not in_loop, in_loop[:5]


# A 64-bit scalar operand written as a 32-bit literal: gfx950 zero-extends it,
# so a value that is a sign-extended 32-bit number (0xffffffff8xxxxxxx ..
# 0xffffffffffffffef, not an inline constant) comes out with the upper half
# clear.  The compiler emitted exactly that for lane masks such as lanes >= 5
# (s_mov_b64 sX, 0xffffffffffffffe0; tools/probe_lmask.hip),
# so the PSP lane masks build those values from two 32-bit halves.  This scan
# keeps such an instruction out of the shipped ISA.
LIT64 = re.compile(r"^\s*(s_\w+_[biu]64)\s+(.*)$")


def sext32_literals(asm_text):
    bad = []
    for line in asm_text.splitlines():
        m = LIT64.match(line)
        if not m:
            continue
        for op in (x.strip() for x in m.group(2).split(",")):
            if not re.fullmatch(r"0x[0-9a-f]+|-?\d+", op):
                continue
            v = int(op, 16) if op.startswith("0x") else int(op)
            v &= (1 << 64) - 1
            inline = v <= 64 or v >= (1 << 64) - 16
            if not inline and v >= 0xFFFFFFFF80000000:
                bad.append(line.strip())
    return bad


def test_sext32_literal_scan_catches_the_hazard():
    assert sext32_literals("  s_mov_b64 s[4:5], 0xffffffffffffffe0\n")
    assert not sext32_literals("  s_mov_b64 s[4:5], -2\n  s_mov_b64 vcc, 0x3fffffff\n  s_movk_i32 s2, 0xffe0\n")




@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
@pytest.mark.parametrize("src", ALL_TUS)
def test_isa_has_no_zero_extended_64bit_literal(src):
    """The hazard comes from the compiler, not from the PSP code: every
    translation unit of libuwvk.so, each with its Makefile flags."""
    bad = sext32_literals(compile_asm(src, tu_flags(src))[0])
    assert not bad, bad[:10]


# Address-space casts into the constant address space (scalar loads through the
# scalar cache): valid only for a pointer whose value is a global address.  The
# r04o PSP_EA_LAUNDER variant cast the address of the by-value EpochArgs
# kernel parameter: the escaping address made clang copy the parameter into a
# private alloca (addrspace 5), and `addrspacecast addrspace(5) -> addrspace(4)`
# (private -> constant, disjoint non-flat spaces) is lowered to an undefined
# SGPR pair: the first scalar load through it, s_load_dword s0, s[64:65], 0x298
# (ea.first), read a garbage address and the kernel faulted (UWVK_EDEVICE,
# profiles/EXPERIMENTS.md "r05: the r04o device fault"; tools/eal_variant.py
# rebuilds the variant).  The shipped casts (PoseShared, Qp) start from global
# pointer values loaded from PoseBufs.  This scan keeps private -> constant /
# global casts and private copies of the kernel-argument structs out of the IR.
def ir_cast_findings(ir):
    bad = []
    for line in ir.splitlines():
        if re.search(r"addrspacecast ptr addrspace\(5\) \S+ to ptr addrspace\((1|4)\)", line):
            bad.append(line.strip())
        if re.search(r'alloca %"struct\.uwvk::(EpochArgs|PoseShared|PoseBufs|MeasArgs)"', line):
            bad.append(line.strip())
    return bad


def test_ir_cast_scan_catches_the_r04o_pattern():
    assert ir_cast_findings('  %6 = alloca %"struct.uwvk::EpochArgs", align 8, addrspace(5)\n')
    assert ir_cast_findings("  %467 = addrspacecast ptr addrspace(5) %6 to ptr addrspace(4)\n")
    assert not ir_cast_findings("  %717 = addrspacecast ptr %24 to ptr addrspace(4)\n")


@pytest.mark.skipif(not HAVE_HIPCC, reason="no hipcc")
@pytest.mark.parametrize("src", ALL_TUS)
def test_no_private_to_constant_address_space_cast(src):
    bad = ir_cast_findings(compile_ir(src, tu_flags(src)))
    assert not bad, bad[:10]
