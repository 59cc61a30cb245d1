#!/usr/bin/env python3
"""bench.py — batched PoseUKF predict+update throughput on MI355X.

Metric (BASELINE.json): UKF predict+update steps/sec at batch = 65536 PoseUKF
instances (config C3: full 53-DOF PoseState, 1 kHz IMU + 5 Hz DVL) on 1 GPU,
and 1,048,576 instances on 8 GPUs (config C5: 131,072 per GPU, RCCL
all-reduce of the ensemble statistics).  One "step" = one IMU epoch of ONE
filter instance: RotationRate store -> predictionStep(1 ms) -> Acceleration
update, plus the DVL velocity update when the 5 Hz schedule is due
(SURVEY.md §3, §8d).  `value` counts instance-epochs per second over the whole
job (all ranks).

Multi-GPU: one process per GPU.  `python3 bench.py --gpus N` starts the N rank
processes itself (subprocesses, before any GPU call in the parent); under
`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N` the
launcher's ranks are used (and --gpus must equal WORLD_SIZE).  Instances are
sharded contiguously (weak scaling: --batch-per-gpu instances on every GPU, no
data-path collective); the engine's RCCL communicator exists for the whole run
and sums the ensemble statistics every --stats-every epochs and at the end of
the timed region, inside it (C5).  A gloo process group is the host control
plane (barriers, the RCCL id, the max of the per-rank times).

Inputs are synthetic (uwvk.synth) and resident in HBM before timing starts.
Timing: barrier + device sync on both sides of the timed region, max over
ranks; the dominant kernel's average launch time comes from HIP events on the
handle's stream.  cpu_baseline: the fp64 C oracle (oracle/, "port") on a
bounded sample of the same workload, on rank 0 at N = 1 only.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))

METRIC = "UKF predict+update steps/sec at batch=65536 PoseUKF instances, 1 & 8 GPU"
# frozen algorithmic work per step: n = 53, N = 107
F_PRED = 700_377
F_UPD3 = 853_707
F_STEP = F_PRED + F_UPD3  # 1,554,084 flop: predict + Acceleration update (m = 3), reference algorithm
# flops the engine executes per m = 3 update: apply_delta is the exact rotation
# identity instead of a second LLT + sigma-point GEMM
F_UPD3_EXEC = 155_237
F_STEP_EXEC = F_PRED + F_UPD3_EXEC  # 855,614 (literal kernels, UWVK_OPT_DENSE_SIGMA)


def _pchol_flops(n, k):
    """k-column partial Cholesky of an n x n matrix: the column scales, the
    trailing updates of the panel's columns (c > J, rows >= c) and one
    reciprocal square root + product per pivot."""
    return sum((n - j - 1) + sum(2 * (n - c) for c in range(j + 1, k)) for j in range(k)) + 2 * k


def psp_flops_phases(n=53, k_pred=15, updates=((6, 3, 7),)):
    """Useful flops of one PSP step by phase: the operation
    count of the algorithm, whatever the lane mapping.  Per-point costs are
    counted from the models' code (uwvk_psp_dev.hpp): a sigma point's
    orientation through the process model 215 flop (generation 14, SO3 exp 38
    and product 28 twice, latitude series 28, q-rotation 30, rest 13); a
    manifold-mean term 64 (SO3 product 28, small-angle log 30, weighted sum 6);
    an acceleration / DVL point 132 (generation 14, SO3 exp 38, product 28,
    rotation matrix 30, R^T(a + g) 22).  updates: (k, m, ncols) per update."""
    kp, N2 = k_pred, 2 * k_pred + 1
    npk = n * (n + 1) // 2
    ph = {}
    ph["predict partial Cholesky + R Q_o R^T"] = _pchol_flops(n, kp) + 138
    ph["predict points, mean, deviations, ori x ori, X"] = (N2 * 215 + (N2 * 64 + 70)   # points, 1 mean iteration
                                                          + N2 * 58 + N2 * 12 + 12 + 3 * kp  # deviations, ori x ori, Delta
                                                          + 2 * n * 3 * kp + 9 * n)          # X = 1/2 A L_a Delta
    ph["predict covariance rows (A-coupled, Q' band, mean)"] = 6 * n * 7 + 9 * n + 9 * n + 2 * (n + 1)
    for i, (k, m, nc) in enumerate(updates):
        tag = "update %d (k %d, m %d)" % (i, k, m)
        ph[tag + " partial Cholesky"] = _pchol_flops(n, k)
        ph[tag + " points, zbar, S"] = (2 * k + 1) * (132 if m == 3 else 80) + (2 * k + 1) * (m + m * (m + 1))
        ph[tag + " H, P, G, C, S, gain"] = (30 + 2 * m * k * nc + 2 * n * nc * m + n * m + 2 * 2 * n * k * m
                                            + n * m + 2 * m * m * nc + 40 + 2 * n * m * m + 24 + 2 * n * m)
        ph[tag + " Sigma -= C K^T"] = 2 * npk * m + 2 * n * m
        ph[tag + " apply_delta"] = 38 + 30 + 15 * (n - 3) + 108 + 28 + (n + 1)
    return ph


def psp_flops(n=53, k_pred=15, updates=((6, 3, 7),)):
    """Flops the PSP kernels execute per step (DESIGN.md sections 4.3, 6.1): the
    sum of psp_flops_phases."""
    return sum(psp_flops_phases(n, k_pred, updates).values())


F_STEP_PSP = psp_flops()
F_UPD3_PSP = psp_flops(updates=((6, 3, 7), (6, 3, 3))) - F_STEP_PSP  # one DVL update
# the parameter-decoupled kernel (UWVK_OPT_PARAM_BLOCK): the
# 26-DOF layout's PSP step plus the 27 parameters alone (time scale 2 + its
# reciprocal with two Newton steps 8, dt^2 Q band 3, mean decay 3 per epoch):
# the work it executes, not the 53-DOF algebra's zeros
F_PD_PARAMS = 27 * 16
F_STEP_PSP_PD = psp_flops(26) + F_PD_PARAMS
F_UPD3_PSP_PD = psp_flops(26, updates=((6, 3, 7), (6, 3, 3))) - psp_flops(26)
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 (vector = matrix) spec; probe measured 74 (profiles/r01_probe_fp64.txt)
PEAK_HBM_GBS = 8000.0


# VelocityUKF (config C2) work per step, frozen from the kernel's code
# (uwvk_vel.hip v_deriv / v_rk4), an FMA counted as 2.  One derivative
# evaluation of the Fossen model: the kinematics (position rotation 30,
# quaternion rate 32) ~60, Coriolis 102, linear + quadratic damping 186, the
# restoring forces 42 (VEL_GLIN: with r = R^T e_z, -(f_g + f_b) = (W - B) r and
# -(cog x f_g + cob x f_b) = (W cog - B cob) x r, one rotation + one cross
# product), tau - C - D - g 18, M^-1 72: ~485 flop; an RK4 step = 4 of them +
# the stage sums and normalisation ~170 = 2,110 flop.  A predict integrates the
# 9 sigma points and the side model (10 RK4) plus ~900 flop of 4-DOF UKF
# algebra; DVL (5 Hz) and pressure (10 Hz) updates add ~20 flop per step on
# average.  The reference's own formulation (two rotations and two cross
# products for the restoring forces, ModelSimulation [EXT]) is 90 flop per
# derivative, 2,290 per RK4: reported beside the executed figure.
F_VEL_RK4 = 2_110
F_VEL_RK4_REF = 2_290
F_VEL_STEP = 10 * F_VEL_RK4 + 900 + 20          # 22,020: what k_vel_epoch_g executes
F_VEL_STEP_REF = 10 * F_VEL_RK4_REF + 900 + 20  # 23,820: the reference's formulation


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed epochs")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=0,
                    help="0: 65536 (C3/C4 at N = 1), 131072 (C5: N > 1), 4096 (C2)")
    ap.add_argument("--dof", type=int, default=53)
    ap.add_argument("--mode", default="auto", choices=["auto", "C1", "C2", "C3", "C4", "C5"],
                    help="auto: C3 at N = 1 (headline), C5 at N > 1; C4: ADCP + drop-outs; C2: VelocityUKF; "
                         "C1: one PoseUKF on one CPU core (the oracle's timing build, no GPU)")
    ap.add_argument("--stats-every", type=int, default=1000,
                    help="epochs between ensemble-statistics all-reduces inside the timed region (C5: 1000); "
                         "one more at its end")
    ap.add_argument("--segment-epochs", type=int, default=0,
                    help="generate + upload the log in segments of this many epochs, outside the timed region "
                         "(0: automatic when the IMU log of the whole run exceeds 24 GiB, e.g. C4's full "
                         "40,000-epoch drop-out cycle)")
    ap.add_argument("--c4-cycle", default="30,10",
                    help="C4 DVL drop-out cycle 'on,off' in s; e.g. 0.3,0.1 keeps every event rate of the 30/10 "
                         "cycle (0.25%% efforts epochs) inside a 2000-epoch window")
    ap.add_argument("--vel-groups", type=int, default=-1, help="C2: -1 auto, 0 lane per filter, 1 16-lane rows, 2 16-lane rows each run twice "
                         "in a 32-lane group (diagnostic: twice the waves, same work per wave)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dense", action="store_true", help="literal kernels (all 2n+1 sigma points)")
    ap.add_argument("--so3-left", action="store_true",
                    help="UWVK_OPT_SO3_RIGHT = 0: the nav-frame SO3 boxplus exp(d) q instead of the default body-frame "
                         "q exp(d) (MTK's SO3::boxplus); the PSP kernels' SR = 0 instantiations (DESIGN.md 4.3)")
    ap.add_argument("--tail-chunks", type=int, default=0,
                    help="UWVK_OPT_TAIL_CHUNKS (diagnostic A/B): force this many chunks per tail instance, 0 = planner")
    ap.add_argument("--persist", type=int, default=-1,
                    help="UWVK_OPT_PERSIST: 1 persistent workgroups taking work units from a ticket counter, "
                         "0 one workgroup per instance, -1 the engine default")
    ap.add_argument("--param-block", type=int, default=-1,
                    help="UWVK_OPT_PARAM_BLOCK: -1 the engine's default (on), 0 always the general 53-DOF kernel, "
                         "1 the parameter-decoupled kernel while the model-parameter block is uncoupled")
    ap.add_argument("--pair", type=int, default=-1,
                    help="UWVK_OPT_PAIR: -1 the engine's default, 1 the parameter-decoupled kernel with two "
                         "instances per wave, 0 one per wave")
    ap.add_argument("--tail-slots", type=int, default=0,
                    help="UWVK_OPT_TAIL_SLOTS: 0 runtime occupancy, > 0 blocks per XCD, < 0 no tail spreading")
    ap.add_argument("--lds-pad", type=int, default=0,
                    help="UWVK_OPT_LDS_PAD (diagnostic): unused dynamic LDS bytes per PSP epoch workgroup, lowering "
                         "its occupancy (use with --tail-slots -1)")
    ap.add_argument("--config", default="",
                    help="YAML / JSON filter configuration (uwvk.config: PoseUKFConfig, UWVParameters, engine "
                         "options) instead of the synthetic defaults; the line names it in config.config_file")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core available to this process")
    ap.add_argument("--init", default="mc", choices=["mc", "config"],
                    help="mc: Monte-Carlo start drawn around the truth from priors small enough for a consistent "
                         "filter (uwvk.synth.mc_start, second constructor); config: the first constructor's prior "
                         "(v = 0 against a 1 m/s truth: ensemble NEES ~37 instead of 9, DESIGN.md section 8)")
    return ap.parse_args()


def window_shift(warmup, steps):
    """Epochs run before the warm-up so that the 5 Hz DVL schedule puts at least
    one DVL epoch inside the timed window (exactly the 1-in-200 rate when
    steps >= 200): a DVL epoch (k % 200 == 0) lands mid-window."""
    target = warmup + min(steps, 200) // 2
    shift = (200 - (target + 1) % 200) % 200
    # diagnostic only (never the headline): UWVK_BENCH_WINDOW_OFFSET moves the window
    # off the DVL epoch (100: no DVL update in a window of < 100 epochs); the line
    # reports dvl_epochs_in_window either way
    return shift + int(os.environ.get("UWVK_BENCH_WINDOW_OFFSET", "0"))


def dvl_aligned_log(synth, batch, warmup, steps, mode, dof, first_instance, c4_cycle=(30.0, 10.0), cfg=None,
                    epoch0=0, epochs=None):
    """Log of shift + warmup + steps epochs (window_shift), or its segment
    [epoch0, epoch0 + epochs) (synth.make_pose_log epoch0: a bitwise slice)."""
    shift = window_shift(warmup, steps)
    total = shift + warmup + steps
    n = total - epoch0 if epochs is None else epochs
    log = synth.make_pose_log(batch, n, mode=mode, dof=dof, first_instance=first_instance,
                              dropout_on=c4_cycle[0], dropout_off=c4_cycle[1], cfg=cfg, epoch0=epoch0)
    return log, shift


# host + device bytes of the IMU part of a log per instance-epoch (gyro + acc, fp64):
# above SEGMENT_AUTO_BYTES the window is generated and uploaded in segments
LOG_BYTES_PER_INSTANCE_EPOCH = 48
SEGMENT_AUTO_BYTES = 24 << 30


def timed_run(f, dlog, base, e_from, e_to, cut_abs, reduce_stats, truth, dof, barrier):
    """One timed region: absolute epochs [e_from, e_to) of a device log whose
    epoch 0 is absolute epoch `base`, the ensemble statistics reduced at the
    absolute epochs of cut_abs inside (e_from, e_to].  Barrier + device sync on
    both sides; HIP events on the handle's stream around the epoch launches.
    Returns (wall_s, kernel_ms, last statistics or None, run_log calls)."""
    pts = sorted({c for c in cut_abs if e_from < c <= e_to} | {e_to})
    barrier()
    f.synchronize()
    t0 = time.perf_counter()
    f.timer_start()
    prev, stats = e_from, None
    for k, c in enumerate(pts):
        f.run_log(dlog, prev - base, c - prev, sync=False)
        if k == len(pts) - 1:
            f.timer_mark()  # HIP events on the handle's stream around the epoch launches (no host wait)
        if c in cut_abs:
            stats = reduce_stats(truth.state(c, dof))  # synchronous
        prev = c
    f.synchronize()
    barrier()
    return time.perf_counter() - t0, f.timer_elapsed(), stats, len(pts)


def pmc_entry(workload, steps=None):
    """The committed rocprofv3 PMC summary of this workload's kernel for a
    launch of `steps` epochs (profiles/pmc_traffic.json, key WORKLOAD-eSTEPS),
    else the workload's default shape (or {})."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    if steps is not None and ("%s-e%d" % (workload, steps)) in d:
        return d["%s-e%d" % (workload, steps)]
    return d.get(workload) or {}


def counter_roofline(e, waves, epochs, kernel_ms):
    """Executed-work roofline of the timed launch from the committed PMC passes
    (profiles/pmc_traffic.json): fp64 VALU instructions per wave-epoch
    (SQ_INSTS_VALU_{FMA,MUL,ADD}_F64) x 64 lanes x (2 for an FMA, 1 otherwise),
    scaled to this launch's waves x epochs, over the live HIP-event kernel time.
    The counters count issued instructions whatever the exec mask, so these are
    lane-slot flops (an upper bound of the useful work; SQ_THREAD_CYCLES_VALU /
    SQ_ACTIVE_INST_VALU gives the active-lane share).  None without the passes."""
    pw = e.get("per_wave_epoch") or {}
    if not {"valu_fma_f64", "valu_mul_f64", "valu_add_f64"} <= set(pw):
        return None
    lane_flop = 64 * (2 * pw["valu_fma_f64"] + pw["valu_mul_f64"] + pw["valu_add_f64"])
    # f64 MFMA work (the update's rank-M tiles, r03): SQ_INSTS_VALU_MFMA_MOPS_F64 x 512,
    # executed on the same fp64 pipe, so it adds to the VALU figure (0 without the pass)
    mfma_flop = (e.get("mfma") or {}).get("flop_per_wave_epoch", 0.0)
    out = {"fp64_lane_flop_per_wave_epoch": lane_flop, "fp64_mfma_flop_per_wave_epoch": mfma_flop,
           "achieved_tflops": (lane_flop + mfma_flop) * waves * epochs / (kernel_ms * 1e-3) / 1e12,
           "epochs_profiled": e.get("epochs_per_launch"), "source": e.get("valu_source")}
    lanes = (e.get("active_lanes") or {}).get("thread_cycles_per_valu_quad_cycle")
    if lanes:  # VALU lane-slots scaled by the active-lane share; MFMA tiles count whole
        out["active_tflops"] = (lane_flop * lanes / 64.0 + mfma_flop) * waves * epochs / (kernel_ms * 1e-3) / 1e12
    for k in ("valu_busy", "active_lanes", "mfma"):
        if k in e:
            out[k] = e[k]
    return out


def initialise(f, log, cfg, uwv, init, first_instance=0):
    """Both constructors of the reference (PoseUKF.cpp:288-391) on an engine
    handle or an oracle batch: `config` is the first (prior from the config),
    `mc` the Monte-Carlo start (uwvk.synth.mc_start) through the second."""
    from uwvk import abi, synth
    if init == "config":
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        return
    rot0, rot_cov = synth.mc_rotation(log, first_instance=first_instance)
    f.init_from_config(log["pos0"], log["pos_cov"], rot0, rot_cov, cfg, uwv)
    x, P = f.get_state()
    x, P = synth.mc_start(x, P, log, first_instance=first_instance)
    loc = abi.Location(cfg.location.latitude, cfg.location.longitude, cfg.location.altitude)
    f.init_from_state(x, P, loc, uwv, synth.pose_parameter(cfg))
    del x, P


def cpu_baseline(synth, cfg, uwv, mode, dof, threads, init="mc", right=True):
    """The fp64 C oracle's timing build (oracle/liboracle_fast.so: -O3,
    x86-64-v4, one instance per task, pthreads) on a bounded sample of the same
    workload, on every core this process may use; plus one instance on one
    core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as O
    if right is not None:  # the oracle's switch is process-wide (both builds): the whole sample on that side
        with O.so3_side(right):
            return cpu_baseline(synth, cfg, uwv, mode, dof, threads, init, right=None)
    epochs = 2000
    # single core first: it sizes the multi-core sample to ~15 s of wall time
    log1 = synth.make_pose_log(1, epochs, mode=mode, dof=dof, cfg=cfg)
    o1 = O.OraclePoseBatch(1, dof, timing=True)
    initialise(o1, log1, cfg, uwv, init)
    o1.set_process_noise_from_config(cfg, log1["dt"])
    t1 = time.perf_counter()
    o1.run_log(log1, nthreads=1)
    dt1 = time.perf_counter() - t1
    rate1 = epochs / dt1
    per_thread = max(1, int(round(15.0 * rate1 / epochs)))
    batch = per_thread * threads
    log = synth.make_pose_log(batch, epochs, mode=mode, dof=dof, cfg=cfg)
    o = O.OraclePoseBatch(batch, dof, timing=True)
    initialise(o, log, cfg, uwv, init)
    o.set_process_noise_from_config(cfg, log["dt"])
    t0 = time.perf_counter()
    o.run_log(log, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": batch * epochs / dt, "unit": "steps/s", "cores": threads, "kind": "port",
            "algorithm": "literal ukfom (all 2n+1 sigma points: LLT, 107 model evaluations, iterative manifold "
                         "mean, covariance GEMM, literal apply_delta re-spread); the GPU runs PSP, an exact O(n^2) "
                         "reformulation (DESIGN.md 4.3) with ~3.4% of those flops, so the GPU/CPU ratio mixes an "
                         "algorithmic gain (~30x) with the hardware gain",
            "sample": "%d PoseUKF instances x %d epochs (%s, incl. %d DVL updates each), %d pthreads, %.2f s wall; "
                      "oracle timing build -O3 -march=x86-64-v4" % (batch, epochs, mode,
                                                                   int(((log["flags"] & 2) != 0).sum()), threads, dt),
            "single_core": {"value": rate1, "unit": "steps/s", "cores": 1,
                            "sample": "1 PoseUKF instance x %d epochs, %.2f s" % (epochs, dt1)},
            "host": {"cpu": _cpu_model(), "logical_cpus": os.cpu_count(), "available_to_job": threads}}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def available_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup v2
    CPU quota when one is set (the GPU box shares its host)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(per))))
    except (OSError, ValueError):
        pass
    return n


def launched_by_torchrun():
    return "TORCHELASTIC_RUN_ID" in os.environ or ("LOCAL_RANK" in os.environ and "WORLD_SIZE" in os.environ)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def rank_env(base, rank, world, port):
    """Environment of rank `rank` of a self-launched N-rank job."""
    env = dict(base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), UWVK_BENCH_SPAWNED="1")
    return env


def spawn_ranks(argv, world, timeout=None, script=None):
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (subprocesses, never an exec; the parent makes no GPU call) and
    return the worst exit code.  If a rank fails, the others are stopped
    (their exact PIDs) instead of waiting at a barrier forever."""
    port = _free_port()
    script = script or os.path.abspath(__file__)
    procs = [subprocess.Popen([sys.executable, script] + list(argv),
                              env=rank_env(os.environ, r, world, port)) for r in range(world)]
    t0 = time.time()
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = rc or code
                for q in procs:
                    q.terminate()
        if timeout is not None and time.time() - t0 > timeout:
            for q in procs:
                q.kill()
            rc = rc or 124
            break
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def resolve_world(a, env=os.environ):
    """(world, rank, local) of this process; raises SystemExit when --gpus and
    a launcher's WORLD_SIZE disagree."""
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if a.gpus != world:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (the launcher's rank count); pass --gpus %d"
                             % (a.gpus, world, world))
        return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
    return 1, 0, 0


def workload_of(a, world):
    """(mode, batch per GPU): C3 at N = 1, C5 (131,072 per GPU) at N > 1."""
    mode = a.mode if a.mode != "auto" else ("C3" if world == 1 else "C5")
    if a.batch_per_gpu:
        return mode, a.batch_per_gpu
    return mode, {"C2": 4096, "C5": 131072}.get(mode, 65536)


def init_dist(world):
    """The host control plane of a multi-rank job (gloo): barriers, the RCCL
    id, the max of the per-rank times.  None for a single-process run."""
    if world == 1 and not launched_by_torchrun():
        return None
    import torch.distributed as dist
    # gloo prints its connection report on stdout, where the driver reads the
    # one JSON line: send file descriptor 1 to stderr while the group forms
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    return dist


def make_rccl(dist, engine, world, rank, local):
    """The engine's RCCL communicator (rank 0's id broadcast over gloo), or
    (None, reason) on every rank when any rank failed to make it: the ranks
    agree through a gloo MIN, so a failure everywhere (an RCCL that cannot run
    on the node) falls back to the gloo sum and says so in the line, instead of
    ending the run."""
    import torch
    err = None
    uid = [None]
    if rank == 0:
        try:
            uid[0] = engine.RcclComm.unique_id()
        except Exception as e:  # noqa: BLE001 (reported in the line)
            err = "unique_id: %s" % e
    dist.broadcast_object_list(uid, src=0)
    comm = None
    if uid[0] is not None:
        try:
            comm = engine.RcclComm(world, uid[0], rank, local)
        except Exception as e:  # noqa: BLE001
            err = "comm_init on rank %d: %s" % (rank, e)
    ok = torch.tensor([0 if comm is None else 1], dtype=torch.int32)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok[0]) == 1:
        return comm, None
    if comm is not None:
        comm.close()
    err = err or "another rank could not make it"
    print("warning: RCCL communicator unavailable (%s); the statistics are summed over gloo" % err, file=sys.stderr)
    return None, err


def collective_desc(dist, world, comm, comm_err, same_dev):
    """config.collective of the bench line: which all-reduce summed the
    ensemble statistics (None for a single-process run)."""
    if world == 1:
        c = os.environ.get("UWVK_BENCH_COLL", "")
        return {"rccl1": "one-rank RCCL communicator through the timed region (N = 1 rehearsal)",
                "scoped": "one-rank RCCL communicator made around each statistics all-reduce (N = 1 rehearsal)"}.get(c)
    if dist is None:
        return None
    if comm is not None:
        return "RCCL all_reduce of the ensemble statistics on the handle's stream (uwvk_pose_ensemble_allreduce)"
    if comm_err is not None:
        return "gloo all_reduce of the ensemble statistics (host): the RCCL communicator failed (%s)" % comm_err
    return "gloo all_reduce of the ensemble statistics (host)%s" % (
        ": RCCL refuses two ranks on one GPU (UWVK_BENCH_SAME_DEVICE rehearsal)" if same_dev else "")


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(sys.argv[1:], a.gpus))
    if a.mode == "C1":
        return bench_c1(a)
    world, rank, local = resolve_world(a)
    # UWVK_BENCH_SAME_DEVICE=1: rehearsal of the N-rank path on one GPU (all ranks on device 0)
    same_dev = os.environ.get("UWVK_BENCH_SAME_DEVICE") == "1"
    if same_dev:
        local = 0
    dist = init_dist(world)
    from uwvk import engine, ensemble, synth
    mode, B = workload_of(a, world)
    if mode == "C2":
        return bench_vel(a, engine, synth, world, rank, local, dist, B)
    log_mode = "C3" if mode == "C5" else mode
    cfg, uwv, eng_opts = synth.default_pose_config(), synth.default_uwv(), {}
    if a.config:
        from uwvk import config as uconfig
        fc = uconfig.load(a.config)
        cfg, uwv, eng_opts = fc.pose, fc.uwv, fc.engine
        # the file's engine options win over the command line (config.apply_engine_options);
        # mirror them into the arguments, which name the kernel, the flop model and the
        # CPU baseline's side
        if "so3_right" in eng_opts:
            if a.so3_left and eng_opts["so3_right"]:
                print("warning: --so3-left overridden by %s (engine.so3_right: true)" % a.config, file=sys.stderr)
            a.so3_left = not eng_opts["so3_right"]
        if eng_opts.get("dense_sigma") or eng_opts.get("literal_apply_delta"):
            a.dense = True  # either option switches the handle to the literal kernels (use_dense)
        a.literal_apply_delta = bool(eng_opts.get("literal_apply_delta"))
        for k, flag in (("tail_slots", "tail_slots"), ("persist", "persist")):
            if k in eng_opts and getattr(a, flag) != eng_opts[k] and getattr(a, flag) not in (0, -1):
                print("warning: --%s %s overridden by %s (engine.%s: %s)" % (flag.replace("_", "-"), getattr(a, flag),
                                                                             a.config, k, eng_opts[k]), file=sys.stderr)
    cyc = tuple(float(v) for v in a.c4_cycle.split(","))
    shift = window_shift(a.warmup, a.steps)
    total = shift + a.warmup + a.steps
    e0 = shift + a.warmup
    seg = a.segment_epochs
    if seg == 0 and B * total * LOG_BYTES_PER_INSTANCE_EPOCH > SEGMENT_AUTO_BYTES:
        seg = 4000
    seg = seg if 0 < seg < total else 0
    seg_bounds = [(s0, min(total, s0 + seg)) for s0 in range(0, total, seg)] if seg else [(0, total)]
    log, _ = dvl_aligned_log(synth, B, a.warmup, a.steps, log_mode, a.dof, first_instance=rank * B, c4_cycle=cyc,
                             cfg=cfg, epochs=seg_bounds[0][1])
    f = engine.PoseUKFBatch(B, a.dof, device=local)
    f.set_tail_slots(a.tail_slots)
    if a.lds_pad:
        f.set_lds_pad(a.lds_pad)
    if a.persist >= 0:
        f.set_persist(a.persist)
    if a.param_block >= 0:
        f.set_param_block(a.param_block)
    if a.pair >= 0:
        f.set_pair(a.pair)
    if a.tail_chunks:
        f.set_tail_chunks(a.tail_chunks)
    if a.dense:
        f.set_dense_sigma(True)
    if eng_opts:
        uconfig.apply_engine_options(f, eng_opts)
    f.set_so3_right(not a.so3_left)
    initialise(f, log, cfg, uwv, a.init, first_instance=rank * B)
    f.set_process_noise_from_config(cfg, log["dt"])
    # The collective (C5): the per-rank ensemble statistics summed over the
    # engine's RCCL communicator on the handle's stream (uwvk_pose_ensemble_
    # allreduce), every --stats-every epochs and at the end of the window.  The
    # communicator is made before the timed region and lives through it (made
    # around each all-reduce, its set-up would be ~0.6 s of the window; a live
    # one-rank communicator no longer slows the epoch kernel, r06zh, DESIGN.md
    # section 8).  RCCL refuses two ranks on one
    # GPU, so the one-GPU rehearsal (UWVK_BENCH_SAME_DEVICE) sums over gloo;
    # UWVK_BENCH_COLL=host does the same on purpose (A/B).
    # One-GPU measurements of the communicator's cost at
    # N = 1: UWVK_BENCH_COLL=rccl1 makes a one-rank communicator before the
    # timed region and sums through it (the N > 1 lifetime); =scoped makes it
    # around each statistics all-reduce and destroys it after (its set-up
    # inside the timed region).
    coll_env = os.environ.get("UWVK_BENCH_COLL", "")
    coll = "host" if (same_dev or coll_env == "host") else "rccl"
    comm, comm_err = None, None
    if dist is not None and world > 1 and coll == "rccl":
        comm, comm_err = make_rccl(dist, engine, world, rank, local)
    if world == 1 and coll_env == "rccl1":
        comm = engine.RcclComm(1, engine.RcclComm.unique_id(), 0, local)
    scoped = world == 1 and coll_env == "scoped"

    def reduce_stats(truth):
        if scoped:
            c1 = engine.RcclComm(1, engine.RcclComm.unique_id(), 0, local)
            try:
                return f.ensemble_stats(truth, c1)
            finally:
                c1.close()
        st = f.ensemble_stats(truth, comm)
        if dist is not None and world > 1 and comm is None:
            st = ensemble.allreduce_stats(st, dist)
        return st

    def barrier():
        if dist is not None:
            dist.barrier()

    # statistics points inside the window: every --stats-every epochs, and its end
    every = max(1, a.stats_every)
    cuts = sorted({min(a.steps, k) for k in range(every, a.steps, every)} | {a.steps})
    cut_abs = {e0 + c for c in cuts}
    # Segments (a window whose log does not fit host / device memory at once, e.g.
    # C4's full 40,000-epoch drop-out cycle): each segment's inputs are generated
    # and uploaded outside the timed region (bitwise slices of the whole log), the
    # filter state stays on the device, and the window's time is the sum of the
    # segments' timed runs.  Without segments this is one timed region.
    wall, kernel_ms, stats, pieces, windows = 0.0, 0.0, None, 0, []
    truth = log["truth"]
    pd_window = None  # the parameter-decoupled kernel at the window's start (UWVK_OPT_PARAM_BLOCK)
    pair_window = False  # ... in its two-instances-per-wave form (UWVK_OPT_PAIR)
    for si, (s0, s1) in enumerate(seg_bounds):
        if seg:
            print("segment %d/%d: epochs [%d, %d)" % (si + 1, len(seg_bounds), s0, s1), file=sys.stderr, flush=True)
        if si:
            del dlog
            log, _ = dvl_aligned_log(synth, B, a.warmup, a.steps, log_mode, a.dof, first_instance=rank * B,
                                     c4_cycle=cyc, cfg=cfg, epoch0=s0, epochs=s1 - s0)
            truth = log["truth"]
        dlog = f.upload_log(log)
        if si == 0:
            # warm the statistics kernels and the collective (module load, RCCL
            # channel set-up) outside the timed region, ahead of the untimed
            # epochs (its values are discarded)
            reduce_stats(truth.state(s0, a.dof))
        if s0 < e0:  # the alignment shift and the warm-up (untimed)
            # in launches of the timed window's length, the remainder first, so
            # that a kernel-trace summary of the command (rocprofv3 --stats)
            # averages launches of the timed shape and the launch right before
            # the window is one of them (the same epochs either way)
            pre = min(s1, e0) - s0
            n = max(1, a.steps)
            p0 = 0
            if pre % n:
                f.run_log(dlog, 0, pre % n)
                p0 = pre % n
            for q in range(p0, pre, n):
                f.run_log(dlog, q, min(n, pre - q))
        lo = max(s0, e0)
        if lo < s1:
            if pd_window is None:
                pd_window = bool(f.param_block()) and not a.dense
                pair_window = bool(f.pair_active()) and not a.dense
            windows.append(log["flags"][lo - s0:])
            w_s, k_ms, st, n = timed_run(f, dlog, s0, lo, s1, cut_abs, reduce_stats, truth, a.dof, barrier)
            wall, kernel_ms, pieces = wall + w_s, kernel_ms + k_ms, pieces + n
            stats = st if st is not None else stats
    window = np.concatenate(windows)
    assert len(window) == a.steps
    n_dvl = int(((window & 2) != 0).sum())
    if dist is not None:
        import torch
        w = torch.tensor([wall, kernel_ms], dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall, kernel_ms = float(w[0]), float(w[1])
    # untimed check of the collective: the RCCL sum equals the gloo sum of the
    # per-rank statistics (same fixed-order kernel sums on every rank)
    coll_check = None
    if dist is not None and world > 1:
        local_st = f.ensemble_stats(truth.state(e0 + a.steps, a.dof))
        host_sum = ensemble.allreduce_stats(local_st, dist)
        # the two sums add the same per-rank values in different orders: they
        # agree to world x eps x the sum of the magnitudes (elementwise), which
        # also covers components whose total nearly cancels
        mag = ensemble.allreduce_stats(np.abs(local_st), dist)
        coll_check = bool(np.all(np.abs(host_sum - stats) <= 4.0 * world * np.finfo(np.float64).eps * mag + 1e-300))
        if not coll_check:
            print("error: the all-reduced ensemble statistics differ from the host sum", file=sys.stderr)
    status = f.get_status()
    if status.any():
        print("warning: %d instances flagged (status bits)" % int((status != 0).sum()), file=sys.stderr)

    steps_total = B * world * a.steps
    value = steps_total / wall
    # launches in the timed window: the PSP path runs each statistics interval
    # in one k_psp_epoch launch (efforts epochs split it); the literal path one per epoch
    n_eff = int(((window & 0x10) != 0).sum())
    launches = a.steps if a.dense else pieces + 2 * n_eff
    per_launch_ms = kernel_ms / launches
    # reference-equivalent work (the literal ukfom algorithm)
    flops_ref = B * (F_STEP * a.steps + F_UPD3 * n_dvl)
    # the engine's own flop model: the useful work it does
    lad = getattr(a, "literal_apply_delta", False)  # the literal re-spread: the reference's own flops
    step_model, upd_model = ((F_STEP, F_UPD3) if lad else (F_STEP_EXEC, F_UPD3_EXEC)) if a.dense \
        else ((F_STEP_PSP_PD, F_UPD3_PSP_PD) if pd_window else (F_STEP_PSP, F_UPD3_PSP))
    flops_model = B * (step_model * a.steps + upd_model * n_dvl)
    eff_tf = flops_ref / (kernel_ms * 1e-3) / 1e12
    model_tf = flops_model / (kernel_ms * 1e-3) / 1e12
    # the PSP instantiation run (uwvk_psp_k.hip launch_epoch_dof): Q shape, and
    # 1 when the window holds no pressure / ADCP epoch (0x4 | 0x8)
    evs = 0 if (f.epoch_qshape() != 1 or bool(((window & 0xC) != 0).any())) else 1
    sr = 0 if a.so3_left else 1
    persist = a.persist if a.persist >= 0 else 1  # the engine's default scheduler (UWVK_OPT_PERSIST)
    kfam = "k_psp_epoch_p" if persist else "k_psp_epoch"
    if a.dense:
        kname = "k_pose_epoch<%d>" % a.dof
    elif pair_window:  # two instances per wave (uwvk_psp_pair.hip)
        # EVS 0 (the ADCP update compiled in) when an ADCP epoch falls outside the pressure epochs
        adcp_in_pair = bool((((window & 0x8) != 0) & ((window & 0x4) == 0)).any())
        kname = "k_psp_epoch_pair<%d, %d, %d> (%s, 2 instances per wave)" % (
            sr, 0 if adcp_in_pair else 1, 1 if pd_window else 0,
            "53-DOF state, parameter-decoupled" if pd_window else "26-DOF state")
        if bool(((window & 0x4) != 0).any()):  # run_log's split around the pressure epochs
            kname += "; pressure epochs on %s<26, %d, 0, %d, %d>" % (kfam, f.epoch_qshape(), sr, 1 if pd_window else 0)
        if pd_window and bool(((window & 0x10) != 0).any()):
            kname += "; after the first full BodyEfforts epoch the general 53-DOF kernel"
    elif pd_window:  # 53-DOF state on the 26-DOF layout (the parameter-decoupled kernel)
        kname = "%s<26, %d, %d, %d, 1> (53-DOF state, parameter-decoupled)" % (kfam, f.epoch_qshape(), evs, sr)
    else:
        kname = "%s<%d, %d, %d, %d>" % (kfam, a.dof, f.epoch_qshape(), evs, sr)
    workload = "%s-dof%d-b%d%s%s%s%s" % (log_mode, a.dof, B, "-dense" if a.dense else "",
                                         "-lad" if getattr(a, "literal_apply_delta", False) else "", "" if sr else "-left",
                                         ("-pdpair" if pair_window else "-pd") if pd_window else
                                         ("-pair" if pair_window else ""))
    pmc = pmc_entry(workload, a.steps)
    cr = None if a.dense or launches != 1 else counter_roofline(pmc, B, a.steps, kernel_ms)
    traffic = pmc.get("bytes_per_launch") if pmc.get("epochs_per_launch") == a.steps and launches == 1 else None
    frac_useful = model_tf / PEAK_FP64_TFLOPS
    frac_issued = cr["achieved_tflops"] / PEAK_FP64_TFLOPS if cr else None
    lanes = ((cr or {}).get("active_lanes") or {}).get("thread_cycles_per_valu_quad_cycle")
    frac_active = cr["active_tflops"] / PEAK_FP64_TFLOPS if (cr and "active_tflops" in cr) else None
    roof = {"bound": "valu-fp64", "achieved": model_tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": frac_useful, "traffic": traffic,
            "frac_useful": frac_useful, "frac_active": frac_active, "frac_issued": frac_issued,
            "kernel": kname, "launches": launches, "kernel_ms_per_launch": per_launch_ms,
            "achieved_source": "the engine's useful-flop model (bench.py psp_flops: k-column partial Cholesky, "
                               "2k+1 model evaluations, O(n^2) covariance algebra per step, DESIGN.md 4.3) over this "
                               "run's HIP-event kernel time; frac = frac_useful",
            "frac_issued_source": ("fp64 VALU lane-slot flops, 64 x (2 SQ_INSTS_VALU_FMA_F64 + SQ_INSTS_VALU_MUL_F64 "
                                   "+ SQ_INSTS_VALU_ADD_F64), plus 512 x SQ_INSTS_VALU_MFMA_MOPS_F64, per wave-epoch from the committed PMC passes of this "
                                   "launch shape (%s), over this run's kernel time: counts masked lanes, an upper "
                                   "bound" % (cr or {}).get("source")) if cr else None,
            "frac_active_source": ("VALU lane-slot flops x SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU / 64 (%.1f of 64 lanes "
                                   "active per VALU cycle), plus the MFMA flops" % lanes) if frac_active is not None else None,
            "counters": cr,
            "model_flop_per_step": step_model,
            "frac_53dof_model": ((B * (F_STEP_PSP * a.steps + F_UPD3_PSP * n_dvl)) / (kernel_ms * 1e-3) / 1e12
                                 / PEAK_FP64_TFLOPS) if pd_window else None,
            "frac_53dof_model_note": ("the general 53-DOF kernel's useful-flop model (51,140 flop per step) over "
                                      "this run's time: the work the parameter-decoupled kernel does not have to "
                                      "do (the parameter block's zeros) counted as done; for comparison with the "
                                      "general kernel's frac, not the roofline") if pd_window else None,
            "model_tflops": model_tf,
            "effective_tflops": eff_tf,
            "effective_note": "reference-equivalent rate: SURVEY 8(d)'s literal-ukfom work (1,554,084 flop per "
                              "step + 853,707 per DVL update) over the kernel time; the PSP engine computes the "
                              "same result with ~3.4% of those flops (DESIGN.md 4.3), so this is not a roofline",
            "traffic_source": ("rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes, the timed launch of this shape "
                               "(%s)" % pmc.get("source")) if traffic else None}
    if mode == "C5":
        desc = "C5: %d Monte-Carlo PoseUKF %d-DOF instances, %d per GPU, 1 kHz IMU + 5 Hz DVL, ensemble statistics " \
               "all-reduced every %d epochs and at the window's end" % (B * world, a.dof, B, every)
    else:
        desc = "%s: PoseUKF %d-DOF, batch %d per GPU, 1 kHz IMU + 5 Hz DVL%s" % (
            mode, a.dof, B, " + ADCP x4 + DVL drop-out/efforts + pressure" if mode == "C4" else "")
    coll_desc = collective_desc(dist, world, comm, comm_err, same_dev)
    out = {
        "metric": METRIC, "value": value, "unit": "steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": desc,
                   "global_batch": B * world, "batch_per_gpu": B, "step": "one IMU epoch per instance",
                   "dvl_epochs_in_window": n_dvl,
                   "efforts_epochs_in_window": n_eff,
                   "adcp_epochs_in_window": int(((window & 8) != 0).sum()),
                   "c4_cycle_s": list(cyc) if mode == "C4" else None,
                   "segments": ({"count": len(seg_bounds), "epochs_per_segment": seg,
                                 "note": "each segment's inputs generated and uploaded outside the timed region "
                                         "(bitwise slices of the whole log, synth.make_pose_log epoch0); the "
                                         "filter state stays in HBM; value = steps / the sum of the segments' "
                                         "timed runs"} if seg else None),
                   "parallelism": "instance-sharded x%d (no data-path collective)" % world,
                   "collective": coll_desc,
                   "stats_allreduces_in_window": len(cuts) if world > 1 else 0,
                   "same_device_rehearsal": same_dev,
                   "init": ("Monte-Carlo start: truth + draws from a small prior (orientation sd %s rad, velocity "
                            "sd %g m/s), second constructor" % (list(synth.MC_ROT_SD), synth.MC_VEL_SD))
                           if a.init == "mc" else "first constructor (prior from the config)",
                   "path": "dense (all 2n+1 sigma points)" if a.dense else "PSP (partitioned sigma points)",
                   "so3_boxplus": "left (nav frame, exp(d) q)" if a.so3_left else "right (body frame, q exp(d))",
                   "kernel": kname,
                   "config_file": a.config or None},
        "collective_check": coll_check,
        "roofline": roof,
        "timing": {"wall_ms": wall * 1e3, "kernel_ms": kernel_ms, "outside_kernel_ms": wall * 1e3 - kernel_ms},
        "ensemble": {"nees_mean_pos_ori_vel": float(stats[-2] / max(1.0, B * world - stats[-1])),
                     "nees_excluded_instances": int(stats[-1])},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(synth, cfg, uwv, log_mode, a.dof, a.cpu_threads or available_cores(),
                                           a.init, right=not a.so3_left)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()
    if coll_check is False:
        sys.exit(3)


def bench_c1(a):
    """Config C1: one PoseUKF, the kinematic n = 26 layout (the
    config's "~30-dim state") and the full n = 53, a 60 s log = 60,000 IMU
    epochs with 300 DVL updates (5 Hz), on ONE CPU core: the fp64 C oracle's
    timing build (oracle/liboracle_fast.so, -O3 x86-64-v4), i.e. ukfom's literal
    algorithm (all 2n+1 sigma points) restated -- the reference itself cannot be
    built here.  No GPU is used.  --steps sets the epochs (default
    60,000 when --steps is left at its default)."""
    from uwvk import synth
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as O
    epochs = 60_000 if a.steps == 200 else a.steps
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else []
    avail = available_cores()
    if cpus:
        os.sched_setaffinity(0, {cpus[0]})  # one core, as SURVEY 8(d)(i)
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    res = {}
    with O.so3_side(not a.so3_left):
        for dof in (26, 53):
            log = synth.make_pose_log(1, epochs, mode="C3", dof=dof, cfg=cfg)
            o = O.OraclePoseBatch(1, dof, timing=True)
            initialise(o, log, cfg, uwv, a.init)
            o.set_process_noise_from_config(cfg, log["dt"])
            t0 = time.perf_counter()
            counts = o.run_log(log, nthreads=1)
            dt = time.perf_counter() - t0
            x, P = o.get_state()
            res[dof] = {"value": epochs / dt, "seconds": dt, "epochs": epochs,
                        "dvl_updates": int(((log["flags"] & 2) != 0).sum()),
                        "accepted_updates": [int(v) for v in counts[0]],
                        "finite": bool(np.all(np.isfinite(x)) and np.all(np.isfinite(P))),
                        "flop_per_step": (F_STEP if dof == 53 else 192_366)}
            del log, o
    out = {"metric": "PoseUKF predict+update steps/sec, 1 instance on 1 CPU core (config C1)",
           "value": res[26]["value"], "unit": "steps/s", "n_gpus": 0, "steps": epochs, "warmup": 0,
           "ms_per_step": 1e3 / res[26]["value"], "higher_is_better": True, "scaling": None, "vs_baseline": None,
           "dtype": "f64", "data": "synthetic",
           "config": {"workload": "C1: one PoseUKF, n = 26 (kinematic subset, the config's ~30-dim state; value) and "
                                  "n = 53 (full state), %d epochs of 1 kHz IMU + 5 Hz DVL" % epochs,
                      "global_batch": 1, "so3_boxplus": "left (nav frame, exp(d) q)" if a.so3_left
                      else "right (body frame, q exp(d))",
                      "implementation": "fp64 C oracle, timing build (oracle/liboracle_fast.so: -O3 "
                                        "-march=x86-64-v4), ukfom's literal algorithm; the reference is unbuildable "
                                        "here (SURVEY K3)",
                      "init": "Monte-Carlo start (second constructor)" if a.init == "mc" else "first constructor"},
           "dof26": res[26], "dof53": res[53],
           "host": {"cpu": _cpu_model(), "nproc": os.cpu_count(), "available_to_job": avail,
                    "pinned_cpu": cpus[0] if cpus else None}}
    print(json.dumps(out), flush=True)


def bench_vel(a, engine, synth, world, rank, local, dist, B):
    """Config C2: VelocityUKF (VelocityUKF.cpp:79-130), batch 4096 per GPU,
    1 kHz gyro + efforts, 5 Hz DVL, 10 Hz pressure.  One step = one epoch of
    one instance (gyro/efforts store, predict, due updates)."""
    log = synth.make_vel_log(B, a.warmup + a.steps, first_instance=rank * B)
    f = engine.VelocityUKFBatch(B, device=local)
    f.set_lane_groups(a.vel_groups)
    f.init(log["x0"], log["P0"])
    f.set_gyro(log["gyro"][0])
    f.setup_motion_model(synth.default_uwv())
    d = f.upload_log(log)
    f.run_log(d, 0, a.warmup)
    if dist is not None:
        dist.barrier()
    f.synchronize()
    t0 = time.perf_counter()
    f.timer_start()
    f.run_log(d, a.warmup, a.steps, sync=False)
    kernel_ms = f.timer_stop()
    f.synchronize()
    if dist is not None:
        dist.barrier()
    wall = time.perf_counter() - t0
    if dist is not None:
        import torch
        w = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    groups = a.vel_groups if a.vel_groups >= 0 else int(B <= 30720)  # uwvk_vel.hip kVelGroupsMaxBatch
    launches = (a.steps + 4095) // 4096
    flops = B * F_VEL_STEP * a.steps
    tf = flops / (kernel_ms * 1e-3) / 1e12
    tf_ref = B * F_VEL_STEP_REF * a.steps / (kernel_ms * 1e-3) / 1e12
    kname = "k_vel_epoch_g" if groups else "k_vel_epoch"
    out = {
        "metric": "VelocityUKF predict+update steps/sec at batch=%d (config C2)" % B, "value": B * world * a.steps / wall,
        "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C2: VelocityUKF 4-DOF, batch %d per GPU, 1 kHz gyro + efforts, 5 Hz DVL, 10 Hz depth"
                               % B, "global_batch": B * world, "batch_per_gpu": B,
                   "layout": {0: "one filter per lane", 1: "16 lanes per filter",
                              2: "16 lanes per filter, each filter run twice in a 32-lane group (diagnostic)"}[groups],
                   "kernel": kname if groups != 2 else kname + "<32>"},
        "roofline": {"bound": "valu-fp64", "achieved": tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf / PEAK_FP64_TFLOPS, "traffic": None, "kernel": kname, "launches": launches,
                     "kernel_ms_per_launch": kernel_ms / launches, "algorithmic_flop_per_step": F_VEL_STEP,
                     "achieved_source": "the kernel's executed formulation (bench.py F_VEL_STEP: restoring forces "
                                        "through one rotation, VEL_GLIN) over the HIP-event kernel time",
                     "reference_formulation": {"flop_per_step": F_VEL_STEP_REF, "tflops": tf_ref,
                                               "frac": tf_ref / PEAK_FP64_TFLOPS,
                                               "note": "the same time priced at the reference's formulation "
                                                       "(two rotations for the restoring forces); not a roofline"}},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = a.cpu_threads or available_cores()
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle_ctypes as O
        # bounded sample (~10 s on 16 cores): the 2000-epoch log replayed `passes` times
        nb, ne, passes = 64 * threads, 2000, 30
        clog = synth.make_vel_log(nb, ne)
        o = O.OracleVelBatch(nb, timing=True)
        o.init(clog["x0"], clog["P0"])
        o.set_gyro(clog["gyro"][0])
        o.setup_motion_model(synth.default_uwv())
        c0 = time.perf_counter()
        for _ in range(passes):
            o.run_log(clog, nthreads=threads)
        cdt = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": nb * ne * passes / cdt, "unit": "steps/s", "cores": threads, "kind": "port",
                               "sample": "%d VelocityUKF instances x %d epochs x %d passes (C2), %d pthreads, %.2f s wall"
                                         % (nb, ne, passes, threads, cdt)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
