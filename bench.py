#!/usr/bin/env python3
"""bench.py — batched PoseUKF predict+update throughput on MI355X.

Metric (BASELINE.json): UKF predict+update steps/sec at batch = 65536 PoseUKF
instances (config C3: full 53-DOF PoseState, 1 kHz IMU + 5 Hz DVL).
One "step" = one IMU epoch of ONE filter instance: RotationRate store ->
predictionStep(1 ms) -> Acceleration update, plus the DVL velocity update
when the 5 Hz schedule is due.  `value` counts
instance-epochs per second over the whole job (all ranks).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
instances are sharded across ranks (weak scaling: --batch-per-gpu instances on
every GPU, no data-path collective); the only collective is the RCCL
all-reduce of the ensemble statistics at the end of the timed region.

Inputs are synthetic (uwvk.synth) and resident in HBM before timing starts.
Timing: barrier + device sync on both sides of the timed region, max over
ranks; the dominant kernel's average launch time comes from HIP events on the
handle's stream.  cpu_baseline: the fp64 C oracle (oracle/, "port") on a
bounded sample of the same workload, on rank 0 at N = 1 only.
"""
import argparse
import json
import os
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


def psp_flops(n=53, k_pred=15, updates=((6, 3, 7),)):
    """Flops the PSP kernels execute per step: k-column
    partial Cholesky, 2k+1 model evaluations, O(n^2) covariance algebra.
    updates: (k, m, ncols) per update of the step."""
    def pchol(k):
        return 2 * sum((k - 1 - j) * (n - j) for j in range(k)) + 3 * k * (n - k // 2)
    np_ = n * (n + 1) // 2
    f = pchol(k_pred) + (2 * k_pred + 1) * (120 + 3 * 60)  # points + 3 mean iterations
    f += 2 * n * k_pred * 3 + 6 * 2 * (2 * k_pred + 1)      # L Delta, ori x ori
    f += 7 * 6 * n + 4 * np_                                # A-coupled rows, decays + Q'
    for k, m, nc in updates:
        f += pchol(k) + (2 * k + 1) * 50 + 2 * m * k * nc + 2 * n * nc * m
        f += 2 * n * k * m + 2 * n * m * m + 2 * np_ * m + 2 * 9 * n
    return f


F_STEP_PSP = psp_flops()
F_UPD3_PSP = psp_flops(updates=((6, 3, 7), (6, 3, 3))) - F_STEP_PSP  # one DVL update
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 (vector = matrix) spec; probe measured 74 (profiles/r01_probe_fp64.txt)
PEAK_HBM_GBS = 8000.0


# VelocityUKF (config C2) work per step, frozen from the kernel's code
# (uwvk_vel.hip): one RK4 step of the Fossen model = 4 derivative evaluations
# x ~530 flop (rotations 90, Coriolis 102, damping 186, restoring 90, M^-1 72)
# + stage sums / normalisation ~170 = 2,290 flop; a predict integrates the 9
# sigma points and the side model (10 RK4) plus ~900 flop of 4-DOF UKF algebra;
# DVL (5 Hz) and pressure (10 Hz) updates add ~20 flop per step on average.
F_VEL_RK4 = 2_290
F_VEL_STEP = 10 * F_VEL_RK4 + 900 + 20  # 23,820


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200, help="timed epochs")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch-per-gpu", type=int, default=0, help="0: 65536 (C3/C4), 4096 (C2)")
    ap.add_argument("--dof", type=int, default=53)
    ap.add_argument("--mode", default="C3", choices=["C2", "C3", "C4"],
                    help="C3 (headline) / C4: PoseUKF; C2: VelocityUKF (secondary line)")
    ap.add_argument("--c4-cycle", default="30,10",
                    help="C4 DVL drop-out cycle 'on,off' in s; e.g. 0.3,0.1 keeps every event rate of the 30/10 "
                         "cycle (0.25%% efforts epochs) inside a 2000-epoch window")
    ap.add_argument("--vel-groups", type=int, default=-1, help="C2: -1 auto, 0 lane per filter, 1 16-lane rows")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dense", action="store_true", help="literal kernels (all 2n+1 sigma points)")
    ap.add_argument("--tail-slots", type=int, default=0,
                    help="UWVK_OPT_TAIL_SLOTS: 0 runtime occupancy, > 0 blocks per XCD, < 0 no tail spreading")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core available to this process")
    return ap.parse_args()


def dvl_aligned_log(synth, batch, warmup, steps, mode, dof, first_instance, c4_cycle=(30.0, 10.0)):
    """Log of warmup+steps epochs whose 5 Hz DVL schedule puts at least one DVL
    epoch inside the timed window (exactly the 1-in-200 rate when steps >= 200)."""
    total = warmup + steps
    # shift the start so that a DVL epoch (k % 200 == 0) lands mid-window
    target = warmup + min(steps, 200) // 2
    shift = (200 - (target + 1) % 200) % 200
    # diagnostic only (never the headline): UWVK_BENCH_WINDOW_OFFSET moves the window
    # off the DVL epoch (100: no DVL update in a window of < 100 epochs); the line
    # reports dvl_epochs_in_window either way
    shift += int(os.environ.get("UWVK_BENCH_WINDOW_OFFSET", "0"))
    log = synth.make_pose_log(batch, total + shift, mode=mode, dof=dof, first_instance=first_instance,
                              dropout_on=c4_cycle[0], dropout_off=c4_cycle[1])
    return log, shift


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
    out = {"fp64_lane_flop_per_wave_epoch": lane_flop,
           "achieved_tflops": lane_flop * waves * epochs / (kernel_ms * 1e-3) / 1e12,
           "epochs_profiled": e.get("epochs_per_launch"), "source": e.get("valu_source")}
    for k in ("valu_busy", "active_lanes"):
        if k in e:
            out[k] = e[k]
    return out


def cpu_baseline(synth, cfg, uwv, mode, dof, threads):
    """The fp64 C oracle's timing build (oracle/liboracle_fast.so: -O3,
    x86-64-v4, one instance per task, pthreads) on a bounded sample of the same
    workload, on every core this process may use; plus one instance on one
    core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as O
    epochs = 2000
    # single core first: it sizes the multi-core sample to ~15 s of wall time
    log1 = synth.make_pose_log(1, epochs, mode=mode, dof=dof)
    o1 = O.OraclePoseBatch(1, dof, timing=True)
    o1.init_from_config(log1["pos0"], log1["pos_cov"], log1["rot0"], log1["rot_cov"], cfg, uwv)
    o1.set_process_noise_from_config(cfg, log1["dt"])
    t1 = time.perf_counter()
    o1.run_log(log1, nthreads=1)
    dt1 = time.perf_counter() - t1
    rate1 = epochs / dt1
    per_thread = max(1, int(round(15.0 * rate1 / epochs)))
    batch = per_thread * threads
    log = synth.make_pose_log(batch, epochs, mode=mode, dof=dof)
    o = O.OraclePoseBatch(batch, dof, timing=True)
    o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o.set_process_noise_from_config(cfg, log["dt"])
    t0 = time.perf_counter()
    o.run_log(log, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"value": batch * epochs / dt, "unit": "steps/s", "cores": threads, "kind": "port",
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


def init_dist(world, local, backend):
    """One process per GPU: the process group is made whenever the job runs
    under torch.distributed.run (world size 1 included) or with WORLD_SIZE > 1.
    It is a host-side control plane (gloo by default): barriers, the id of the
    RCCL check communicator and the 163-double statistics sum.  An RCCL
    communicator in the process (torch's nccl group or the engine's own) slows
    the concurrently running epoch kernel by 6-7% on the GPU (r02: 9.20 ->
    9.88 ms per 20-epoch launch, rocprofv3 kernel trace),
    so none exists during the timed region."""
    if world == 1 and not launched_by_torchrun():
        return None
    import torch
    import torch.distributed as dist
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    return dist


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("UWVK_BENCH_BACKEND", "gloo")
    # UWVK_BENCH_SAME_DEVICE=1: rehearsal of the N-rank path on one GPU (all ranks on device 0)
    if os.environ.get("UWVK_BENCH_SAME_DEVICE") == "1":
        local = 0
    stat_dev = "cuda" if backend == "nccl" else None
    dist = init_dist(world, local, backend)
    from uwvk import engine, ensemble, synth

    if a.mode == "C2":
        return bench_vel(a, engine, synth, world, rank, local, dist)
    B = a.batch_per_gpu or 65536
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    cyc = tuple(float(v) for v in a.c4_cycle.split(","))
    log, shift = dvl_aligned_log(synth, B, a.warmup, a.steps, a.mode, a.dof, first_instance=rank * B, c4_cycle=cyc)
    f = engine.PoseUKFBatch(B, a.dof, device=local)
    f.set_tail_slots(a.tail_slots)
    if a.dense:
        f.set_dense_sigma(True)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    dlog = f.upload_log(log)
    flags = log["flags"]
    # advance through the alignment shift (untimed)
    if shift:
        f.run_log(dlog, 0, shift)
    f.run_log(dlog, shift, a.warmup)  # warmup (untimed)
    e0 = shift + a.warmup
    window = flags[e0:e0 + a.steps]
    n_dvl = int(((window & 2) != 0).sum())
    truth = log["truth"].state(e0 + a.steps, a.dof)
    # the collective of the timed region: the per-rank statistics summed over the
    # process group (host side, 163 doubles).  UWVK_BENCH_COLL=rccl sums them with
    # the engine's RCCL communicator on the handle's stream instead (slower, see
    # init_dist); by default RCCL runs after the timed region as a cross-check.
    comm = None
    coll = os.environ.get("UWVK_BENCH_COLL", "host")

    def make_comm():
        uid = [engine.RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        return engine.RcclComm(world, uid[0], rank, local)

    if dist is not None and coll == "rccl":
        comm = make_comm()
    # warm the statistics kernels and the collective (module load, communicator
    # set-up) outside the timed region
    st_w = f.ensemble_stats(truth, comm)
    if dist is not None and comm is None:
        ensemble.allreduce_stats(st_w, dist, device=stat_dev)

    def barrier():
        if dist is not None:
            dist.barrier()

    barrier()
    f.synchronize()
    t0 = time.perf_counter()
    f.timer_start()
    f.run_log(dlog, e0, a.steps, sync=False)
    f.timer_mark()  # HIP events on the handle's stream around the epoch launches (no host wait)
    # synchronous; RCCL over xGMI (comm) is the only collective of the workload
    stats = f.ensemble_stats(truth, comm)
    if dist is not None and comm is None:
        stats = ensemble.allreduce_stats(stats, dist, device=stat_dev)
    f.synchronize()
    barrier()
    wall = time.perf_counter() - t0
    kernel_ms = f.timer_elapsed()
    if dist is not None:
        import torch
        w = torch.tensor([wall], dtype=torch.float64)
        if stat_dev:
            w = w.cuda()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        wall = float(w.item())
    # untimed: the same sum through the engine's RCCL path (uwvk_pose_ensemble_allreduce)
    rccl_check = None
    same_dev = os.environ.get("UWVK_BENCH_SAME_DEVICE") == "1"  # RCCL refuses two ranks on one GPU
    if dist is not None and comm is None and not same_dev and os.environ.get("UWVK_BENCH_RCCL_CHECK", "1") == "1":
        try:  # a cross-check after timing: its failure is reported, it does not void the line
            comm = make_comm()
            rs = f.ensemble_stats(truth, comm)
            rccl_check = bool(np.allclose(rs, stats, rtol=1e-12, atol=1e-12))
        except Exception as ex:  # noqa: BLE001
            print("warning: RCCL cross-check failed: %r" % (ex,), file=sys.stderr)
            rccl_check = False
    status = f.get_status()
    if status.any():
        print("warning: %d instances flagged (status bits)" % int((status != 0).sum()), file=sys.stderr)

    steps_total = B * world * a.steps
    value = steps_total / wall
    # launches in the timed window: the PSP path runs the whole window in one
    # k_psp_epoch launch (efforts epochs split it); the literal path one per epoch
    n_eff = int(((window & 0x10) != 0).sum())
    launches = a.steps if a.dense else 1 + 2 * n_eff
    per_launch_ms = kernel_ms / launches
    # reference-equivalent work (the literal ukfom algorithm)
    flops_ref = B * (F_STEP * a.steps + F_UPD3 * n_dvl)
    # the engine's own flop model
    flops_model = B * ((F_STEP_EXEC * a.steps + F_UPD3_EXEC * n_dvl) if a.dense
                       else (F_STEP_PSP * a.steps + F_UPD3_PSP * n_dvl))
    eff_tf = flops_ref / (kernel_ms * 1e-3) / 1e12
    model_tf = flops_model / (kernel_ms * 1e-3) / 1e12
    kname = ("k_pose_epoch<%d>" if a.dense else "k_psp_epoch<%d>") % a.dof
    workload = "%s-dof%d-b%d%s" % (a.mode, a.dof, B, "-dense" if a.dense else "")
    pmc = pmc_entry(workload, a.steps)
    cr = None if a.dense or launches != 1 else counter_roofline(pmc, B, a.steps, kernel_ms)
    traffic = pmc.get("bytes_per_launch") if pmc.get("epochs_per_launch") == a.steps else None
    achieved = cr["achieved_tflops"] if cr else model_tf
    roof = {"bound": "mfma", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic,
            "kernel": kname, "launches": launches, "kernel_ms_per_launch": per_launch_ms,
            "achieved_source": ("fp64 VALU lane-flops from SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 of the committed PMC "
                                "passes of this launch shape (%s), over this run's HIP-event kernel time"
                                % (cr or {}).get("source") if cr else
                                "the engine's flop model (no PMC pass of this shape committed)"),
            "counters": cr,
            "model_flop_per_step": (F_STEP_EXEC if a.dense else F_STEP_PSP),
            "model_tflops": model_tf,
            "effective_tflops": eff_tf,
            "effective_note": "reference-equivalent rate: SURVEY 8(d)'s literal-ukfom work (1,554,084 flop per "
                              "step + 853,707 per DVL update) over the kernel time; the PSP engine computes the "
                              "same result with ~3.4% of those flops (DESIGN.md 4.3), so this is not a roofline",
            "traffic_source": ("rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, separate passes, the timed launch of this shape "
                               "(%s)" % pmc.get("source")) if traffic else None}
    out = {
        "metric": METRIC, "value": value, "unit": "steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "%s: PoseUKF %d-DOF, batch %d per GPU, 1 kHz IMU + 5 Hz DVL%s"
                               % (a.mode, a.dof, B, " + ADCP x4 + DVL drop-out/efforts + pressure"
                                  if a.mode == "C4" else ""),
                   "global_batch": B * world, "batch_per_gpu": B, "step": "one IMU epoch per instance",
                   "dvl_epochs_in_window": n_dvl,
                   "efforts_epochs_in_window": n_eff,
                   "adcp_epochs_in_window": int(((window & 8) != 0).sum()),
                   "c4_cycle_s": list(cyc) if a.mode == "C4" else None,
                   "parallelism": "instance-sharded x%d (no data-path collective)" % world,
                   "collective": (("RCCL all_reduce of the ensemble statistics on the handle's stream "
                                   "(uwvk_pose_ensemble_allreduce)") if coll == "rccl" else
                                  ("%s all_reduce of the ensemble statistics (host); untimed RCCL cross-check: %s"
                                   % (backend, rccl_check))) if dist else None,
                   "path": "dense (all 2n+1 sigma points)" if a.dense else "PSP (partitioned sigma points)",
                   "kernel": kname},
        "roofline": roof,
        "timing": {"wall_ms": wall * 1e3, "kernel_ms": kernel_ms, "outside_kernel_ms": wall * 1e3 - kernel_ms},
        "ensemble": {"nees_mean_pos_ori_vel": float(stats[-2] / max(1.0, B * world - stats[-1])),
                     "nees_excluded_instances": int(stats[-1])},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(synth, cfg, uwv, a.mode, a.dof, a.cpu_threads or available_cores())
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()


def bench_vel(a, engine, synth, world, rank, local, dist):
    """Config C2: VelocityUKF (VelocityUKF.cpp:79-130), batch 4096 per GPU,
    1 kHz gyro + efforts, 5 Hz DVL, 10 Hz pressure.  One step = one epoch of
    one instance (gyro/efforts store, predict, due updates)."""
    B = a.batch_per_gpu or 4096
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
    groups = a.vel_groups if a.vel_groups >= 0 else int(B <= 24576)  # uwvk_vel.hip kVelGroupsMaxBatch
    launches = (a.steps + 4095) // 4096
    flops = B * F_VEL_STEP * a.steps
    tf = flops / (kernel_ms * 1e-3) / 1e12
    kname = "k_vel_epoch_g" if groups else "k_vel_epoch"
    out = {
        "metric": "VelocityUKF predict+update steps/sec at batch=%d (config C2)" % B, "value": B * world * a.steps / wall,
        "unit": "steps/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C2: VelocityUKF 4-DOF, batch %d per GPU, 1 kHz gyro + efforts, 5 Hz DVL, 10 Hz depth"
                               % B, "global_batch": B * world, "batch_per_gpu": B,
                   "layout": "16 lanes per filter" if groups else "one filter per lane", "kernel": kname},
        "roofline": {"bound": "mfma", "achieved": tf, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf / PEAK_FP64_TFLOPS, "traffic": None, "kernel": kname, "launches": launches,
                     "kernel_ms_per_launch": kernel_ms / launches, "algorithmic_flop_per_step": F_VEL_STEP},
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
