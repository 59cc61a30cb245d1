"""Instance sharding over ranks (world_size 2, gloo on CPU): each rank runs its
contiguous shard with the CPU oracle; per-instance results are bit-identical to
the single-process run and the all-reduced ensemble statistics equal the
single-process statistics."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

B, EPOCHS = 6, 220


def _run_shard(lo, hi):
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle_ctypes as O
    from uwvk import synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(hi - lo, EPOCHS, "C3", first_instance=lo)
    o = O.OraclePoseBatch(hi - lo)
    o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o.set_process_noise_from_config(cfg, log["dt"])
    o.run_log(log)
    x, P = o.get_state()
    return x, P, log["truth"].state(EPOCHS)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import ensemble
    lo, hi = ensemble.shard_range(rank, world, B)
    x, P, truth = _run_shard(lo, hi)
    stats = ensemble.allreduce_stats(ensemble.ensemble_stats_host(x, P, truth), dist)
    q.put((rank, lo, hi, x, P, stats))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_match_single_process():
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import ensemble
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    x1, P1, truth = _run_shard(0, B)
    for rank, lo, hi, x, P, stats in res:
        assert np.array_equal(x, x1[lo:hi]) and np.array_equal(P, P1[lo:hi])  # bit-identical per instance
        np.testing.assert_allclose(stats, ensemble.ensemble_stats_host(x1, P1, truth), rtol=1e-12, atol=1e-12)


def test_shard_ranges_cover_batch():
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import ensemble
    for world in (1, 2, 3, 8):
        r = [ensemble.shard_range(k, world, 1048576 + 5) for k in range(world)]
        assert r[0][0] == 0 and r[-1][1] == 1048576 + 5
        assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))


@pytest.mark.gpu
def test_ensemble_stats_kernel_matches_host():
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import engine, ensemble, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(300, 50, "C3")
    f = engine.PoseUKFBatch(300)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    f.run_log(f.upload_log(log))
    truth = log["truth"].state(50)
    x, P = f.get_state()
    np.testing.assert_allclose(f.ensemble_stats(truth), ensemble.ensemble_stats_host(x, P, truth), rtol=1e-9,
                               atol=1e-12)
    # fixed-order two-stage reduction: repeated calls agree bitwise
    np.testing.assert_array_equal(f.ensemble_stats(truth), f.ensemble_stats(truth))


@pytest.mark.gpu
def test_ensemble_stats_many_partials():
    """Batch 20,000: 313 wave partials (more than the 256 threads of the final
    sum), ragged last wave; host reference and bitwise repeatability."""
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import engine, ensemble, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(20000, 2, "C3")
    f = engine.PoseUKFBatch(20000)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    truth = log["truth"].state(0)
    x, P = f.get_state()
    got = f.ensemble_stats(truth)
    np.testing.assert_allclose(got, ensemble.ensemble_stats_host(x, P, truth), rtol=1e-9, atol=1e-12)
    np.testing.assert_array_equal(got, f.ensemble_stats(truth))


@pytest.mark.gpu
def test_rccl_allreduce_through_c_abi():
    """uwvk_pose_ensemble_allreduce over an RCCL communicator made by the C ABI
    (uwvk_comm_*): with one rank the RCCL sum equals the local statistics
    (the N-rank case runs in the driver's 8-GPU bench)."""
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import engine, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(70, 30, "C3")
    f = engine.PoseUKFBatch(70)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    f.run_log(f.upload_log(log))
    truth = log["truth"].state(30)
    comm = engine.RcclComm(1, engine.RcclComm.unique_id(), 0, 0)
    np.testing.assert_array_equal(f.ensemble_stats(truth, comm), f.ensemble_stats(truth))
    comm.close()


# ---- the sharded path on the HIP engine -----------------------

SHARD = int(os.environ.get("UWVK_TEST_SHARD", "131072"))  # C5: 1,048,576 instances / 8 GPUs
GPU_EPOCHS = 220  # includes the 5 Hz DVL update at epoch 199


def _digest(P):
    """Per-instance 64-bit digest of the covariance bytes (weighted wrap-around
    sum of the fp64 bit patterns): equal digests <=> bitwise-equal rows, up to
    a 2^-64 collision chance."""
    w = np.random.default_rng(123).integers(1, 2 ** 63, size=P.shape[1:], dtype=np.uint64) | np.uint64(1)
    v = np.ascontiguousarray(P).view(np.uint64)
    with np.errstate(over="ignore"):
        return (v * w).sum(axis=(1, 2), dtype=np.uint64)


def _gpu_shard_run(lo, hi, device=0):
    from uwvk import engine, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(hi - lo, GPU_EPOCHS, "C3", first_instance=lo)
    f = engine.PoseUKFBatch(hi - lo, device=device)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    f.run_log(f.upload_log(log))
    assert not f.get_status().any()
    return f, log["truth"].state(GPU_EPOCHS)


def _gpu_worker(rank, world, port, outdir, q):
    try:
        import torch.distributed as dist  # torch (and its bundled HIP runtime / RCCL) first, as in bench.py
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
        from uwvk import ensemble
        lo, hi = ensemble.shard_range(rank, world, SHARD * world)
        f, truth = _gpu_shard_run(lo, hi)
        local = f.ensemble_stats(truth)
        summed = ensemble.allreduce_stats(local, dist)
        x, P = f.get_state()
        np.save(os.path.join(outdir, "x%d.npy" % rank), x)
        q.put((rank, lo, hi, _digest(P), local, summed, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, None, None, None, None, None, repr(e)))


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_gpu_two_rank_shards_bitwise(tmp_path):
    """Two ranks (processes, gloo) each drive libuwvk on device 0 with C5's
    shard size (131,072 instances per rank): per-instance mu bit-identical and
    Sigma digests equal to ONE process running all 262,144 instances, the
    all-reduced statistics equal to the sum of the per-rank ones and to the
    host reduction over the full batch."""
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import ensemble
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() % 1000)
    world = 2
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
    errs = [r[-1] for r in res if r[-1]]
    assert not errs, errs
    assert all(p.exitcode == 0 for p in procs)
    f, truth = _gpu_shard_run(0, SHARD * world)
    x1, P1 = f.get_state()
    d1 = _digest(P1)
    for rank, lo, hi, dig, local, summed, _ in res:
        x = np.load(str(tmp_path / ("x%d.npy" % rank)))
        np.testing.assert_array_equal(x, x1[lo:hi])
        np.testing.assert_array_equal(dig, d1[lo:hi])
        np.testing.assert_array_equal(summed, res[0][5])
    np.testing.assert_array_equal(res[0][5], res[0][4] + res[1][4])  # a two-term sum is exact in any order
    host = ensemble.ensemble_stats_host(x1, P1, truth)
    np.testing.assert_allclose(res[0][5], host, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(res[0][5], f.ensemble_stats(truth), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
def test_rccl_c_abi_two_devices():
    """uwvk_pose_ensemble_allreduce across two GPUs (rank r on device r) through
    the C ABI's own RCCL communicator; skipped on a one-GPU box."""
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import engine
    import ctypes as C
    n = C.c_int(0)
    hip = C.CDLL("libamdhip64.so.7")
    hip.hipGetDeviceCount(C.byref(n))
    if n.value < 2:
        pytest.skip("needs 2 GPUs (%d visible)" % n.value)
    import subprocess
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_two_rank.py"), "--ranks", "2"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr
    assert engine.device_available(1)


@pytest.mark.gpu
def test_ensemble_stats_excludes_non_pd_instances():
    """An instance whose (position, orientation, velocity) block is not positive
    definite is counted in out[3 store + 1] and left out of the NEES sum
    instead of turning the whole batch's NEES into NaN (advisor r01)."""
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import abi, engine, ensemble, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    B = 130
    log = synth.make_pose_log(B, 2, "C3")
    f = engine.PoseUKFBatch(B)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    x, P = f.get_state()
    P[7, 0, 0] = -1.0  # indefinite
    P[64, 4, 4] = 0.0  # singular
    f.init_from_state(x, P, abi.Location(synth.LAT0, synth.LON0, 0.0), uwv, abi.PoseParameter())
    truth = log["truth"].state(0)
    got = f.ensemble_stats(truth)
    host = ensemble.ensemble_stats_host(x, P, truth)
    assert np.all(np.isfinite(got))
    assert got[-1] == 2 and host[-1] == 2
    np.testing.assert_allclose(got, host, rtol=1e-9, atol=1e-12)
    # a NaN state (velocity) is left out of the NEES sum by both (advisor r02);
    # the plain sums of that component are NaN on both sides
    x[20, 8] = np.nan
    f.init_from_state(x, P, abi.Location(synth.LAT0, synth.LON0, 0.0), uwv, abi.PoseParameter())
    got = f.ensemble_stats(truth)
    host = ensemble.ensemble_stats_host(x, P, truth)
    assert got[-1] == 3 and host[-1] == 3 and np.isfinite(got[-2])
    np.testing.assert_allclose(got, host, rtol=1e-9, atol=1e-12, equal_nan=True)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("ranks", [2, 4])
def test_bench_self_launches_ranks(ranks):
    """`bench.py --gpus N` with no launcher starts its N rank processes itself
    (one-GPU rehearsal: UWVK_BENCH_SAME_DEVICE puts all on device 0, where
    RCCL refuses a second rank, so the statistics sum goes over gloo) and
    reports the whole job: n_gpus N, the global batch of all shards."""
    import json
    import subprocess
    env = dict(os.environ, UWVK_BENCH_SAME_DEVICE="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(ranks), "--steps", "20", "--warmup",
                        "2", "--batch-per-gpu", "16384", "--no-cpu-baseline"], capture_output=True, text=True,
                       timeout=500, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == ranks and d["config"]["global_batch"] == ranks * 16384
    assert d["config"]["workload"].startswith("C5") and d["collective_check"] is True
    assert d["value"] > 0 and d["config"]["stats_allreduces_in_window"] == 1
