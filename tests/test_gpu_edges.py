"""GPU edge cases and full-size properties of the PoseUKF engine (C ABI).

- batch 1 (the drop-in single-filter case) against the oracle;
- BASELINE.json's full batch (65,536): per-instance results do not depend on
  where an instance sits in the batch (a half-batch handle reproduces the
  full handle's second half BITWISE: the property the instance sharding of
  SURVEY.md section 8(e) relies on), Sigma stays exactly symmetric with a
  positive diagonal, and a rerun is bitwise deterministic;
- count = 0 and argument errors."""
import numpy as np
import pytest

from helpers import cov_err, init_both, pose_setup, state_err
from uwvk import abi, engine, synth

pytestmark = pytest.mark.gpu

TOL_LOG = 1e-7


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")


@pytest.mark.parametrize("dof", [53, 26])
def test_single_filter(dof):
    import oracle_ctypes as O
    cfg, uwv, log = pose_setup(1, dof, "C3", 450)
    o, g = O.OraclePoseBatch(1, dof), engine.PoseUKFBatch(1, dof)
    init_both(o, g, cfg, uwv, log)
    o.run_log(log)
    g.run_log(g.upload_log(log))
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    assert state_err(xg, xo, Po, dof).max() < TOL_LOG
    assert cov_err(Pg, Po).max() < TOL_LOG
    assert not g.get_status().any()


def _slice(log, lo, hi):
    """the instances [lo, hi) of a pose log (epoch-major arrays)"""
    out = dict(log)
    out["batch"] = hi - lo
    for k in ("gyro", "acc", "dvl"):
        out[k] = np.ascontiguousarray(log[k][:, lo:hi])
    for k in ("pos0", "pos_cov", "rot0", "rot_cov"):
        out[k] = np.ascontiguousarray(log[k][lo:hi])
    return out


def test_full_batch_position_independent_and_deterministic():
    B, E = 65536, 40
    cfg, uwv, log = pose_setup(B, 53, "C3", E)
    # one DVL update inside the window (the synthetic 5 Hz schedule first fires at epoch 200)
    log["flags"] = log["flags"].copy()
    log["flags"][20] |= abi.EV_DVL
    log["dvl_index"] = log["dvl_index"].copy()
    log["dvl_index"][20] = 0
    log["dvl"] = np.zeros((1, B, 3))
    log["dvl"][0, :, 0] = 1.0
    runs = []
    for rep in range(2):
        g = engine.PoseUKFBatch(B, 53)
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        g.set_process_noise_from_config(cfg, log["dt"])
        g.run_log(g.upload_log(log))
        runs.append(g.get_state())
        assert not g.get_status().any()
        g.close()
    (x, P), (x2, P2) = runs
    np.testing.assert_array_equal(x, x2)  # deterministic
    np.testing.assert_array_equal(P, P2)
    np.testing.assert_array_equal(P, np.swapaxes(P, 1, 2))  # exactly symmetric
    assert (np.diagonal(P, axis1=1, axis2=2) > 0).all() and np.isfinite(P).all()
    h = B // 2
    sub = _slice(log, h, B)
    g = engine.PoseUKFBatch(B - h, 53)
    g.init_from_config(sub["pos0"], sub["pos_cov"], sub["rot0"], sub["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, log["dt"])
    g.run_log(g.upload_log(sub))
    xs, Ps = g.get_state()
    np.testing.assert_array_equal(xs, x[h:])  # bitwise: a shard reproduces the full run
    np.testing.assert_array_equal(Ps, P[h:])


def test_count_zero_and_argument_errors():
    cfg, uwv, log = pose_setup(5, 53, "C3", 10)
    g = engine.PoseUKFBatch(5, 53)
    d = g.upload_log(log)
    with pytest.raises(engine.UWVKError) as e:  # no state yet
        g.run_log(d, 0, 1)
    assert e.value.code == 7  # UWVK_ENOTINIT
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, log["dt"])
    x0, P0 = g.get_state()
    g.run_log(d, 3, 0)  # no epochs: nothing changes
    x1, P1 = g.get_state()
    np.testing.assert_array_equal(x0, x1)
    np.testing.assert_array_equal(P0, P1)
    with pytest.raises(engine.UWVKError) as e:  # past the end of the log
        g.run_log(d, 5, 6)
    assert e.value.code == 1
    with pytest.raises(engine.UWVKError) as e:
        engine.PoseUKFBatch(0, 53)
    assert e.value.code == 1
    with pytest.raises(engine.UWVKError) as e:  # unsupported state layout
        engine.PoseUKFBatch(4, 30)
    assert e.value.code == 1


def test_device_buffer_read_after_async_run_log():
    """run_log(sync=False) leaves the epoch kernels in flight on the handle's
    non-blocking stream; DeviceBuffer.read (uwvk_memcpy_d2h: waits for all
    device work) and DeviceBuffer.read(stream=...) (ordered on that stream)
    must both return the finished accept counts, equal to a synchronous run."""
    B, E = 65536, 400  # ~40 ms of kernel work queued before the reads
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C4", dropout_on=0.3, dropout_off=0.1)
    counts = []
    for mode in ("sync", "async_device", "async_stream"):
        f = engine.PoseUKFBatch(B)
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, 1e-3)
        d = f.upload_log(log)
        acc = engine.DeviceBuffer(np.zeros((B, 4), np.uint32))
        f.run_log(d, accept_counts=acc, sync=(mode == "sync"))
        counts.append(acc.read(np.uint32, (B, 4), stream=f.stream if mode == "async_stream" else None))
        f.synchronize()
    assert counts[0].sum() > 0
    np.testing.assert_array_equal(counts[1], counts[0])
    np.testing.assert_array_equal(counts[2], counts[0])


def test_split_timer_and_stats_after_async_run_log():
    """bench.py's timed region: timer_mark records the stop event without a
    host wait, the statistics kernels queue behind the epoch launch on the
    same stream, and timer_elapsed waits for the event.  The statistics equal
    those of the blocking sequence (timer_stop, then ensemble_stats) bitwise."""
    B, E = 4096, 60
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    truth = log["truth"].state(E, 53)
    out = []
    for split in (False, True):
        f = engine.PoseUKFBatch(B)
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, log["dt"])
        d = f.upload_log(log)
        f.synchronize()
        f.timer_start()
        f.run_log(d, sync=not split)
        if split:
            f.timer_mark()
            st = f.ensemble_stats(truth)
            ms = f.timer_elapsed()
        else:
            ms = f.timer_stop()
            st = f.ensemble_stats(truth)
        assert ms > 0.0
        out.append(st)
    np.testing.assert_array_equal(out[1], out[0])
    assert out[0][-1] == 0.0 and np.isfinite(out[0]).all()
