"""GPU parity of the two-instances-per-wavefront PSP epoch kernel
(UWVK_OPT_PAIR, k_psp2_epoch, uwvk_psp2_dev.hpp): the row phases of a pair's
two instances run one after the other over 64 lanes, the sigma-point phases
side by side in the two 32-lane halves.  Same algorithm as
k_psp_epoch, different summation order: equal to the oracle at the
test_gpu_parity.py tolerances, on both SO3 sides and both state sizes, in C3
logs (every launch paired) and C4 logs (pressure epochs send their launch to
the one-instance kernel, efforts epochs to theirs, so the state crosses
between the kernels several times per log); NaN measurements of one instance
of a pair leave the other's update intact; an odd batch runs unpaired."""
import numpy as np
import pytest

import oracle_ctypes as O
from helpers import cov_err, pose_setup, state_err

pytestmark = pytest.mark.gpu

TOL_LOG = 1e-7


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


def _engine(eng, batch, dof, cfg, uwv, log, right=True, pair=True):
    g = eng.PoseUKFBatch(batch, dof)
    g.set_so3_right(right)
    g.set_pair(pair)
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    return g


def _oracle(batch, dof, cfg, uwv, log, right=True):
    with O.so3_side(right):
        o = O.OraclePoseBatch(batch, dof)
        o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        o.set_process_noise_from_config(cfg, 1e-3)
    return o


def _close(xg, Pg, xo, Po, dof, tol):
    assert np.all(np.isfinite(xg)) and np.all(np.isfinite(Pg))
    se, ce = state_err(xg, xo, Po, dof).max(), cov_err(Pg, Po).max()
    assert se < tol and ce < tol, (se, ce)


@pytest.mark.parametrize("side", ["right", "left"])
@pytest.mark.parametrize("dof,mode,epochs,batch", [(53, "C3", 400, 4), (26, "C3", 400, 6),
                                                   (53, "C4", 1000, 4), (26, "C4", 600, 2)])
def test_pair_run_log_oracle(eng, dof, mode, epochs, batch, side):
    right = side == "right"
    cfg, uwv, log = pose_setup(batch, dof, mode, epochs)
    o = _oracle(batch, dof, cfg, uwv, log, right)
    g = _engine(eng, batch, dof, cfg, uwv, log, right)
    with O.so3_side(right):
        counts_o = o.run_log(log)
        xo, Po = o.get_state()
    acc = eng.DeviceBuffer(np.zeros((batch, 4), np.uint32))
    g.run_log(g.upload_log(log), accept_counts=acc)
    np.testing.assert_array_equal(counts_o, acc.read(np.uint32, (batch, 4)))
    assert not g.get_status().any()
    xg, Pg = g.get_state()
    _close(xg, Pg, xo, Po, dof, TOL_LOG)


def test_pair_split_calls_and_long_launch(eng):
    """1500 C3 epochs as three run_log calls (the pair kernel's fold every
    1024 epochs inside the long one), against the oracle."""
    B, dof = 4, 53
    cfg, uwv, log = pose_setup(B, dof, "C3", 1500)
    o = _oracle(B, dof, cfg, uwv, log)
    g = _engine(eng, B, dof, cfg, uwv, log)
    o.run_log(log)
    dlog = g.upload_log(log)
    for first, count in ((0, 7), (7, 1100), (1107, 393)):
        g.run_log(dlog, first=first, count=count)
    xo, Po = o.get_state()
    xg, Pg = g.get_state()
    _close(xg, Pg, xo, Po, dof, TOL_LOG)


def test_pair_nan_one_instance(eng):
    """NaN gyro / acceleration / DVL samples of instance 1 (pair 0's second
    half) and instance 2 (pair 1's first): both flagged UWVK_ST_NAN, the
    paired partners (0, 3) and the flagged instances agree with the unpaired
    kernel's result on the same log."""
    B, dof = 4, 53
    cfg, uwv, log = pose_setup(B, dof, "C3", 1000)  # DVL at 5 Hz: 5 samples
    log = dict(log)
    for key in ("gyro", "acc", "dvl"):
        log[key] = np.array(log[key], copy=True)
    log["gyro"][40, 1, 0] = np.nan
    log["acc"][41, 1, 2] = np.nan
    log["acc"][120, 2, 1] = np.nan
    log["dvl"][1, 2, 0] = np.nan
    log["dvl"][3, 1, 1] = np.nan
    res = []
    for pair in (False, True):
        g = _engine(eng, B, dof, cfg, uwv, log, pair=pair)
        acc = eng.DeviceBuffer(np.zeros((B, 4), np.uint32))
        g.run_log(g.upload_log(log), accept_counts=acc)
        res.append((g.get_state(), g.get_status(), acc.read(np.uint32, (B, 4))))
    (x0, P0), st0, c0 = res[0]
    (x1, P1), st1, c1 = res[1]
    np.testing.assert_array_equal(st0, st1)
    assert st1[1] and st1[2] and not st1[0] and not st1[3]
    np.testing.assert_array_equal(c0, c1)
    _close(x1, P1, x0, P0, dof, 1e-9)


@pytest.mark.parametrize("batch", [4096, 4097])
def test_pair_against_unpaired_at_scale(eng, batch):
    """A 4096-instance C3 log (2048 pairs: a full grid of pair workgroups), paired
    and unpaired, to rounding; 4097 (odd) runs unpaired, bitwise the default."""
    dof = 53
    cfg, uwv, log = pose_setup(batch, dof, "C3", 100)
    out = []
    for pair in (False, True):
        g = _engine(eng, batch, dof, cfg, uwv, log, pair=pair)
        g.run_log(g.upload_log(log))
        assert not g.get_status().any()
        out.append(g.get_state())
    (x0, P0), (x1, P1) = out
    if batch % 2:
        np.testing.assert_array_equal(x0, x1)
        np.testing.assert_array_equal(P0, P1)
    else:
        _close(x1, P1, x0, P0, dof, 1e-9)
