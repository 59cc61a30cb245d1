"""GPU parity on both sides of the SO3 boxplus, the largest unpinned semantic
(SURVEY 8(c) item 5): right, q exp(d) -- MTK's SO3::boxplus and the default
since r05 (PoseState.hpp:15, PoseUKF.cpp:32) -- and left, exp(d) q, the
option.  The engine with UWVK_OPT_SO3_RIGHT = side against the oracle under
or_set_so3_right(side), for the predict, every update kind and multi-epoch
logs, on all three engine paths: psp (the default: the SR instantiations of
the PSP kernels, with apply_delta's T = R(exp d)^T on the right, R(exp d) on
the left), dense (the literal kernels) and literal (the
literal kernels with ukfom's literal apply_delta re-spread).  Tolerances as in
test_gpu_parity.py."""
import numpy as np
import pytest

import oracle_ctypes as O
from helpers import cov_err, pose_setup, state_err

pytestmark = pytest.mark.gpu

TOL_STEP = 1e-9
TOL_LOG = 1e-7


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


class SideOracle:
    """OraclePoseBatch whose every call runs with the given boxplus side (the
    oracle's switch is process-wide: set for the call, restored after)."""

    def __init__(self, right, *a):
        self.right = right
        self.o = O.OraclePoseBatch(*a)

    def __getattr__(self, name):
        fn = getattr(self.o, name)

        def call(*a, **k):
            with O.so3_side(self.right):
                return fn(*a, **k)
        return call


PATHS = ["psp", "dense", "literal"]
SIDES = ["right", "left"]


def _pair(eng, batch, dof, mode="C3", epochs=10, path="psp", side="right"):
    cfg, uwv, log = pose_setup(batch, dof, mode, epochs)
    right = side == "right"
    o = SideOracle(right, batch, dof)
    g = eng.PoseUKFBatch(batch, dof)
    g.set_so3_right(right)
    if path == "dense":
        g.set_dense_sigma(True)
    elif path == "literal":
        g.set_literal_apply_delta(True)
    for f in (o, g):
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, 1e-3)
    return cfg, uwv, log, o, g


def _check(o, g, dof, tol):
    (xo, Po), (xg, Pg) = o.get_state(), g.get_state()
    assert np.all(np.isfinite(xg)) and np.all(np.isfinite(Pg))
    se, ce = state_err(xg, xo, Po, dof).max(), cov_err(Pg, Po).max()
    assert se < tol and ce < tol, (se, ce)


@pytest.mark.parametrize("side", SIDES)
@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("dof", [53, 26])
def test_predict_side(eng, dof, path, side):
    cfg, uwv, log, o, g = _pair(eng, 6, dof, path=path, side=side)
    for k in range(3):
        for f in (o, g):
            f.set_rotation_rate(log["gyro"][k])
            f.predict(1e-3)
    _check(o, g, dof, TOL_STEP)


@pytest.mark.parametrize("side", SIDES)
@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("kind", ["acceleration", "velocity", "pressure", "water_velocity", "xy", "z", "efforts",
                                  "efforts_vel", "geographic", "delayed_xy"])
def test_single_update_side(eng, kind, path, side):
    dof, B = 53, 5
    cfg, uwv, log, o, g = _pair(eng, B, dof, path=path, side=side)
    for f in (o, g):
        f.set_rotation_rate(log["gyro"][0])
        f.predict(1e-3)
    x, _ = o.get_state()
    rng = np.random.default_rng(11)
    extra, only_vel = None, 0
    if kind == "acceleration":
        mu, cov = log["acc"][0], log["acc_cov"]
    elif kind == "velocity":
        mu, cov = x[:, 7:10] + 0.01 * rng.standard_normal((B, 3)), np.eye(3) * 1e-4
    elif kind == "pressure":
        mu, cov = (101325.0 + 10.0 * 9.81 * 1025 + 50 * rng.standard_normal(B))[:, None], np.array([[1e4]])
        extra = np.array([0.1, -0.2, 0.3])
    elif kind == "water_velocity":
        mu, cov = 0.3 * rng.standard_normal((B, 2)), np.eye(2) * 0.05 ** 2
        extra = np.array([0.0, 0.25, 0.5, 0.75, 1.0])
    elif kind in ("xy", "delayed_xy"):
        mu, cov = x[:, 0:2] + rng.standard_normal((B, 2)), np.eye(2) * 0.5
        if kind == "delayed_xy":
            extra = x[:, 0:2] - 0.3
    elif kind == "z":
        mu, cov = x[:, 2:3] + 0.1 * rng.standard_normal((B, 1)), np.array([[0.01]])
    elif kind in ("efforts", "efforts_vel"):
        mu, cov = 20 * rng.standard_normal((B, 6)), np.diag([25.0, 25, 25, 1, 1, 1])
        only_vel = 1 if kind == "efforts_vel" else 0
        kind = "efforts"
    else:  # geographic
        from uwvk import synth
        lat = synth.LAT0 + (x[:, 0] + rng.standard_normal(B)) / 6.39e6
        lon = synth.LON0 - (x[:, 1] + rng.standard_normal(B)) / 3.84e6
        mu, cov = np.stack([lat, lon], 1), np.eye(2) * 4.0
        extra = np.array([0.5, 0.0, -0.2])
    np.testing.assert_array_equal(o.update(kind, mu, cov, extra=extra, only_vel=only_vel),
                                  g.update(kind, mu, cov, extra=extra, only_vel=only_vel))
    _check(o, g, dof, TOL_STEP)


@pytest.mark.parametrize("side", SIDES)
@pytest.mark.parametrize("dof,mode,epochs,path", [(53, "C3", 400, "psp"), (26, "C3", 400, "psp"),
                                                  (53, "C4", 1000, "psp"), (26, "C4", 1000, "psp"),
                                                  (53, "C3", 400, "dense"), (26, "C3", 400, "dense"),
                                                  (53, "C4", 1000, "dense"), (53, "C3", 400, "literal")])
def test_run_log_side(eng, dof, mode, epochs, path, side):
    cfg, uwv, log, o, g = _pair(eng, 4, dof, mode, epochs, path=path, side=side)
    counts_o = o.run_log(log)
    acc = eng.DeviceBuffer(np.zeros((4, 4), np.uint32))
    g.run_log(g.upload_log(log), accept_counts=acc)
    np.testing.assert_array_equal(counts_o, acc.read(np.uint32, (4, 4)))
    assert not g.get_status().any()
    _check(o, g, dof, TOL_LOG)


@pytest.mark.parametrize("dense", [False, True])
def test_right_differs_from_left(eng, dense):
    """The switch reaches the kernels: the same 400-epoch C3 log on the left
    and right engine paths differs by far more than the parity tolerance, and
    a fresh handle runs the right side (the default)."""
    cfg, uwv, log = pose_setup(2, 53, "C3", 400)
    xs = []
    for right in (False, True):
        g = eng.PoseUKFBatch(2, 53)
        g.set_dense_sigma(dense)
        g.set_so3_right(right)
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        g.set_process_noise_from_config(cfg, 1e-3)
        g.run_log(g.upload_log(log))
        xs.append(g.get_state())
    assert state_err(xs[1][0], xs[0][0], xs[0][1], 53).max() > 0.1
    d = eng.PoseUKFBatch(2, 53)  # no set_so3_right: the default side
    d.set_dense_sigma(dense)
    d.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    d.set_process_noise_from_config(cfg, 1e-3)
    d.run_log(d.upload_log(log))
    np.testing.assert_array_equal(d.get_state()[0], xs[1][0])


@pytest.mark.parametrize("side", SIDES)
@pytest.mark.parametrize("dof", [53, 26])
def test_visual_landmark_side(eng, dof, side):
    """The marker-augmented visual update (PoseUKF.cpp:613-654) with both SO3
    segments (filter and marker orientation) on the given side, against the
    oracle's same side (aug / sm SEG_SO3R on the right, SEG_SO3 on the left)."""
    from test_small_filters import pose_scene, visual_common
    B = 5
    cfg, uwv, log, o, g = _pair(eng, B, dof, "C3", 60, side=side)
    o.run_log(log)
    g.run_log(g.upload_log(log))
    x0 = o.get_state()[0]
    true_t, true_q, marker, px = pose_scene(x0)
    fcov, fpos, cm, cam, cib = visual_common(B)
    for f in (g, o):
        f.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    _check(o, g, dof, TOL_STEP * 10)
    assert not g.get_status().any()


@pytest.mark.parametrize("side", SIDES)
def test_ensemble_stats_side(eng, side):
    """uwvk_pose_ensemble_stats measures the orientation error on the handle's
    side, log(t^-1 q) (right) or log(q t^-1) (left), like the host reference."""
    from uwvk import ensemble
    B = 130  # two partial rows of 64 plus a remainder
    right = side == "right"
    cfg, uwv, log, o, g = _pair(eng, B, 53, "C3", 50, side=side)
    g.run_log(g.upload_log(log))
    x, P = g.get_state()
    truth = np.array(log["truth"].state(50, 53), dtype=np.float64)
    # a truth orientation far from the identity, where the nav- and body-frame
    # errors differ (the synthetic heading is ~0): 1.2 rad about (0.6, -0.3, 0.74)
    ax = np.array([0.6, -0.3, 0.74]) / np.linalg.norm([0.6, -0.3, 0.74])
    truth[3:7] = np.r_[np.cos(0.6), np.sin(0.6) * ax]
    got = g.ensemble_stats(truth)
    np.testing.assert_allclose(got, ensemble.ensemble_stats_host(x, P, truth, right=right), rtol=1e-9, atol=1e-12)
    other = ensemble.ensemble_stats_host(x, P, truth, right=not right)
    assert not np.allclose(got[2 * 54 + 3:2 * 54 + 6], other[2 * 54 + 3:2 * 54 + 6], rtol=1e-3)
