"""Two independent CPU restatements agree: the C oracle (oracle/uwvk_oracle.c)
and the numpy twin (oracle/numpy_twin.py) on seeded single-filter trajectories.
Agreement to ~1e-12 is the guard against a restatement bug in either one
(the reference itself cannot run here: SURVEY.md K3/K4)."""
import numpy as np
import pytest

import numpy_twin as T
import oracle_ctypes as O
from helpers import cov_err, state_err
from uwvk import synth

TOL = 1e-10


@pytest.fixture(params=["right", "left"])
def side(request):
    """Both SO3 [+] sides (right, MTK's q exp(d), is the default; left is the
    option): the oracle's process-wide switch and the twin's module switch."""
    right = request.param == "right"
    prev = T.SO3_RIGHT
    T.SO3_RIGHT = right
    with O.so3_side(right):
        yield request.param
    T.SO3_RIGHT = prev


def _pair(dof, mode="C3", epochs=50, seed=synth.SEED):
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(1, epochs, mode=mode, seed=seed, dof=dof)
    o = O.OraclePoseBatch(1, dof)
    o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o.set_process_noise_from_config(cfg, log["dt"])
    t = T.PoseTwin.from_config(dof, log["pos0"][0], log["pos_cov"][0], log["rot0"][0], log["rot_cov"][0],
                               T.cfg_dict(cfg), T.UWV.from_abi(uwv))
    t.set_noise_from_config(T.cfg_dict(cfg), log["dt"])
    return log, o, t


def _cmp(o, t, dof, tol=TOL):
    xo, Po = o.get_state()
    se = state_err(t.mu[None], xo, Po, dof)
    ce = cov_err(t.P[None], Po)
    assert se.max() < tol and ce.max() < tol, (se.max(), ce.max())


@pytest.mark.parametrize("dof", [53, 26])
def test_init_and_noise_identical(dof):
    log, o, t = _pair(dof)
    xo, Po = o.get_state()
    np.testing.assert_allclose(t.mu, xo[0], rtol=0, atol=1e-15)
    np.testing.assert_allclose(t.P, Po[0], rtol=0, atol=1e-18)


@pytest.mark.parametrize("dof", [53, 26])
def test_predict_and_updates(dof, side):
    log, o, t = _pair(dof)
    for e in range(40):
        o.set_rotation_rate(log["gyro"][e])
        t.w = log["gyro"][e][0]
        o.predict(log["dt"])
        t.predict(log["dt"])
        o.update("acceleration", log["acc"][e], log["acc_cov"])
        t.update("acceleration", log["acc"][e][0], log["acc_cov"])
    _cmp(o, t, dof)
    x, _ = o.get_state()
    rng = np.random.default_rng(1)
    cases = [("velocity", x[0, 7:10] + 0.01, np.eye(3) * 1e-4, None),
             ("pressure", np.array([101325.0 + 9.81 * 1025 * 10.2]), np.array([[1e4]]), np.array([0.1, 0, 0.2])),
             ("water_velocity", np.array([0.9, -0.1]), np.eye(2) * 0.05 ** 2, 0.5),
             ("xy", x[0, 0:2] + 0.5, np.eye(2) * 0.5, None),
             ("z", x[0, 2:3] - 0.1, np.array([[0.01]]), None),
             ("delayed_xy", x[0, 0:2] + 0.2, np.eye(2) * 0.5, x[0, 0:2] - 0.1),
             ("efforts", 10 * rng.standard_normal(6), np.diag([25.0, 25, 25, 1, 1, 1]), None)]
    for kind, z, R, extra in cases:
        ao = o.update(kind, z[None], R, extra=extra if kind != "delayed_xy" else extra[None])
        at = t.update(kind, z, R, extra=extra)
        assert bool(ao[0]) == bool(at), kind
        _cmp(o, t, dof)


@pytest.mark.parametrize("dof", [53])
def test_constrain_velocity_after_efforts(dof, side):
    log, o, t = _pair(dof)
    rng = np.random.default_rng(3)
    for e in range(5):
        o.set_rotation_rate(log["gyro"][e])
        t.w = log["gyro"][e][0]
        o.predict(log["dt"])
        t.predict(log["dt"])
    R = np.diag([25.0, 25, 25, 1, 1, 1])
    for k in range(3):
        z = 10 * rng.standard_normal(6)
        o.update("efforts", z[None], R, only_vel=0)
        t.update("efforts", z, R, only_vel=False)
        z = 10 * rng.standard_normal(6)
        o.update("efforts", z[None], R, only_vel=1)
        t.update("efforts", z, R, only_vel=True)
        _cmp(o, t, dof)


def test_geographic_and_gate(side):
    log, o, t = _pair(53)
    x, _ = o.get_state()
    lat, lon = T.nav_to_world(t.loc, x[0, 0] + 0.3, x[0, 1] - 0.4)
    z = np.array([lat, lon])
    ao = o.update("geographic", z[None], np.eye(2) * 4.0, extra=np.array([0.5, 0.0, -0.2]))
    at = t.update("geographic", z, np.eye(2) * 4.0, extra=np.array([0.5, 0.0, -0.2]))
    assert ao[0] == at == 1
    _cmp(o, t, 53)
    lat, lon = T.nav_to_world(t.loc, x[0, 0] + 300.0, x[0, 1])  # far outlier: d2p95 gate rejects
    ao = o.update("geographic", np.array([[lat, lon]]), np.eye(2) * 4.0)
    at = t.update("geographic", np.array([lat, lon]), np.eye(2) * 4.0)
    assert ao[0] == at == 0
    _cmp(o, t, 53)


@pytest.mark.parametrize("mode", ["C3", "C4"])
def test_run_log_matches_twin(mode, side):
    epochs = 300 if mode == "C3" else 1100
    log, o, t = _pair(53, mode, epochs)
    o.run_log(log)
    for e in range(epochs):
        t.w = log["gyro"][e][0]
        t.predict(log["dt"])
        f = log["flags"][e]
        t.update("acceleration", log["acc"][e][0], log["acc_cov"])
        if f & 2:
            t.update("velocity", log["dvl"][log["dvl_index"][e]][0], log["dvl_cov"])
        if f & 4:
            t.update("pressure", log["pressure"][log["pressure_index"][e]][:1], np.array([[log["pressure_cov"]]]),
                     extra=log["pressure_sensor_in_imu"])
        if f & 8:
            for c in range(log["adcp_cells"]):
                t.update("water_velocity", log["adcp"][log["adcp_index"][e]][c][0], log["adcp_cov"],
                         extra=log["adcp_cell_weighting"][c])
        if f & 16:
            t.update("efforts", log["efforts"][log["efforts_index"][e]][0], log["efforts_cov"], only_vel=bool(f & 32))
    _cmp(o, t, 53, tol=1e-8)


def test_velocity_ukf_twin():
    uwv = synth.default_uwv()
    log = synth.make_vel_log(1, 400)
    o = O.OracleVelBatch(1)
    o.init(log["x0"], log["P0"])
    o.set_gyro(log["gyro"][0])
    o.setup_motion_model(uwv)
    t = T.VelTwin(log["x0"][0], log["P0"][0], T.UWV.from_abi(uwv))
    t.set_gyro(log["gyro"][0][0])
    o.run_log(log)
    for e in range(log["epochs"]):
        t.set_gyro(log["gyro"][e][0])
        t.tau = log["efforts"][e][0]
        t.predict(log["dt"])
        if log["flags"][e] & 2:
            t.update_dvl(log["dvl"][log["dvl_index"][e]][0], log["dvl_cov"])
        if log["flags"][e] & 4:
            t.update_pressure(log["pressure"][log["pressure_index"][e]][0], log["pressure_cov"])
    xo, Po, mo = o.get_state(model=True)
    sd = np.sqrt(np.diag(Po[0]))
    assert np.max(np.abs(t.mu - xo[0]) / sd) < 1e-9
    assert cov_err(t.P[None], Po).max() < 1e-9
    np.testing.assert_allclose(t.model, mo[0], rtol=0, atol=1e-12)
