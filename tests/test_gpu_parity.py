"""GPU parity: the HIP engine (libuwvk.so, via the C ABI) against the CPU
oracle (oracle/liboracle.so) on identical seeded synthetic inputs.

Tolerance (fp64, north_star "stated float tolerance"): mean errors in units of
the oracle's standard deviation, covariance errors relative to
sqrt(P_ii P_jj).  Single steps: 1e-9; multi-epoch logs: 1e-7 (summation-order
and FMA-contraction differences accumulate through the recursion).
"""
import numpy as np
import pytest

from helpers import cov_err, init_both, pose_setup, state_err

pytestmark = pytest.mark.gpu

TOL_STEP = 1e-9
TOL_LOG = 1e-7


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


@pytest.fixture(scope="module")
def orc():
    import oracle_ctypes
    return oracle_ctypes


# engine paths: "psp" (default, partitioned sigma points), "dense" (all 2n+1
# points, exact apply_delta identity), "literal" (dense + ukfom's re-spread)
PATHS = ["psp", "dense", "literal"]


def _pair(eng, orc, batch, dof=53, mode="C3", epochs=10, path="psp"):
    cfg, uwv, log = pose_setup(batch, dof, mode, epochs)
    o = orc.OraclePoseBatch(batch, dof)
    g = eng.PoseUKFBatch(batch, dof)
    if path == "dense":
        g.set_dense_sigma(True)
    elif path == "literal":
        g.set_literal_apply_delta(True)
    init_both(o, g, cfg, uwv, log)
    return cfg, uwv, log, o, g


def _check(o, g, dof, tol):
    xo, Po = o.get_state()
    xg, Pg = g.get_state()
    se = state_err(xg, xo, Po, dof)
    ce = cov_err(Pg, Po)
    assert np.all(np.isfinite(xg)) and np.all(np.isfinite(Pg))
    assert se.max() < tol, "state error %g" % se.max()
    assert ce.max() < tol, "covariance error %g" % ce.max()
    return se.max(), ce.max()


@pytest.mark.parametrize("path", ["psp", "dense"])
@pytest.mark.parametrize("dof", [53, 26])
def test_init_and_predict(eng, orc, dof, path):
    cfg, uwv, log, o, g = _pair(eng, orc, 6, dof, path=path)
    _check(o, g, dof, 1e-15)
    for f in (o, g):
        f.set_rotation_rate(log["gyro"][0])
        f.predict(1e-3)
    _check(o, g, dof, TOL_STEP)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("dof", [53, 26])
@pytest.mark.parametrize("kind", ["acceleration", "velocity", "pressure", "water_velocity", "xy", "z",
                                  "efforts", "efforts_vel", "geographic", "delayed_xy"])
def test_single_update(eng, orc, dof, kind, path):
    cfg, uwv, log, o, g = _pair(eng, orc, 5, dof, path=path)
    for f in (o, g):
        f.set_rotation_rate(log["gyro"][0])
        f.predict(1e-3)
    B = 5
    x, _ = o.get_state()
    rng = np.random.default_rng(7)
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
    elif kind == "geographic":
        from uwvk import synth
        lat = synth.LAT0 + (x[:, 0] + rng.standard_normal(B)) / 6.39e6
        lon = synth.LON0 - (x[:, 1] + rng.standard_normal(B)) / 3.84e6
        mu, cov = np.stack([lat, lon], 1), np.eye(2) * 4.0
        extra = np.array([0.5, 0.0, -0.2])
    ao = o.update(kind, mu, cov, extra=extra, only_vel=only_vel)
    ag = g.update(kind, mu, cov, extra=extra, only_vel=only_vel)
    np.testing.assert_array_equal(ao, ag)
    _check(o, g, dof, TOL_STEP)


@pytest.mark.parametrize("dof,mode,epochs,path", [(53, "C3", 400, "psp"), (26, "C3", 400, "psp"),
                                                  (53, "C4", 1000, "psp"), (26, "C4", 1000, "psp"),
                                                  (53, "C3", 400, "dense"), (53, "C4", 1000, "dense"),
                                                  (53, "C3", 400, "literal"), (53, "C4", 1000, "literal")])
def test_run_log(eng, orc, dof, mode, epochs, path):
    """C3 over 400 epochs (IMU + 2 DVL), C4 over 1000 (IMU, 5 DVL, 10 pressure,
    1 ADCP x 4 cells); at the default 30 s / 10 s cycle the 1 s of C4 holds no
    drop-out, so no BodyEfforts epoch: the efforts split is covered by
    test_run_log_long_single_launch and the golden pose_c4* fixtures."""
    cfg, uwv, log, o, g = _pair(eng, orc, 4, dof, mode, epochs, path=path)
    counts_o = o.run_log(log)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((4, 4), np.uint32))
    g.run_log(dlog, accept_counts=acc)
    counts_g = acc.read(np.uint32, (4, 4))
    np.testing.assert_array_equal(counts_o, counts_g)
    assert not g.get_status().any()
    _check(o, g, dof, TOL_LOG)


@pytest.mark.parametrize("groups,B", [(0, 16), (1, 16), (1, 13), (-1, 70)])
def test_velocity_ukf(eng, orc, groups, B):
    """run_log on both kernel layouts: one filter per lane (0) and one per
    16-lane row (1, incl. a batch that leaves a partial wave); -1 = auto."""
    from uwvk import synth
    log = synth.make_vel_log(B, 600)
    uwv = synth.default_uwv()
    o = orc.OracleVelBatch(B)
    g = eng.VelocityUKFBatch(B)
    g.set_lane_groups(groups)
    for f in (o, g):
        f.init(log["x0"], log["P0"])
        f.set_gyro(log["gyro"][0])
        f.setup_motion_model(uwv)
    o.run_log(log)
    g.run_log(g.upload_log(log))
    xo, Po, mo = o.get_state(model=True)
    xg, Pg, mg = g.get_state(model=True)
    sd = np.sqrt(np.diagonal(Po, axis1=1, axis2=2))
    assert np.max(np.abs(xg - xo) / sd) < TOL_LOG
    assert cov_err(Pg, Po).max() < TOL_LOG
    assert np.max(np.abs(mg - mo)) < 1e-9


@pytest.mark.parametrize("groups", [0, 1])
def test_velocity_ukf_process_noise(eng, orc, groups):
    """setProcessNoiseCovariance [EXT base] with a full 4x4 Q (incl. z and couplings)."""
    from uwvk import synth
    B = 9
    log = synth.make_vel_log(B, 300)
    A = np.array([[2e-2, 1e-3, 0, 0], [0, 1e-2, 2e-3, 0], [0, 0, 1e-2, 0], [1e-3, 0, 0, 5e-3]])
    Q = A @ A.T
    o, g = orc.OracleVelBatch(B), eng.VelocityUKFBatch(B)
    g.set_lane_groups(groups)
    for f in (o, g):
        f.init(log["x0"], log["P0"])
        f.set_process_noise(Q)
        f.set_gyro(log["gyro"][0])
        f.setup_motion_model(synth.default_uwv())
    o.run_log(log)
    g.run_log(g.upload_log(log))
    (xo, Po), (xg, Pg) = o.get_state(), g.get_state()
    sd = np.sqrt(np.diagonal(Po, axis1=1, axis2=2))
    assert np.max(np.abs(xg - xo) / sd) < TOL_LOG
    assert cov_err(Pg, Po).max() < TOL_LOG


@pytest.mark.parametrize("groups", [0, 1])
def test_velocity_ukf_model_change_between_runs(eng, orc, groups):
    """The VelocityUKF kernels read the model parameters from the handle's
    device copy (VEL_SMEM): setupMotionModel (VelocityUKF.cpp:65-74) and
    setProcessNoiseCovariance between two run_log calls must reach the second
    run.  The second model has off-diagonal inertia / damping couplings (every
    entry of the 6x6 matrices is used) and unequal weight / buoyancy with
    general centres, and the single-call predict after it goes through
    k_vel_predict."""
    from uwvk import abi, synth
    B = 12
    log = synth.make_vel_log(B, 400)
    uwv2 = synth.default_uwv()
    M, Dl, Dq = synth.uwv_arrays(uwv2)
    C = np.zeros((6, 6))
    C[0, 4] = C[4, 0] = 8.0
    C[1, 3] = C[3, 1] = -6.0
    C[2, 5] = C[5, 2] = 3.0
    abi.fill(uwv2.inertia_matrix, (M * 1.3 + C).ravel())
    abi.fill(uwv2.damping_matrices[0], (Dl * 0.7 + 0.5 * C).ravel())
    abi.fill(uwv2.damping_matrices[1], (Dq * 1.5 + 0.25 * np.abs(C)).ravel())
    # unequal weight / buoyancy and general centres (the default model has
    # W = B and cog = 0): every term of the restoring forces, which the kernels
    # evaluate through one rotation (VEL_GLIN, uwvk_vel.hip v_deriv)
    uwv2.weight, uwv2.buoyancy = 2100.0, 1950.0
    abi.fill(uwv2.distance_body2centerofgravity, [0.02, -0.01, 0.03])
    abi.fill(uwv2.distance_body2centerofbuoyancy, [0.01, 0.015, 0.06])
    Q2 = np.diag([3e-2, 2e-2, 1e-2, 4e-3])
    o, g = orc.OracleVelBatch(B), eng.VelocityUKFBatch(B)
    g.set_lane_groups(groups)
    for f in (o, g):
        f.init(log["x0"], log["P0"])
        f.set_gyro(log["gyro"][0])
        f.setup_motion_model(synth.default_uwv())
    o.run_log(log, 0, 200)
    dlog = g.upload_log(log)
    g.run_log(dlog, 0, 200)
    for f in (o, g):
        f.setup_motion_model(uwv2)
        f.set_process_noise(Q2)
    o.run_log(log, 200, 199)
    g.run_log(dlog, 200, 199)
    for f in (o, g):
        f.set_gyro(log["gyro"][399])
        f.set_efforts(log["efforts"][399])
        f.predict(log["dt"])
    (xo, Po, mo), (xg, Pg, mg) = o.get_state(model=True), g.get_state(model=True)
    sd = np.sqrt(np.diagonal(Po, axis1=1, axis2=2))
    assert np.max(np.abs(xg - xo) / sd) < TOL_LOG
    assert cov_err(Pg, Po).max() < TOL_LOG
    assert np.max(np.abs(mg - mo)) < 1e-9
    # the change mattered: the default model over the same log ends elsewhere
    d = eng.VelocityUKFBatch(B)
    d.set_lane_groups(groups)
    d.init(log["x0"], log["P0"])
    d.set_gyro(log["gyro"][0])
    d.setup_motion_model(synth.default_uwv())
    d.run_log(d.upload_log(log), 0, 399)
    assert np.max(np.abs(d.get_state()[0] - xo) / sd) > 1e-3


def test_velocity_ukf_api(eng, orc):
    from uwvk import synth
    B = 8
    log = synth.make_vel_log(B, 10)
    uwv = synth.default_uwv()
    o = orc.OracleVelBatch(B)
    g = eng.VelocityUKFBatch(B)
    for f in (o, g):
        f.init(log["x0"], log["P0"])
    with pytest.raises(eng.UWVKError):
        g.predict(1e-3)  # VelocityUKF.cpp:117-118: no motion model -> error
    for f in (o, g):
        f.setup_motion_model(uwv)
        f.set_gyro(log["gyro"][0])
        f.set_efforts(log["efforts"][0])
        f.predict(1e-3)
        f.update_dvl(np.array([[1.0, 0.02, -0.01]] * B), log["dvl_cov"])
        f.update_pressure(np.full(B, -10.02), log["pressure_cov"])
    xo, Po = o.get_state()
    xg, Pg = g.get_state()
    sd = np.sqrt(np.diagonal(Po, axis1=1, axis2=2))
    assert np.max(np.abs(xg - xo) / sd) < TOL_STEP
    assert cov_err(Pg, Po).max() < TOL_STEP


def test_nan_measurement_rejected(eng):
    from uwvk import synth
    cfg, uwv, log = pose_setup(3)
    g = eng.PoseUKFBatch(3)
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    x0, P0 = g.get_state()
    bad = log["acc"][0].copy()
    bad[1, 2] = np.nan
    with pytest.raises(eng.UWVKError) as e:
        g.update("acceleration", bad, log["acc_cov"])
    assert e.value.code == 2
    x1, P1 = g.get_state()
    np.testing.assert_array_equal(x0, x1)
    np.testing.assert_array_equal(P0, P1)


def test_run_log_long_single_launch(eng, orc):
    """3000 C4 epochs in ONE run_log call: exercises the PSP kernel's periodic
    fold of the time scale (every 1024 epochs) and the efforts-epoch split.  The
    drop-out cycle is compressed (0.5 s on / 0.25 s off) so that the 3 s hold
    DVL drop-outs and their BodyEfforts epochs (the default 30 s / 10 s cycle
    would hold none)."""
    from uwvk import abi, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(3, 3000, "C4", dropout_on=0.5, dropout_off=0.25)
    n_eff = int(((log["flags"] & abi.EV_EFFORTS) != 0).sum())
    assert n_eff >= 8, n_eff  # the launch really splits at efforts epochs, before and after the fold
    assert ((log["flags"][1024:] & abi.EV_EFFORTS) != 0).any()
    o = orc.OraclePoseBatch(3, 53)
    g = eng.PoseUKFBatch(3, 53)
    init_both(o, g, cfg, uwv, log)
    counts_o = o.run_log(log)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((3, 4), np.uint32))
    g.run_log(dlog, accept_counts=acc)
    np.testing.assert_array_equal(counts_o, acc.read(np.uint32, (3, 4)))
    assert not g.get_status().any()
    _check(o, g, 53, TOL_LOG)


def test_run_log_device_flags_only(eng, orc):
    """run_log without the host copy of the flags (the engine reads them back)."""
    cfg, uwv, log, o, g = _pair(eng, orc, 3, 53, "C4", 600)
    o.run_log(log)
    dlog = g.upload_log(log)
    dlog.s.host_flags = None
    g.run_log(dlog)
    _check(o, g, 53, TOL_LOG)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("groups,B", [(1, 4096), (0, 8192)])
def test_velocity_ukf_config_batch(eng, orc, groups, B):
    """Config C2 at its size (VelocityUKF.cpp:6-130): 4,096 instances over
    2,000 epochs through the 16-lane-row kernel (k_vel_epoch_g), and the
    lane-per-filter kernel (k_vel_epoch) at a larger batch.  16 instances
    spread over the batch are checked against the oracle, each generated ALONE
    (its own one-instance log: counter-based noise, so the same numbers), and
    a second run of the whole batch is bitwise equal."""
    from uwvk import synth
    E = 2000
    uwv = synth.default_uwv()
    log = synth.make_vel_log(B, E)
    runs = []
    for _ in range(2):
        g = eng.VelocityUKFBatch(B)
        g.set_lane_groups(groups)
        g.init(log["x0"], log["P0"])
        g.set_gyro(log["gyro"][0])
        g.setup_motion_model(uwv)
        g.run_log(g.upload_log(log))
        runs.append(g.get_state(model=True))
    for a, b in zip(*runs):
        np.testing.assert_array_equal(a, b)
    xg, Pg, mg = runs[0]
    picks = np.unique(np.linspace(0, B - 1, 16).astype(int))
    for i in picks:
        li = synth.make_vel_log(1, E, first_instance=int(i))
        np.testing.assert_array_equal(li["gyro"][:, 0], log["gyro"][:, i])
        o = orc.OracleVelBatch(1)
        o.init(li["x0"], li["P0"])
        o.set_gyro(li["gyro"][0])
        o.setup_motion_model(uwv)
        o.run_log(li)
        xo, Po, mo = o.get_state(model=True)
        sd = np.sqrt(np.diagonal(Po, axis1=1, axis2=2))
        assert np.max(np.abs(xg[i] - xo[0]) / sd[0]) < TOL_LOG, i
        assert cov_err(Pg[i:i + 1], Po).max() < TOL_LOG, i
        assert np.max(np.abs(mg[i] - mo[0])) < 1e-9, i
