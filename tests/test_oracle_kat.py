"""Known-answer tests of the CPU oracle: closed-form
results that hold independently of any implementation.  These pin the oracle
(whose own parity against the reference binary is unpinned: K3/K4)."""
import ctypes as C

import numpy as np
import pytest

import oracle_ctypes as O
from uwvk import abi, synth

L = O.lib()
DP = C.POINTER(C.c_double)


def p(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(DP)


def so3_exp(v):
    o = np.zeros(4)
    L.or_so3_exp(p(v), o.ctypes.data_as(DP))
    return o


def so3_log(q):
    o = np.zeros(3)
    L.or_so3_log(p(q), o.ctypes.data_as(DP))
    return o


def test_so3_exp_log_roundtrip():
    rng = np.random.default_rng(0)
    assert np.array_equal(so3_exp(np.zeros(3)), [1, 0, 0, 0])
    for _ in range(200):
        v = rng.standard_normal(3)
        v *= rng.uniform(0, 3.1) / np.linalg.norm(v)
        q = so3_exp(v)
        assert abs(np.linalg.norm(q) - 1) < 1e-15
        np.testing.assert_allclose(so3_log(q), v, rtol=0, atol=1e-13)
        np.testing.assert_allclose(so3_log(-q), v, rtol=0, atol=1e-13)  # double cover


def test_manifold_identities():
    lay = C.create_string_buffer(32 * 4)
    L.or_layout_init(lay, 53)
    rng = np.random.default_rng(1)
    x = rng.standard_normal(54)
    x[3:7] = so3_exp(rng.standard_normal(3) * 0.5)
    out = np.zeros(54)
    d = np.zeros(53)
    L.or_boxplus(lay, p(x), p(np.zeros(53)), C.c_double(1.0), out.ctypes.data_as(DP))
    np.testing.assert_array_equal(out, x)  # x [+] 0 = x
    delta = rng.standard_normal(53) * 0.3
    L.or_boxplus(lay, p(x), p(delta), C.c_double(1.0), out.ctypes.data_as(DP))
    L.or_boxminus(lay, p(out), p(x), d.ctypes.data_as(DP))
    np.testing.assert_allclose(d, delta, rtol=0, atol=1e-13)  # (x [+] d) [-] x = d


def _quat_mul(a, b):
    o = np.zeros(4)
    L.or_quat_mul(p(a), p(b), o.ctypes.data_as(DP))
    return o


def test_so3_side_switch_identities():
    """The default right [+] (q * exp(d), MTK's SO3::boxplus) vs the left [+]
    option (exp(d) * q): each satisfies the manifold identities, and they differ
    exactly by the side the increment multiplies on."""
    lay = C.create_string_buffer(32 * 4)
    L.or_layout_init(lay, 53)
    rng = np.random.default_rng(11)
    x = rng.standard_normal(54)
    x[3:7] = so3_exp(rng.standard_normal(3) * 0.8)
    delta = rng.standard_normal(53) * 0.3
    out_l, out_r, d = np.zeros(54), np.zeros(54), np.zeros(53)
    assert L.or_get_so3_right() == 1
    with O.so3_left():
        assert L.or_get_so3_right() == 0
        L.or_boxplus(lay, p(x), p(delta), C.c_double(1.0), out_l.ctypes.data_as(DP))
        L.or_boxminus(lay, p(out_l), p(x), d.ctypes.data_as(DP))
        np.testing.assert_allclose(d, delta, rtol=0, atol=1e-13)   # (x [+] d) [-] x = d
    assert L.or_get_so3_right() == 1
    L.or_boxplus(lay, p(x), p(delta), C.c_double(1.0), out_r.ctypes.data_as(DP))
    L.or_boxminus(lay, p(out_r), p(x), d.ctypes.data_as(DP))
    np.testing.assert_allclose(d, delta, rtol=0, atol=1e-13)   # (x [+] d) [-] x = d
    L.or_boxplus(lay, p(x), p(np.zeros(53)), C.c_double(1.0), out_r.ctypes.data_as(DP))
    np.testing.assert_array_equal(out_r, x)                     # x [+] 0 = x
    L.or_boxplus(lay, p(x), p(delta), C.c_double(1.0), out_r.ctypes.data_as(DP))
    e = so3_exp(delta[3:6])
    np.testing.assert_allclose(out_l[3:7], _quat_mul(e, x[3:7]), atol=1e-15)
    np.testing.assert_allclose(out_r[3:7], _quat_mul(x[3:7], e), atol=1e-15)
    np.testing.assert_array_equal(np.delete(out_l, range(3, 7)), np.delete(out_r, range(3, 7)))
    assert np.linalg.norm(out_l[3:7] - out_r[3:7]) > 1e-2


def test_so3_side_changes_c3_trajectory():
    """The two [+] conventions give materially different C3 filters (400 epochs,
    2 DVL updates): the side (right by default, MTK's SO3::boxplus) is an
    unpinned choice, not a rounding detail.  Both runs stay finite and positive definite."""
    from helpers import state_err
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(2, 400, "C3")
    res = []
    for right in (False, True):
        o = O.OraclePoseBatch(2, 53)
        with O.so3_side(right):
            o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
            o.set_process_noise_from_config(cfg, log["dt"])
            o.run_log(log)
        x, P = o.get_state()
        assert np.all(np.isfinite(x)) and np.all(np.isfinite(P))
        assert all(np.all(np.linalg.eigvalsh(P[i]) > 0) for i in range(2))
        res.append((x, P))
    (xl, Pl), (xr, Pr) = res
    # after 0.4 s the trajectories differ by ~0.3-0.6 standard deviations: 10^6 x the
    # 1e-7 parity tolerance, so the choice of side is never hidden by the tests
    assert state_err(xr, xl, Pl, 53).max() > 0.1
    assert L.or_get_so3_right() == 1


def test_cholesky():
    rng = np.random.default_rng(2)
    A = rng.standard_normal((53, 53))
    P = A @ A.T + np.diag(np.logspace(-10, 2, 53))
    Lo = np.zeros((53, 53))
    assert L.or_cholesky(53, p(P), Lo.ctypes.data_as(DP)) == 0
    np.testing.assert_allclose(Lo @ Lo.T, P, rtol=1e-13, atol=1e-13 * np.abs(P).max())
    assert np.all(np.triu(Lo, 1) == 0)
    P[5, 5] = -1.0
    assert L.or_cholesky(53, p(P), Lo.ctypes.data_as(DP)) == -1


def _filter(dof=53, block_diag_ori=False):
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(1, 5, dof=dof)
    o = O.OraclePoseBatch(1, dof)
    o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o.set_process_noise_from_config(cfg, 1e-3)
    for e in range(3):
        o.set_rotation_rate(log["gyro"][e])
        o.predict(1e-3)
        o.update("acceleration", log["acc"][e], log["acc_cov"])
    return o, log


def _reinit(o, x, P):
    o2 = O.OraclePoseBatch(1, o.dof)
    param = abi.PoseParameter()
    param.gyro_bias_tau = param.acc_bias_tau = 600.0
    param.inertia_tau = param.lin_damping_tau = param.quad_damping_tau = 3600.0
    param.water_velocity_tau, param.adcp_bias_tau, param.water_density_tau = 900.0, 900.0, 3600.0
    param.atmospheric_pressure = 101325.0
    loc = abi.Location(synth.LAT0, synth.LON0, 0.0)
    o2.init_from_state(x, P, loc, synth.default_uwv(), param)
    return o2


def test_linear_update_equals_kalman_filter():
    """Z_Position update (h linear) with no orientation cross-covariance equals
    the textbook KF: the weight-1/2 unscaled sigma points are exact for linear h
    and delta has no orientation part, so apply_delta leaves Sigma unchanged."""
    o, _ = _filter()
    x, P = o.get_state()
    Pm = P[0].copy()
    for r in range(3, 6):
        for c in range(53):
            if not 3 <= c < 6:
                Pm[r, c] = Pm[c, r] = 0.0
    o2 = _reinit(o, x, Pm[None])
    z, R = np.array([x[0, 2] - 0.37]), np.array([[0.04]])
    o2.update("z", z[None], R)
    x2, P2 = o2.get_state()
    H = np.zeros((1, 53))
    H[0, 2] = 1
    K = Pm @ H.T @ np.linalg.inv(H @ Pm @ H.T + R)
    dx = (K @ (z - x[0, 2:3])).ravel()
    np.testing.assert_allclose(np.delete(x2[0], [3, 4, 5, 6]), np.delete(x[0], [3, 4, 5, 6]) + np.delete(dx, [3, 4, 5]),
                               rtol=1e-12, atol=1e-12)
    assert np.array_equal(x2[0, 3:7], x[0, 3:7])
    scale = np.sqrt(np.outer(np.diag(Pm), np.diag(Pm)))
    assert np.max(np.abs(P2[0] - (Pm - K @ H @ Pm)) / scale) < 1e-11


def test_linear_predict_block():
    """Vector components propagate linearly (PoseUKF.cpp:25,35-78): the
    (p, v, a, biases, params, currents, density) block of the predicted
    covariance equals F Sigma F^T + Q' exactly (up to rounding)."""
    o, log = _filter()
    x, P = o.get_state()
    dt = 1e-3
    n = 53
    F = np.eye(n)
    F[0:3, 6:9] = dt * np.eye(3)
    F[6:9, 9:12] = dt * np.eye(3)
    for d0, tau, k in ((12, 600.0, 3), (15, 600.0, 3), (19, 3600.0, 27), (46, 900.0, 4), (50, 900.0, 2),
                       (52, 3600.0, 1)):
        for i in range(k):
            F[d0 + i, d0 + i] = 1 - dt / tau
    cfg = synth.default_pose_config()
    o.set_rotation_rate(log["gyro"][3])
    vs = x[0, 7:10] * np.array([1, 1, 10])
    o.predict(dt)
    x2, P2 = o.get_state()
    Q = np.zeros((n, n))
    O.lib().or_pose_set_process_noise_from_config  # noqa: B018 (documented source of Q)
    oq = O.OraclePoseBatch(1, 53)
    oq.init_from_state(x, P, abi.Location(synth.LAT0, synth.LON0, 0.0), synth.default_uwv(), abi.PoseParameter())
    oq.set_process_noise_from_config(cfg, dt)
    # fetch Q through a zero-covariance-free predict is not possible; rebuild it in numpy
    import numpy_twin as T
    tw = T.PoseTwin.from_config(53, log["pos0"][0], log["pos_cov"][0], log["rot0"][0], log["rot_cov"][0],
                                T.cfg_dict(cfg), T.UWV.from_abi(synth.default_uwv()))
    tw.set_noise_from_config(T.cfg_dict(cfg), dt)
    Q = tw.Q.copy()
    add = cfg.water_velocity.scale * (vs @ vs) * dt
    for d0 in (46, 48):
        Q[d0:d0 + 2, d0:d0 + 2] += add * np.eye(2)
    vec = [d for d in range(n) if not 3 <= d < 6 and d not in (12, 13, 14)]  # gyro bias feeds orientation only
    pred = F @ P[0] @ F.T + dt * dt * Q
    blk = np.ix_(vec, vec)
    scale = np.sqrt(np.outer(np.diag(pred)[vec], np.diag(pred)[vec]))
    assert np.max(np.abs(P2[0][blk] - pred[blk]) / scale) < 1e-10


def test_gate_leaves_state_bit_identical():
    o, _ = _filter()
    x0, P0 = o.get_state()
    acc = o.update("water_velocity", np.array([[50.0, -40.0]]), np.eye(2) * 0.05 ** 2, extra=0.5)
    assert acc[0] == 0
    x1, P1 = o.get_state()
    assert np.array_equal(x0, x1) and np.array_equal(P0, P1)


def test_measurement_models_closed_form():
    """h(x) at hand-computed states via a zero-covariance-limit update: with
    Sigma -> tiny, the predicted measurement is h(mu)."""
    import numpy_twin as T
    q = T.so3_exp(np.array([0.0, 0.0, np.pi / 2]))  # 90 deg yaw
    v = np.array([1.0, 0.0, 0.5])
    np.testing.assert_allclose(T.qrot(T.qconj(q), v), [0.0, -1.0, 0.5], atol=1e-15)
    a, g, ba = np.array([0.1, 0.2, 0.0]), 9.81, np.array([0.01, 0.0, -0.02])
    np.testing.assert_allclose(T.qrot(T.qconj(q), a + [0, 0, g]) + ba, [0.21, -0.1, 9.79], atol=1e-14)
    # pressure: p_atm - z g rho at 10 m depth
    assert abs((101325.0 - (-10.0) * 9.81 * 1025.0) - 201877.5) < 1e-9


def test_efforts_closed_form():
    u = synth.default_uwv()
    tau = np.zeros(6)
    acc6 = np.array([0.5, 0, 0, 0, 0, 0])
    vel6 = np.array([1.0, 0, 0, 0, 0, 0])
    q = np.array([1.0, 0, 0, 0])
    L.or_calc_efforts(C.byref(u), p(acc6), p(vel6), p(q), tau.ctypes.data_as(DP))
    # M a + D_l v + D_q |v| v (no rotation -> no Coriolis; W = B, r_b on z -> no restoring)
    np.testing.assert_allclose(tau, [200 * 0.5 + 20 + 50, 0, 0, 0, 0, 0], atol=1e-12)


def test_rk4_against_analytic_decay():
    """Pure linear surge damping: m v' = -d v  ->  v(t) = v0 exp(-d t / m)."""
    u = abi.UWVParams()
    abi.fill(u.inertia_matrix, np.diag([200.0, 250, 300, 20, 30, 30]).ravel())
    abi.fill(u.damping_matrices[0], np.diag([20.0, 30, 40, 5, 5, 5]).ravel())
    Minv = np.linalg.inv(np.diag([200.0, 250, 300, 20, 30, 30]))
    s = np.array([0, 0, 0, 1.0, 0, 0, 0, 1.0, 0, 0, 0, 0, 0])
    out = np.zeros(13)
    for _ in range(1000):
        L.or_model_rk4(C.byref(u), p(Minv), p(np.zeros(6)), C.c_double(1e-3), p(s), out.ctypes.data_as(DP))
        s = out.copy()
    assert abs(s[7] - np.exp(-20.0 / 200.0 * 1.0)) < 1e-12
    assert abs(s[0] - (200.0 / 20.0) * (1 - np.exp(-0.1))) < 1e-10


def test_nan_measurement_rejected():
    o, _ = _filter()
    with pytest.raises(RuntimeError):
        o.update("velocity", np.array([[np.nan, 0, 0]]), np.eye(3))


def test_efforts_side_effect_reaches_velocity_only_update():
    """measurementEfforts leaves the filter's shared DynamicModel holding the
    LAST sigma point's model parameters (PoseUKF.cpp:158-173); the next
    velocity-only update (constrainVelocity, :592) evaluates that model.  A
    filter re-created from the same state (PoseUKF.cpp:374-391: model = the
    configured UWV parameters) must therefore give a different velocity-only
    update: the GPU tests of the full -> velocity-only sequence
    (tests/test_gpu_surface.py) exercise a real dependency.  The last sigma
    point is mu (-) L_{n-1}, which differs from mu only in the water density
    (L lower triangular), so the model left behind is the PRIOR mean's
    parameters: two full updates are needed before they differ from the
    configured ones."""
    B = 2
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, 10, "C4")
    a = O.OraclePoseBatch(B, 53)
    a.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    a.set_process_noise_from_config(cfg, 1e-3)
    R = np.diag([25.0, 25, 25, 1, 1, 1])
    for e, t in enumerate((30.0, 35.0)):
        a.set_rotation_rate(log["gyro"][e])
        a.predict(1e-3)
        a.update("efforts", np.full((B, 6), t), R, only_vel=0)
    x, P = a.get_state()
    b = O.OraclePoseBatch(B, 53)
    param = abi.PoseParameter()
    param.gyro_bias_tau = param.acc_bias_tau = 600.0
    param.inertia_tau = param.lin_damping_tau = param.quad_damping_tau = 3600.0
    param.water_velocity_tau, param.adcp_bias_tau, param.water_density_tau = 900.0, 900.0, 3600.0
    param.water_velocity_limits, param.water_velocity_scale = 0.1, 1e-3
    param.atmospheric_pressure = 101325.0
    b.init_from_state(x, P, abi.Location(synth.LAT0, synth.LON0, 0.0), uwv, param)
    b.set_rotation_rate(log["gyro"][1])
    np.testing.assert_array_equal(a.get_rotation_rate(), b.get_rotation_rate())
    tau = np.full((B, 6), -10.0)
    for f in (a, b):
        f.update("efforts", tau, R, only_vel=1)
    va, vb = a.get_state()[0][:, 7:10], b.get_state()[0][:, 7:10]
    assert np.all(np.isfinite(va)) and np.all(np.isfinite(vb))
    assert np.max(np.abs(va - vb)) > 1e-9
