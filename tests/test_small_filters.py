"""BottomUKF, IndirectPoseUKF and the marker-augmented visual-landmark updates
(SURVEY.md §8(f) ranks 3-4).

CPU: the oracle (oracle/uwvk_small_oracle.c) against closed forms:
  S2 manifold identities, linear-limit Kalman updates, the exactly linear
  predict blocks, and consistency of the visual updates with a true pose.
GPU (-m gpu): the HIP lane-group kernels through the C ABI against the oracle
on seeded random batches (fp64; tolerances in units of the oracle's standard
deviations, 1e-9 per short sequence)."""
import numpy as np
import pytest

import oracle_ctypes as O
import visual_scene as V
from helpers import cov_err, pose_setup, qlog_err, state_err
from uwvk import engine, synth
from uwvk.small import BottomUKFBatch, IndirectPoseUKFBatch

L = O.lib()
DP = O.DP
TOL = 1e-9


def _s2(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def s2_plus(x, d):
    o = np.zeros(3)
    L.or_s2_boxplus(O.dp(x), O.dp(d), O.C.c_double(1.0), o.ctypes.data_as(DP))
    return o


def s2_minus(y, x):
    o = np.zeros(2)
    L.or_s2_boxminus(O.dp(y), O.dp(x), o.ctypes.data_as(DP))
    return o


# ---------------------------------------------------------------------------
# CPU: the oracle
# ---------------------------------------------------------------------------
def test_s2_manifold_identities():
    rng = np.random.default_rng(1)
    for _ in range(200):
        x = _s2(rng.standard_normal(3) + [0, 0, 2.0])
        d = rng.uniform(-1.0, 1.0, 2)
        y = s2_plus(x, d)
        assert abs(np.linalg.norm(y) - 1.0) < 1e-14
        np.testing.assert_allclose(s2_minus(y, x), d, atol=1e-12)
        z = _s2(rng.standard_normal(3) + [0, 0, 2.0])
        np.testing.assert_allclose(s2_plus(x, s2_minus(z, x)), z, atol=1e-12)
        # geodesic: |y [-] x| is the angle between them
        ang = np.arccos(np.clip(np.dot(z, x), -1, 1))
        assert abs(np.linalg.norm(s2_minus(z, x)) - ang) < 1e-12
    np.testing.assert_allclose(s2_plus(np.array([0, 0, 1.0]), np.zeros(2)), [0, 0, 1.0], atol=0)


def bottom_state(B, seed=5):
    rng = np.random.default_rng(seed)
    x = np.zeros((B, 4))
    x[:, 0] = 10.0 + rng.uniform(-1, 1, B)
    x[:, 1:] = _s2(np.c_[rng.normal(0, 0.1, (B, 2)), np.ones(B)])
    P = np.zeros((B, 3, 3))
    for i in range(B):
        A = rng.normal(0, 1, (3, 3)) * [0.3, 0.05, 0.05]
        P[i] = A @ A.T + np.diag([0.05, 0.003, 0.003])
    return x, P


def test_bottom_predict_is_exact_shift():
    o = O.OracleBottomBatch(3)
    x, P = bottom_state(3)
    o.init(x, P)
    o.set_velocity([0.0, 0.0, 0.3])  # |v_xy| = 0 -> no process noise
    for _ in range(20):
        o.predict(0.1)
    xo, Po = o.get_state()
    np.testing.assert_allclose(xo[:, 0], x[:, 0] - 20 * 0.1 * 0.3, rtol=0, atol=1e-12)
    np.testing.assert_allclose(xo[:, 1:], x[:, 1:], atol=1e-12)
    assert cov_err(Po, P).max() < 1e-11


def test_bottom_range_linear_limit_is_kalman():
    B = 4
    x = np.tile([10.0, 0.0, 0.0, 1.0], (B, 1))
    P = np.tile(np.diag([0.5, 1e-14, 1e-14]), (B, 1, 1))
    z = np.array([9.0, 10.5, 11.0, 10.0])
    R = 0.2
    o = O.OracleBottomBatch(B)
    o.init(x, P)
    o.update_range(z, R, [0.0, 0.0, -1.0], [0.0, 0.0, 0.0])  # h = d exactly at n = e3
    xo, Po = o.get_state()
    k = 0.5 / (0.5 + R)
    np.testing.assert_allclose(xo[:, 0], 10.0 + k * (z - 10.0), rtol=1e-9)
    np.testing.assert_allclose(Po[:, 0, 0], 0.5 * R / (0.5 + R), rtol=1e-9)


def test_bottom_normal_update_moves_toward_measurement():
    B = 2
    x = np.tile([10.0, 0.0, 0.0, 1.0], (B, 1))
    P = np.tile(np.diag([0.5, 1e-4, 1e-4]), (B, 1, 1))
    zt = np.array([0.01, -0.02])  # tangent offset of the measured normal
    zv = s2_plus(np.array([0, 0, 1.0]), zt)
    o = O.OracleBottomBatch(B)
    o.init(x, P)
    o.update_normal(np.tile(zv, (B, 1)), np.eye(2) * 1e-4)
    xo, Po = o.get_state()
    moved = s2_minus(xo[0, 1:], np.array([0, 0, 1.0]))
    np.testing.assert_allclose(moved, 0.5 * zt, rtol=1e-3)  # K = P / (P + R) = 1/2
    np.testing.assert_allclose(Po[0, 1, 1], 0.5e-4, rtol=1e-3)


def test_ipose_predict_blocks():
    """orientation error decays exactly: Sigma_oo' = (1 - dt/tau)^2 Sigma_oo + Q'."""
    o = O.OracleIndirectPoseBatch(1)
    pos_std, ori_std, tau, dt = np.array([0.1, 0.2, 0.3]), np.array([0.01, 0.02, 0.03]), 20.0, 0.1
    o.init(pos_std, ori_std, tau, None, np.array([1.0, 2.0, 3.0]))
    x0, P0 = o.get_state()
    o.predict(dt)
    x1, P1 = o.get_state()
    np.testing.assert_allclose(x1[0], [0, 0, 0, 1, 0, 0, 0], atol=1e-15)
    np.testing.assert_allclose(np.diag(P1[0])[:3], np.diag(P0[0])[:3] + dt ** 2 * pos_std ** 2, rtol=1e-12)
    a = 1 - dt / tau
    np.testing.assert_allclose(np.diag(P1[0])[3:], a * a * ori_std ** 2 + 2 * dt / tau * ori_std ** 2, rtol=1e-12)


def ipose_scene(B, seed=11):
    rng = np.random.default_rng(seed)
    ref_t = rng.normal(0, 5, (B, 3))
    ref_q = V.qexp(rng.normal(0, 0.3, (B, 3)))
    p_err = rng.normal(0, 0.3, (B, 3))
    q_err = V.qexp(rng.normal(0, 0.02, (B, 3)))
    body_t = ref_t + V.qrot(ref_q, p_err)
    body_q = V.qmul(ref_q, q_err)
    marker = V.marker_ahead(body_t, body_q)
    px, zc = V.project(body_t, body_q, marker)
    assert (zc > 1.0).all()
    px = px + V.pixel_noise(B, seed + 1, 0.3)
    ref = np.concatenate([ref_t, ref_q], 1)
    return ref, p_err, q_err, marker, px


def visual_common(B):
    fcov = np.tile(np.eye(2) * 0.09, (4, 1, 1))
    cov_marker = np.diag([1e-4] * 3 + [1e-5] * 3)
    return fcov, V.CORNERS, cov_marker, V.CAMERA, V.CAM_IN_BODY


def test_ipose_visual_update_reduces_error():
    B = 6
    ref, p_err, q_err, marker, px = ipose_scene(B)
    o = O.OracleIndirectPoseBatch(B)
    o.init([0.1] * 3, [0.01] * 3, 20.0, None, [0.5] * 3)
    o.set_pose_reference(ref)
    fcov, fpos, cm, cam, cib = visual_common(B)
    P0 = o.get_state()[1]
    o.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    x, P = o.get_state()
    e0 = np.linalg.norm(p_err, axis=1)
    e1 = np.linalg.norm(x[:, :3] - p_err, axis=1)
    assert (e1 < 0.5 * e0).all(), (e0, e1)
    assert (np.trace(P[:, :3, :3], axis1=1, axis2=2) < 0.5 * np.trace(P0[:, :3, :3], axis1=1, axis2=2)).all()
    corr = o.get_corrected_pose()
    true_t = ref[:, :3] + V.qrot(ref[:, 3:], p_err)
    assert (np.linalg.norm(corr[:, :3] - true_t, axis=1) < 0.5 * e0).all()


def test_ipose_visual_nan_feature_changes_nothing():
    B = 2
    ref, p_err, q_err, marker, px = ipose_scene(B)
    o = O.OracleIndirectPoseBatch(B)
    o.init([0.1] * 3, [0.01] * 3, 20.0)
    o.set_pose_reference(ref)
    before = o.get_state()
    px[0, 2, 1] = np.nan
    fcov, fpos, cm, cam, cib = visual_common(B)
    with pytest.raises(RuntimeError):
        o.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    after = o.get_state()
    np.testing.assert_array_equal(before[0][0], after[0][0])


def pose_scene(x, seed=21):
    """marker ahead of each (perturbed) PoseUKF estimate; true pose = estimate + offset"""
    B = len(x)
    rng = np.random.default_rng(seed)
    true_t = x[:, :3] + rng.normal(0, 0.2, (B, 3))
    true_q = V.qmul(V.qexp(rng.normal(0, 0.01, (B, 3))), x[:, 3:7])
    marker = V.marker_ahead(true_t, true_q)
    px, zc = V.project(true_t, true_q, marker)
    assert (zc > 1.0).all()
    return true_t, true_q, marker, px + V.pixel_noise(B, seed + 1, 0.3)


@pytest.mark.parametrize("right", [True, False])
@pytest.mark.parametrize("dof", [53, 26])
def test_pose_visual_update_reduces_error(dof, right):
    """Both SO3 segments of PoseStateWithMarker on the filter's side
    (or_set_so3_right: sm SEG_SO3R on the default right side, SEG_SO3 on the
    left); the side reaches the augmented update."""
    B = 3
    cfg, uwv, log = pose_setup(B, dof=dof, epochs=5)
    o = O.OraclePoseBatch(B, dof)
    o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o.set_process_noise_from_config(cfg, log["dt"])
    x0, P0 = o.get_state()
    true_t, true_q, marker, px = pose_scene(x0)
    fcov, fpos, cm, cam, cib = visual_common(B)
    with O.so3_side(right):
        o.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    x1, P1 = o.get_state()
    o2 = O.OraclePoseBatch(B, dof)  # the other side differs
    o2.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    o2.set_process_noise_from_config(cfg, log["dt"])
    with O.so3_side(not right):
        o2.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    assert np.abs(o2.get_state()[1] - P1).max() > 1e-9
    e0 = np.linalg.norm(x0[:, :3] - true_t, axis=1)
    e1 = np.linalg.norm(x1[:, :3] - true_t, axis=1)
    assert (e1 < e0).all(), (e0, e1)
    assert (np.trace(P1[:, :3, :3], axis1=1, axis2=2) < np.trace(P0[:, :3, :3], axis1=1, axis2=2)).all()
    # (bearings to a 0.4 m marker at 3 m leave yaw and lateral position coupled:
    #  no per-instance orientation claim)


# ---------------------------------------------------------------------------
# GPU: the HIP kernels through the C ABI against the oracle
# ---------------------------------------------------------------------------
def _vec_err(xa, xb, P):
    """max |xa - xb| / sqrt(P_ii) over the vector part (distance / position)."""
    return float(np.max(np.abs(xa - xb) / np.sqrt(P)))


@pytest.mark.gpu
def test_gpu_bottom_sequence():
    B = 37  # not a multiple of the 8 instances per wave
    x, P = bottom_state(B)
    rng = np.random.default_rng(3)
    g, o = BottomUKFBatch(B), O.OracleBottomBatch(B)
    Q = np.diag([0.02, 0.001, 0.001])
    beams = [(_s2([0.5, 0.0, -0.866]), [0.1, 0.0, 0.0]), (_s2([-0.5, 0.0, -0.866]), [-0.1, 0.0, 0.0]),
             (_s2([0.0, 0.5, -0.866]), [0.0, 0.1, 0.0]), (_s2([0.0, -0.5, -0.866]), [0.0, -0.1, 0.0])]
    for f in (g, o):
        f.init(x, P)
        f.set_process_noise(Q)
    for step in range(30):
        v = np.c_[rng.normal(0.5, 0.1, B), rng.normal(0, 0.1, B), rng.normal(0, 0.05, B)]
        for f in (g, o):
            f.set_velocity(v)
            f.predict(0.2)
        d, bo = beams[step % 4]
        z = 10.0 / 0.866 + rng.normal(0, 0.05, B)
        cov = rng.uniform(0.01, 0.03, B)
        for f in (g, o):
            f.update_range(z, cov, d, bo)
        if step % 5 == 4:
            zn = _s2(np.c_[rng.normal(0, 0.03, (B, 2)), np.ones(B)])
            for f in (g, o):
                f.update_normal(zn, np.eye(2) * 4e-4)
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    assert _vec_err(xg[:, 0], xo[:, 0], Po[:, 0, 0]) < TOL
    ang = np.linalg.norm(np.cross(xg[:, 1:], xo[:, 1:]), axis=1)  # sin of the angle (arccos loses 1e-8)
    assert float(np.max(ang / np.sqrt(np.minimum(Po[:, 1, 1], Po[:, 2, 2])))) < TOL
    assert cov_err(Pg, Po).max() < TOL
    assert not g.get_status().any()


@pytest.mark.gpu
def test_gpu_bottom_mask_and_errors():
    B = 9
    x, P = bottom_state(B)
    g, o = BottomUKFBatch(B), O.OracleBottomBatch(B)
    for f in (g, o):
        f.init(x, P)
    mask = np.arange(B) % 2 == 0
    z = np.full(B, 9.5)
    x0, P0 = g.get_state()
    g.update_range(z, 0.02, [0, 0, -1.0], [0, 0, 0], mask=mask)
    o.update_range(z, 0.02, [0, 0, -1.0], [0, 0, 0], mask=mask)
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    np.testing.assert_array_equal(xg[~mask], x0[~mask])  # masked-out instances untouched
    np.testing.assert_array_equal(Pg[~mask], P0[~mask])
    assert _vec_err(xg[:, 0], xo[:, 0], Po[:, 0, 0]) < TOL
    assert cov_err(Pg, Po).max() < TOL
    z[1] = np.nan
    g.update_range(z, 0.02, [0, 0, -1.0], [0, 0, 0], mask=mask)  # NaN in a masked-out instance: ignored
    z[2] = np.nan
    with pytest.raises(engine.UWVKError) as e:
        g.update_range(z, 0.02, [0, 0, -1.0], [0, 0, 0], mask=mask)
    assert e.value.code == 2


@pytest.mark.gpu
@pytest.mark.parametrize("right", [True, False])
def test_gpu_ipose_predict_and_visual(right):
    """Both sides of the orientation_error's SO3 [+] (right, the default; left
    via uwvk_ipose_set_option) against the oracle's same side."""
    B = 13  # not a multiple of 2 / 4 instances per wave
    ref, p_err, q_err, marker, px = ipose_scene(B)
    g, o = IndirectPoseUKFBatch(B), O.OracleIndirectPoseBatch(B)
    if not right:
        g.set_so3_right(False)
    ipe = np.random.default_rng(2).normal(0, 0.1, (B, 3))
    fcov, fpos, cm, cam, cib = visual_common(B)
    with O.so3_side(right):
        for f in (g, o):
            f.init([0.1, 0.1, 0.2], [0.01, 0.01, 0.02], 20.0, ipe, [0.5, 0.5, 0.5])
            f.set_pose_reference(ref)
        for step in range(4):
            for f in (g, o):
                f.predict(0.1)
            for f in (g, o):
                f.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    assert _vec_err(xg[:, :3], xo[:, :3], np.diagonal(Po, axis1=1, axis2=2)[:, :3]) < TOL
    assert float(np.max(qlog_err(xg[:, 3:], xo[:, 3:]) / np.sqrt(np.min(np.diagonal(Po, axis1=1, axis2=2)[:, 3:],
                                                                        1)))) < TOL
    assert cov_err(Pg, Po).max() < TOL
    np.testing.assert_allclose(g.get_corrected_pose(), o.get_corrected_pose(), atol=1e-9)
    assert not g.get_status().any()


@pytest.mark.gpu
@pytest.mark.parametrize("dof", [53, 26])
def test_gpu_pose_visual_landmark(dof):
    B = 5
    cfg, uwv, log = pose_setup(B, dof=dof, epochs=60)
    g, o = engine.PoseUKFBatch(B, dof), O.OraclePoseBatch(B, dof)
    for f in (g, o):
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, log["dt"])
    o.run_log(log)
    g.run_log(g.upload_log(log))
    x0 = o.get_state()[0]
    true_t, true_q, marker, px = pose_scene(x0)
    fcov, fpos, cm, cam, cib = visual_common(B)
    per_inst_cov = np.tile(fcov, (B, 1, 1, 1))
    for rep in range(2):  # a repeated call reuses the handle's staging buffer
        for f in (g, o):
            f.update_visual(px, per_inst_cov if rep == 0 else fcov, fpos, marker, cm, cam, cib)
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    assert state_err(xg, xo, Po, dof).max() < TOL
    assert cov_err(Pg, Po).max() < TOL
    assert not g.get_status().any()
    # a NaN feature fails the whole call and changes nothing
    px[1, 0, 0] = np.nan
    with pytest.raises(engine.UWVKError) as e:
        g.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    assert e.value.code == 2
    np.testing.assert_array_equal(g.get_state()[0], xg)


@pytest.mark.gpu
def test_gpu_ipose_process_noise():
    """setProcessNoiseCovariance [EXT base] with cross terms between position and orientation error."""
    B = 7
    ref, p_err, q_err, marker, px = ipose_scene(B)
    g, o = IndirectPoseUKFBatch(B), O.OracleIndirectPoseBatch(B)
    A = np.random.default_rng(4).normal(0, 1, (6, 6)) * np.r_[[0.1] * 3, [0.01] * 3][:, None]
    Q = A @ A.T + np.diag([1e-3] * 3 + [1e-5] * 3)
    for f in (g, o):
        f.init([0.1, 0.1, 0.2], [0.01, 0.01, 0.02], 20.0, None, [0.5, 0.5, 0.5])
        f.set_process_noise(Q)
        f.set_pose_reference(ref)
    for step in range(5):
        for f in (g, o):
            f.predict(0.1)
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    assert cov_err(Pg, Po).max() < TOL
    assert float(np.max(qlog_err(xg[:, 3:], xo[:, 3:]))) < 1e-12
