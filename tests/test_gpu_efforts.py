"""The BodyEfforts update on PSP (r05): measurementEfforts (PoseUKF.cpp:153-196)
in its full form (k_psp_efforts<DOF, 0, SR>: prefix k = 48 / 21, 2k + 1 model
evaluations, the blocked in-place Cholesky with MFMA panel updates) and
constrainVelocity (k = 9), against the literal kernels (UWVK_OPT_DENSE_SIGMA)
at a full grid, on both SO3 sides and both state sizes; the oracle parity at
small batches is tests/test_gpu_parity.py::test_single_update (efforts,
efforts_vel) and the C4 logs.  Tolerances: test_gpu_parity.py's single step."""
import numpy as np
import pytest

from helpers import cov_err, pose_setup, state_err

pytestmark = pytest.mark.gpu

TOL_STEP = 1e-9


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


def _handles(eng, B, dof, right):
    cfg, uwv, log = pose_setup(B, dof, "C3", 20)
    out = []
    for dense in (False, True):
        g = eng.PoseUKFBatch(B, dof)
        g.set_so3_right(right)
        g.set_dense_sigma(dense)
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        g.set_process_noise_from_config(cfg, 1e-3)
        g.run_log(g.upload_log(log))
        out.append(g)
    return out


@pytest.mark.parametrize("right", [True, False])
@pytest.mark.parametrize("dof", [53, 26])
@pytest.mark.parametrize("only_vel", [0, 1])
def test_efforts_psp_against_literal_full_grid(eng, dof, right, only_vel):
    B = 3000  # 3000 one-wave workgroups: every CU, several generations
    psp, lit = _handles(eng, B, dof, right)
    rng = np.random.default_rng(3 + only_vel)
    mu = 20 * rng.standard_normal((B, 6))
    cov = np.diag([25.0, 25, 25, 1, 1, 1])
    for g in (psp, lit):
        np.testing.assert_array_equal(g.update("efforts", mu, cov, only_vel=only_vel), np.ones(B, np.uint8))
    (xp, Pp), (xl, Pl) = psp.get_state(), lit.get_state()
    assert not psp.get_status().any() and not lit.get_status().any()
    se, ce = state_err(xp, xl, Pl, dof).max(), cov_err(Pp, Pl).max()
    assert se < TOL_STEP and ce < TOL_STEP, (se, ce)


def test_efforts_psp_model_side_effect(eng):
    """PoseUKF.cpp:173: the full update leaves the shared model's parameter
    blocks at the pre-update mean's (the next velocity-only update reads
    them): a full update followed by a velocity-only one agrees between the
    PSP and literal paths."""
    B, dof = 64, 53
    psp, lit = _handles(eng, B, dof, True)
    rng = np.random.default_rng(11)
    cov = np.diag([25.0, 25, 25, 1, 1, 1])
    for only_vel in (0, 1):
        mu = 20 * rng.standard_normal((B, 6))
        for g in (psp, lit):
            g.update("efforts", mu, cov, only_vel=only_vel)
    (xp, Pp), (xl, Pl) = psp.get_state(), lit.get_state()
    se, ce = state_err(xp, xl, Pl, dof).max(), cov_err(Pp, Pl).max()
    assert se < 10 * TOL_STEP and ce < 10 * TOL_STEP, (se, ce)


def test_efforts_psp_nan_leaves_state(eng):
    """checkMeasurment [EXT]: a NaN efforts measurement is refused before any
    kernel runs (UWVK_ENAN), the state untouched."""
    B, dof = 8, 53
    psp, _ = _handles(eng, B, dof, True)
    x0, P0 = psp.get_state()
    mu = np.zeros((B, 6))
    mu[3, 2] = np.nan
    with pytest.raises(eng.UWVKError) as e:
        psp.update("efforts", mu, np.eye(6))
    assert e.value.code == 2
    x1, P1 = psp.get_state()
    np.testing.assert_array_equal(x0, x1)
    np.testing.assert_array_equal(P0, P1)
