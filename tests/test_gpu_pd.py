"""The parameter-decoupled epoch kernel (UWVK_OPT_PARAM_BLOCK, DESIGN.md section
4.6, csrc/uwvk_psp_dev.hpp PspSmemPD): while the 27 model-parameter DOFs of a
53-DOF instance are uncoupled (their rows of Sigma zero off the diagonal, as
the reference's P0 and Q make them, PoseUKF.cpp:333-335 / :417-422), run_log
runs the other 26 DOFs in the 26-DOF layout with the 53-DOF weights and each
parameter alone.  The results must be BITWISE those of the general 53-DOF
kernel (up to the sign of zeros: numpy's array_equal treats -0 == 0), on C3
and C4 logs, across the 1024-epoch fold, with tail chunks handed on (static
and persistent), and the handle must leave the kernel once the full
BodyEfforts update couples the block.  Oracle parity of the default (PD) path
is every other run_log test in the suite."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


def _run(eng, log, cfg, uwv, pd, pieces, slots=-1, persist=True, init="config", expect_pd=None):
    from uwvk import abi, synth
    B = log["gyro"].shape[1]
    g = eng.PoseUKFBatch(B, 53)
    g.set_param_block(pd)
    g.set_pair(False)  # the one-instance PD kernel (the pair form is not bitwise)
    g.set_tail_slots(slots)
    g.set_persist(persist)
    if init == "config":
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    else:  # the bench's Monte-Carlo start through the second constructor
        rot0, rot_cov = synth.mc_rotation(log)
        g.init_from_config(log["pos0"], log["pos_cov"], rot0, rot_cov, cfg, uwv)
        x, P = g.get_state()
        x, P = synth.mc_start(x, P, log)
        loc = abi.Location(cfg.location.latitude, cfg.location.longitude, cfg.location.altitude)
        g.init_from_state(x, P, loc, uwv, synth.pose_parameter(cfg))
    g.set_process_noise_from_config(cfg, 1e-3)
    assert g.param_block() == (1 if pd else 0)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((B, 4), np.uint32))
    for a, n in pieces:
        g.run_log(dlog, a, n, accept_counts=acc)
    x, P = g.get_state()
    if expect_pd is not None:
        assert g.param_block() == expect_pd
    return x, P, acc.read(np.uint32, (B, 4)), g.get_status(), g.get_rotation_rate()


NAMES = ("state", "covariance", "accept counts", "status", "rotation rate")


@pytest.mark.parametrize("E,pieces,slots,persist,init", [
    (300, [(0, 300)], -1, True, "config"),
    (1100, [(0, 1100)], -1, False, "config"),      # across the 1024-epoch fold of the time scale
    (200, [(0, 57), (57, 143)], 3, True, "mc"),     # tail chunks over the ticket counter, MC start
    (200, [(0, 200)], 3, False, "config"),          # static tail-spread chunks
])
def test_pd_bitwise_c3(eng, E, pieces, slots, persist, init):
    from uwvk import synth
    B = 96
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run(eng, log, cfg, uwv, False, pieces, slots, persist, init)
    got = _run(eng, log, cfg, uwv, True, pieces, slots, persist, init, expect_pd=1)
    for name, a, b in zip(NAMES, got, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert not got[3].any()
    # the parameter block stayed decoupled (the PD kernel never writes those zeros)
    P = got[1]
    blk = P[:, 19:46, :].copy()
    for t in range(27):
        blk[:, t, 19 + t] = 0.0
    assert not blk.any()


@pytest.mark.parametrize("vo", [False, True])
def test_pd_bitwise_c4(eng, vo):
    """C4 with a compressed drop-out cycle: pressure and ADCP epochs on the PD
    kernel, then the BodyEfforts epochs: the full model couples the block and
    the rest of the log runs on the general kernel (bitwise the same overall);
    the velocity-only form (constrainVelocity) keeps it decoupled."""
    from uwvk import abi, synth
    B, E = 64, 800
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C4", dropout_on=0.3, dropout_off=0.1, adcp_every=100,
                              efforts_velocity_only=vo)
    assert ((log["flags"] & abi.EV_EFFORTS) != 0).any() and ((log["flags"] & abi.EV_ADCP) != 0).any()
    pieces = [(0, 450), (450, 350)]
    ref = _run(eng, log, cfg, uwv, False, pieces)
    got = _run(eng, log, cfg, uwv, True, pieces, expect_pd=1 if vo else 0)
    for name, a, b in zip(NAMES, got, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)


def test_pd_eligibility(eng):
    """The host's checks: a coupled initial covariance, a coupled Q, the 26-DOF
    layout and the option each select the general kernel."""
    from uwvk import abi, synth
    B = 16
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, 10, "C3")
    g = eng.PoseUKFBatch(B, 53)
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    assert g.param_block() == 1
    x, P = g.get_state()
    loc = abi.Location(cfg.location.latitude, cfg.location.longitude, cfg.location.altitude)
    Pc = P.copy()
    Pc[5, 20, 7] = Pc[5, 7, 20] = 1e-6  # one instance's inertia couples with the velocity
    g.init_from_state(x, Pc, loc, uwv, synth.pose_parameter(cfg))
    g.set_process_noise_from_config(cfg, 1e-3)
    assert g.param_block() == 0
    g.init_from_state(x, P, loc, uwv, synth.pose_parameter(cfg))
    Q = np.zeros((53, 53))
    np.fill_diagonal(Q, 1e-6)
    g.set_process_noise(Q)
    assert g.param_block() == 1
    Q[30, 31] = Q[31, 30] = 1e-9  # coupled within the parameter block
    g.set_process_noise(Q)
    assert g.param_block() == 0
    np.fill_diagonal(Q, 1e-6)
    Q[30, 31] = Q[31, 30] = 0.0
    g.set_process_noise(Q)
    g.set_param_block(False)
    assert g.param_block() == 0
    g.set_param_block(True)
    assert g.param_block() == 1
    # the full BodyEfforts update (single call) couples the block
    z = np.zeros((B, 6))
    g.update("efforts", z, np.eye(6) * 25.0, only_vel=True)
    assert g.param_block() == 1
    g.update("efforts", z, np.eye(6) * 25.0)
    assert g.param_block() == 0
    g26 = eng.PoseUKFBatch(B, 26)
    l26 = synth.make_pose_log(B, 10, "C3", dof=26)
    g26.init_from_config(l26["pos0"], l26["pos_cov"], l26["rot0"], l26["rot_cov"], cfg, uwv)
    assert g26.param_block() == 0


# ---- the two-instances-per-wave form (UWVK_OPT_PAIR, csrc/uwvk_psp_pair.hip) ----
def _run_pair(eng, log, cfg, uwv, pair, pieces, slots=-1, chunks=0, pd=True, dof=53):
    from uwvk import abi
    B = log["gyro"].shape[1]
    g = eng.PoseUKFBatch(B, dof)
    g.set_param_block(pd)
    g.set_pair(pair)
    g.set_tail_slots(slots)
    if chunks:
        g.set_tail_chunks(chunks)
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    assert g.pair_active() == (1 if pair else 0)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((B, 4), np.uint32))
    for a, n in pieces:
        g.run_log(dlog, a, n, accept_counts=acc)
    x, P = g.get_state()
    return x, P, acc.read(np.uint32, (B, 4)), g.get_status(), g.get_rotation_rate()


@pytest.mark.parametrize("mode,E,pieces,dof", [("C3", 300, [(0, 300)], 53), ("C3", 1100, [(0, 600), (600, 500)], 53),
                                               ("C4", 800, [(0, 450), (450, 350)], 53),
                                               ("C3", 600, [(0, 350), (350, 250)], 26),
                                               ("C4", 800, [(0, 450), (450, 350)], 26)])
def test_pair_matches_single(eng, mode, E, pieces, dof):
    """The pair kernel against the one-instance kernel (PD at 53 DOF, the
    handle's own layout at 26).  C4: the launches split around the pressure
    epochs, ADCP epochs inside the pair runs; at 53 DOF the first full efforts
    epoch hands both handles to the general kernel, at 26 DOF the pair kernel
    continues.  The same filter to rounding (the rank-M update's order), gate
    decisions bitwise."""
    from helpers import cov_err, state_err
    from uwvk import synth
    B = 96
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    extra = dict(dropout_on=0.3, dropout_off=0.1, adcp_every=150) if mode == "C4" else {}
    log = synth.make_pose_log(B, E, mode, dof=dof, **extra)
    ref = _run_pair(eng, log, cfg, uwv, False, pieces, dof=dof)
    got = _run_pair(eng, log, cfg, uwv, True, pieces, dof=dof)
    np.testing.assert_array_equal(got[2], ref[2])
    np.testing.assert_array_equal(got[3], ref[3])
    # the rotation rate less the gyro-bias estimate (getRotationRate): to rounding
    np.testing.assert_allclose(got[4], ref[4], rtol=1e-9, atol=1e-15)
    assert state_err(got[0], ref[0], ref[1], dof).max() < 1e-9
    assert cov_err(got[1], ref[1]).max() < 1e-9


@pytest.mark.parametrize("chunks", [2, 5])
def test_pair_tail_chunks_bitwise(eng, chunks):
    """Tail chunks of pair units handed on (Sigma~ and the time scale unfolded):
    bitwise the unchunked pair run."""
    from uwvk import synth
    B, E = 96, 120
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run_pair(eng, log, cfg, uwv, True, [(0, 70), (70, 50)])
    got = _run_pair(eng, log, cfg, uwv, True, [(0, 70), (70, 50)], slots=1, chunks=chunks)
    for name, a, b in zip(NAMES, got, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert not got[3].any()


@pytest.mark.parametrize("mode,dof", [("C3", 53), ("C4", 53), ("C3", 26), ("C4", 26)])
def test_pair_matches_oracle(eng, mode, dof):
    """Pair-default handles (53-DOF decoupled, 26-DOF) against the oracle.  C4
    (compressed drop-out cycle): the launches split around the pressure epochs
    (those on the one-instance kernel, the runs between them on the pair kernel,
    ADCP epochs 150 / 450 / 750 inside the runs); at 53 DOF the first full
    efforts epoch (399) couples the parameters and the general kernel takes
    over, at 26 DOF the pair kernel runs to the end."""
    from helpers import cov_err, init_both, state_err
    import oracle_ctypes as orc
    from uwvk import abi, synth
    B, E = 6, 400 if mode == "C3" else 900
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    # ADCP every 150 epochs: some on pressure epochs (one-instance kernel), some
    # inside the pair runs (k_psp_epoch_pair<SR, 0>)
    extra = dict(dropout_on=0.4, dropout_off=0.1, adcp_every=150) if mode == "C4" else {}
    log = synth.make_pose_log(B, E, mode, dof=dof, **extra)
    if mode == "C4":
        fl = log["flags"]
        assert ((fl & abi.EV_PRESSURE) != 0).any() and ((fl & abi.EV_ADCP) != 0).any()
        assert ((fl & abi.EV_EFFORTS) != 0).any()
    o = orc.OraclePoseBatch(B, dof)
    g = eng.PoseUKFBatch(B, dof)
    g.set_pair(True)
    init_both(o, g, cfg, uwv, log)
    co = o.run_log(log)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((B, 4), np.uint32))
    g.run_log(dlog, accept_counts=acc)
    np.testing.assert_array_equal(co, acc.read(np.uint32, (B, 4)))
    xo, Po = o.get_state()
    xg, Pg = g.get_state()
    assert state_err(xg, xo, Po, dof).max() < 1e-7 and cov_err(Pg, Po).max() < 1e-7


def test_pair_eligibility(eng):
    """Where run_log takes the pair kernel (uwvk_pose_pair_active): 53-DOF
    handles while decoupled and 26-DOF handles, on an even batch, the
    persistent scheduler and the PSP path; otherwise one instance per wave."""
    from uwvk import synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()

    def mk(B, dof):
        log = synth.make_pose_log(B, 4, "C3", dof=dof)
        g = eng.PoseUKFBatch(B, dof)
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        g.set_process_noise_from_config(cfg, 1e-3)
        return g
    assert mk(6, 53).pair_active() == 1
    assert mk(6, 26).pair_active() == 1
    assert mk(5, 53).pair_active() == 0  # odd batch
    g = mk(6, 53)
    g.set_persist(False)
    assert g.pair_active() == 0
    g.set_persist(True)
    g.set_pair(False)
    assert g.pair_active() == 0
    g.set_pair(True)
    g.set_param_block(False)  # the general 53-DOF kernel
    assert g.pair_active() == 0
    g = mk(6, 26)
    g.set_dense_sigma(True)
    assert g.pair_active() == 0
