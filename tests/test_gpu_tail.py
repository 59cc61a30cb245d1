"""Last-generation spreading of the PSP run_log launch (UWVK_OPT_TAIL_SLOTS,
csrc/uwvk_psp_k.hip: plan_tail / tail_unit): the tail instances of each XCD
run as epoch chunks handed from block to block.  Sigma~ and its time scale are
handed on unfolded, so the result must be bitwise the one-block-per-instance
run: state, covariance, accept counts, status words and rotation rate.

The slot counts here are small overrides so that batches of a few dozen
instances have a partial last generation; the default plan (runtime
occupancy, 384 blocks per XCD on MI355X) is exercised by the full-batch C4
test in test_gpu_surface.py, whose sampled instances include tail ones."""
import numpy as np
import pytest

from helpers import pose_setup

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device / libuwvk.so not loadable: the HIP path is mandatory")
    return engine


def _run(eng, B, dof, log, cfg, uwv, slots, pieces, persist=False, force=0, pair=False):
    g = eng.PoseUKFBatch(B, dof)
    g.set_tail_slots(slots)
    g.set_persist(persist)
    g.set_pair(pair)  # the pair form (default on, persistent only) is not bitwise the one-instance kernel
    if force:
        g.set_tail_chunks(force)
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    dlog = g.upload_log(log)
    acc = eng.DeviceBuffer(np.zeros((B, 4), np.uint32))
    for a, n in pieces:
        g.run_log(dlog, a, n, accept_counts=acc)
    x, P = g.get_state()
    return x, P, acc.read(np.uint32, (B, 4)), g.get_status(), g.get_rotation_rate()


CASES = [  # dof, mode, epochs, slots per XCD, instances per XCD, run_log pieces
    (53, "C3", 200, 3, 20, [(0, 200)]),
    (53, "C3", 20, 3, 12, [(0, 20)]),
    (53, "C4", 600, 2, 12, [(0, 600)]),
    (26, "C4", 400, 3, 16, [(0, 37), (37, 363)]),
    (53, "C3", 9, 2, 9, [(0, 9)]),
]


@pytest.mark.parametrize("dof,mode,E,slots,n,pieces", CASES)
def test_tail_chunks_bitwise(eng, dof, mode, E, slots, n, pieces):
    from uwvk import synth
    B = 8 * n
    for _, cnt in pieces:
        assert eng.lib().uwvk_pose_tail_chunks(n, slots, cnt) > 1
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    extra = dict(dropout_on=0.1, dropout_off=0.05) if mode == "C4" else {}
    log = synth.make_pose_log(B, E, mode, dof=dof, **extra)
    ref = _run(eng, B, dof, log, cfg, uwv, -1, pieces)
    got = _run(eng, B, dof, log, cfg, uwv, slots, pieces)
    names = ("state", "covariance", "accept counts", "status", "rotation rate")
    for name, a, b in zip(names, got, ref):
        np.testing.assert_array_equal(a, b, err_msg=name)
    assert not got[3].any()


def test_tail_default_plan_repeat(eng):
    """The runtime-occupancy plan on a batch that leaves a partial last
    generation on every XCD (n = 8,192 + 64 per XCD): two runs with the flags
    of the first still in memory (the per-launch tag) agree bitwise with the
    unspread run."""
    from uwvk import synth
    B, E = 8 * (8192 + 64), 60
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run(eng, B, 53, log, cfg, uwv, -1, [(0, 30), (30, 30)])
    got = _run(eng, B, 53, log, cfg, uwv, 0, [(0, 30), (30, 30)])
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


def test_xcd_round_robin_on_this_device(eng):
    """The probe that gates tail spreading: the box's single-partition MI355X
    places block b on the XCC of block b % 8 (hardware XCC_ID)."""
    assert eng.lib().uwvk_xcd_round_robin(0) == 1


@pytest.mark.timeout(900)
@pytest.mark.parametrize("B", [65536, 131072])
def test_every_chunk_count_at_full_batch(eng, B):
    """C3 / C5-shard batches with the runtime's resident slots: each chunk
    count 2..8 (forced, UWVK_OPT_TAIL_CHUNKS; the planner's choice is a host
    unit test) run on a 20-epoch piece, then one unspread epoch, so that the
    piece's final Sigma reaches the mean.  The means are bitwise those of a
    handle that never spreads, with no status bits and equal accept counts."""
    from uwvk import synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    piece = 20
    E = 7 * (piece + 1)
    log = synth.make_pose_log(B, E, "C3")
    hs = []
    for spread in (False, True):
        g = eng.PoseUKFBatch(B, 53)
        g.set_tail_slots(0 if spread else -1)
        g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        g.set_process_noise_from_config(cfg, 1e-3)
        hs.append((g, g.upload_log(log), eng.DeviceBuffer(np.zeros((B, 4), np.uint32))))
    e = 0
    for c in range(2, 9):
        for (g, d, acc), spread in zip(hs, (False, True)):
            g.set_tail_chunks(c if spread else 0)
            g.run_log(d, e, piece, accept_counts=acc)
            g.set_tail_chunks(0)
            g.set_tail_slots(-1)
            g.run_log(d, e + piece, 1, accept_counts=acc)
            g.set_tail_slots(0 if spread else -1)
        e += piece + 1
        (x0, _), (x1, _) = [(g.get_state_mu(), None) for g, _, _ in hs]
        np.testing.assert_array_equal(x1, x0, err_msg="chunks=%d" % c)
    for g, _, _ in hs:
        assert not g.get_status().any()
    np.testing.assert_array_equal(hs[1][2].read(np.uint32, (B, 4)), hs[0][2].read(np.uint32, (B, 4)))


# Persistent scheduling (UWVK_OPT_PERSIST): resident workgroups take units from
# a ticket counter; chunk k of a tail instance may run on any XCD after chunk
# k - 1.  Bitwise the one-workgroup-per-instance run, with and without chunks,
# on every chunk count the planner can be forced to.  pair=True: the
# two-instances-per-wave form (persistent only), its chunked runs bitwise its
# unchunked one (the C4 and 26-DOF cases run no pair launch: the selection).
@pytest.mark.parametrize("pair", [False, True])
@pytest.mark.parametrize("dof,mode,E,slots,n,pieces", CASES)
def test_persist_bitwise(eng, dof, mode, E, slots, n, pieces, pair):
    from uwvk import synth
    B = 8 * n
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    extra = dict(dropout_on=0.1, dropout_off=0.05) if mode == "C4" else {}
    log = synth.make_pose_log(B, E, mode, dof=dof, **extra)
    ref = _run(eng, B, dof, log, cfg, uwv, -1, pieces, persist=pair, pair=pair)
    names = ("state", "covariance", "accept counts", "status", "rotation rate")
    for sl in (-1, slots):  # no chunks; the planner's chunks for `slots` per XCD
        got = _run(eng, B, dof, log, cfg, uwv, sl, pieces, persist=True, pair=pair)
        for name, a, b in zip(names, got, ref):
            np.testing.assert_array_equal(a, b, err_msg="%s (slots %d)" % (name, sl))


@pytest.mark.parametrize("chunks", [2, 3, 5, 8])
def test_persist_forced_chunks(eng, chunks):
    from uwvk import synth
    B, E = 48, 40
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run(eng, B, 53, log, cfg, uwv, -1, [(0, 17), (17, 23)])
    got = _run(eng, B, 53, log, cfg, uwv, 1, [(0, 17), (17, 23)], persist=True, force=chunks)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)
    assert not got[3].any()


def test_persist_default_plan_repeat(eng):
    """The runtime-occupancy plan at C5's shard size plus a partial generation,
    two launches (the ticket base carried between them)."""
    from uwvk import synth
    B, E = 8 * (8192 + 64), 60
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run(eng, B, 53, log, cfg, uwv, -1, [(0, 30), (30, 30)])
    got = _run(eng, B, 53, log, cfg, uwv, 0, [(0, 30), (30, 30)], persist=True)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("persist,pair", [(False, False), (True, False), (True, True)])
def test_handoff_timeout_is_an_error(eng, persist, pair):
    """ABI 3: a timed-out tail-chunk hand-off makes
    uwvk_pose_run_log return UWVK_ESCHEDULE (not only a status bit), the
    chunks after it flag their instances UWVK_ST_SCHEDULE, every other instance
    is bitwise the unspread run, and the handle's fault word is cleared: the
    next launch without forced timeouts returns OK again."""
    from uwvk import synth
    n, slots, E = 12, (2 if pair else 3), 20
    B = 8 * n
    assert eng.lib().uwvk_pose_tail_chunks(n, slots, E) > 1
    assert eng.lib().uwvk_pose_tail_chunks(B, 8 * slots, E) > 1  # the persistent plan
    assert not pair or eng.lib().uwvk_pose_tail_chunks(B // 2, 8 * slots, E) > 1  # the pair units' plan
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E, "C3")
    ref = _run(eng, B, 53, log, cfg, uwv, -1, [(0, E)], persist=pair, pair=pair)
    g = eng.PoseUKFBatch(B, 53)
    g.set_tail_slots(slots)
    g.set_persist(persist)
    g.set_pair(pair)
    g.set_wait_bound(0)  # every chunk k > 0 gives up at once
    g.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    g.set_process_noise_from_config(cfg, 1e-3)
    dlog = g.upload_log(log)
    with pytest.raises(eng.UWVKError, match="UWVK_ESCHEDULE"):
        g.run_log(dlog, 0, E)
    g.synchronize()
    st = g.get_status()
    bad = (st & 0x8) != 0
    assert bad.any() and not bad.all()
    x, P = g.get_state()
    np.testing.assert_array_equal(x[~bad], ref[0][~bad])
    np.testing.assert_array_equal(P[~bad], ref[1][~bad])
    # the fault word was cleared: an unspread launch reports OK
    g.set_tail_slots(-1)
    g.set_wait_bound(-1)
    g.run_log(dlog, 0, E)
