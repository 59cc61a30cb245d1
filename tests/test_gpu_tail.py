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


def _run(eng, B, dof, log, cfg, uwv, slots, pieces):
    g = eng.PoseUKFBatch(B, dof)
    g.set_tail_slots(slots)
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
