"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py).

CPU: the oracle reproduces its committed fixtures (regression pin of the
oracle).  GPU (-m gpu): the HIP engine, through the C ABI, reproduces the
same checkpoints within the fp64 log tolerance.  Each pose fixture records
its SO3 side (`so3_right`: pose_*.npz the default right side, pose_*_left.npz
the left option); oracle and engine run on that side."""
import glob
import os

import numpy as np
import pytest

import oracle_ctypes as O
from helpers import cov_err, state_err
from uwvk import synth

HERE = os.path.dirname(os.path.abspath(__file__))
POSE = sorted(glob.glob(os.path.join(HERE, "golden", "pose_*.npz")))
TOL_GPU = 1e-7


def _log(g):
    log = {k: g[k] for k in g.files}
    log["epochs"] = int(g["epochs"])
    log["dt"] = float(g["dt"])
    log["adcp_cells"] = int(g["adcp_cells"])
    return log


def _run(f, g, chunk, runner):
    """Run f over the fixture log in `mu_every` chunks, collecting checkpoints."""
    mus, covs = [], []
    cov_ep = set(g["cov_epochs"].tolist())
    for e0 in range(0, int(g["epochs"]), chunk):
        runner(e0, chunk)
        x, P = f.get_state()
        mus.append(x)
        if e0 + chunk in cov_ep:
            covs.append(P)
    return np.stack(mus), np.stack(covs)


def test_fixture_sides():
    """Both sides are pinned: every default-side fixture has its left twin."""
    right = [p for p in POSE if not p.endswith("_left.npz")]
    assert right and all(int(np.load(p)["so3_right"]) == 1 for p in right)
    for p in right:
        left = p[:-4] + "_left.npz"
        assert left in POSE and int(np.load(left)["so3_right"]) == 0


@pytest.mark.parametrize("path", POSE, ids=[os.path.basename(p) for p in POSE])
def test_oracle_reproduces_fixture(path):
    g = np.load(path, allow_pickle=False)
    log = _log(g)
    dof, B = int(g["dof"]), g["mu"].shape[1]
    o = O.OraclePoseBatch(B, dof)
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    chunk = int(g["mu_epochs"][0])
    with O.so3_side(bool(g["so3_right"])):
        o.init_from_config(g["pos0"], g["pos_cov"], g["rot0"], g["rot_cov"], cfg, uwv)
        o.set_process_noise_from_config(cfg, log["dt"])
        mus, covs = _run(o, g, chunk, lambda e0, n: o.run_log(log, e0, n))
    for k in range(len(mus)):
        P = g["cov"][-1]
        assert state_err(mus[k], g["mu"][k], P, dof).max() < 1e-11
    for k in range(len(covs)):
        assert cov_err(covs[k], g["cov"][k]).max() < 1e-11


def test_oracle_reproduces_vel_fixture():
    g = np.load(os.path.join(HERE, "golden", "vel_c2.npz"), allow_pickle=False)
    log = {k: g[k] for k in g.files}
    log["epochs"], log["dt"] = int(g["epochs"]), float(g["dt"])
    o = O.OracleVelBatch(g["x0"].shape[0])
    o.init(g["x0"], g["P0"])
    o.set_gyro(g["gyro"][0])
    o.setup_motion_model(synth.default_uwv())
    for k, e0 in enumerate(range(0, log["epochs"], int(g["every"]))):
        o.run_log(log, e0, int(g["every"]))
        x, P, m = o.get_state(model=True)
        sd = np.sqrt(np.diagonal(g["cov"][k], axis1=1, axis2=2))
        assert np.max(np.abs(x - g["mu"][k]) / sd) < 1e-11
        assert cov_err(P, g["cov"][k]).max() < 1e-11
        assert np.max(np.abs(m - g["model"][k])) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("engine_path", ["psp", "dense", "literal"])
@pytest.mark.parametrize("path", POSE, ids=[os.path.basename(p) for p in POSE])
def test_engine_reproduces_fixture(path, engine_path):
    from uwvk import engine
    if not engine.device_available(0):
        pytest.fail("no gfx950 device: the HIP path is mandatory for -m gpu")
    g = np.load(path, allow_pickle=False)
    log = _log(g)
    dof, B = int(g["dof"]), g["mu"].shape[1]
    f = engine.PoseUKFBatch(B, dof)
    f.set_so3_right(bool(g["so3_right"]))
    f.set_dense_sigma(engine_path == "dense")
    f.set_literal_apply_delta(engine_path == "literal")
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    f.init_from_config(g["pos0"], g["pos_cov"], g["rot0"], g["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    d = f.upload_log(log)
    acc = engine.DeviceBuffer(np.zeros((B, 4), np.uint32))
    chunk = int(g["mu_epochs"][0])
    mus, covs = _run(f, g, chunk, lambda e0, n: f.run_log(d, e0, n, accept_counts=acc))
    np.testing.assert_array_equal(acc.read(np.uint32, (B, 4)), g["accept_counts"])
    for k in range(len(mus)):
        assert state_err(mus[k], g["mu"][k], g["cov"][-1], dof).max() < TOL_GPU, k
    for k in range(len(covs)):
        assert cov_err(covs[k], g["cov"][k]).max() < TOL_GPU, k
    assert not f.get_status().any()


@pytest.mark.gpu
@pytest.mark.parametrize("groups", [0, 1])
def test_engine_reproduces_vel_fixture(groups):
    from uwvk import engine
    g = np.load(os.path.join(HERE, "golden", "vel_c2.npz"), allow_pickle=False)
    log = {k: g[k] for k in g.files}
    log["epochs"], log["dt"] = int(g["epochs"]), float(g["dt"])
    f = engine.VelocityUKFBatch(g["x0"].shape[0])
    f.set_lane_groups(groups)
    f.init(g["x0"], g["P0"])
    f.set_gyro(g["gyro"][0])
    f.setup_motion_model(synth.default_uwv())
    d = f.upload_log(log)
    for k, e0 in enumerate(range(0, log["epochs"], int(g["every"]))):
        f.run_log(d, e0, int(g["every"]))
        x, P, m = f.get_state(model=True)
        sd = np.sqrt(np.diagonal(g["cov"][k], axis1=1, axis2=2))
        assert np.max(np.abs(x - g["mu"][k]) / sd) < TOL_GPU
        assert cov_err(P, g["cov"][k]).max() < TOL_GPU
        assert np.max(np.abs(m - g["model"][k])) < 1e-9


def test_oracle_vel_runner_matches_step_api():
    """or_vel_run_log (threaded native loop, the C2 cpu_baseline) == the per-call API loop, bitwise."""
    log = synth.make_vel_log(6, 450)
    uwv = synth.default_uwv()
    a, b = O.OracleVelBatch(6), O.OracleVelBatch(6)
    for f in (a, b):
        f.init(log["x0"], log["P0"])
        f.set_gyro(log["gyro"][0])
        f.setup_motion_model(uwv)
    a.run_log(log, nthreads=3)
    b.run_log_steps(log)
    for u, v in zip(a.get_state(model=True), b.get_state(model=True)):
        np.testing.assert_array_equal(u, v)
