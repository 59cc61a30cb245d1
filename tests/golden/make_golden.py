#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ with the CPU oracle.

The reference (tomcreutz/slam-uwv_kalman_filters) cannot be built or run here
(its UKF arithmetic lives in absent third-party libraries: SURVEY.md K3) and
ships no test vectors (K4), so these fixtures are produced by the fp64 C oracle
(oracle/uwvk_oracle.c), itself cross-checked by the numpy twin and the
known-answer tests.  Each .npz holds the INPUTS (the full measurement log and
initial state) and checkpointed OUTPUTS (mean every `mu_every` epochs,
covariance every `cov_every` epochs), so a fixture is self-contained.

SO3 side: pose_*.npz run the default right side (q exp(d),
MTK's SO3::boxplus); pose_*_left.npz the same logs on the left side (exp(d) q,
the option).  Each file records its side in `so3_right`.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle_ctypes as O  # noqa: E402
from uwvk import synth  # noqa: E402

LOG_KEYS = ["flags", "gyro", "acc", "acc_cov", "dvl_index", "dvl", "dvl_cov", "pressure_index", "pressure",
            "pressure_cov", "pressure_sensor_in_imu", "adcp_index", "adcp", "adcp_cells", "adcp_cell_weighting",
            "adcp_cov", "efforts_index", "efforts", "efforts_cov", "pos0", "pos_cov", "rot0", "rot_cov"]

CASES = {
    # C1: single PoseUKF, 1 kHz IMU + 5 Hz DVL, full and kinematic layouts
    "pose_c1_dof53": dict(dof=53, mode="C3", batch=1, epochs=2000, mu_every=100, cov_every=500),
    "pose_c1_dof26": dict(dof=26, mode="C3", batch=1, epochs=2000, mu_every=100, cov_every=500),
    # C4-style: pressure, ADCP x4 (d2p95), DVL drop-out with BodyEfforts (compressed schedule)
    "pose_c4_dof53": dict(dof=53, mode="C4", batch=2, epochs=3000, mu_every=100, cov_every=1000,
                          kw=dict(dropout_on=1.0, dropout_off=0.5, adcp_every=500)),
    "pose_c4v_dof53": dict(dof=53, mode="C4", batch=1, epochs=3000, mu_every=100, cov_every=1000,
                           kw=dict(dropout_on=1.0, dropout_off=0.5, adcp_every=500, efforts_velocity_only=True)),
}


def make_pose(name, c, right=True):
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(c["batch"], c["epochs"], mode=c["mode"], dof=c["dof"], **c.get("kw", {}))
    o = O.OraclePoseBatch(c["batch"], c["dof"])
    mus, covs, mu_ep, cov_ep = [], [], [], []
    counts = np.zeros((c["batch"], 4), np.uint32)
    with O.so3_side(right):
        o.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        o.set_process_noise_from_config(cfg, log["dt"])
        for e0 in range(0, c["epochs"], c["mu_every"]):
            counts += o.run_log(log, e0, c["mu_every"])
            x, P = o.get_state()
            e = e0 + c["mu_every"]
            mus.append(x)
            mu_ep.append(e)
            if e % c["cov_every"] == 0:
                covs.append(P)
                cov_ep.append(e)
    out = {k: np.asarray(log[k]) for k in LOG_KEYS}
    out.update(dof=c["dof"], epochs=c["epochs"], dt=log["dt"], mu=np.stack(mus), mu_epochs=np.array(mu_ep),
               cov=np.stack(covs), cov_epochs=np.array(cov_ep), accept_counts=counts, so3_right=int(right))
    fn = name + ("" if right else "_left")
    np.savez_compressed(os.path.join(HERE, fn + ".npz"), **out)
    print(fn, "mu", out["mu"].shape, "cov", out["cov"].shape, "accepts", counts.tolist())


def make_vel():
    uwv = synth.default_uwv()
    log = synth.make_vel_log(4, 1000)
    o = O.OracleVelBatch(4)
    o.init(log["x0"], log["P0"])
    o.set_gyro(log["gyro"][0])
    o.setup_motion_model(uwv)
    mus, covs, models = [], [], []
    for e0 in range(0, 1000, 100):
        o.run_log(log, e0, 100)
        x, P, m = o.get_state(model=True)
        mus.append(x)
        covs.append(P)
        models.append(m)
    keys = ["flags", "gyro", "efforts", "dvl_index", "dvl", "dvl_cov", "pressure_index", "pressure",
            "pressure_cov", "x0", "P0"]
    out = {k: np.asarray(log[k]) for k in keys}
    out.update(epochs=1000, dt=log["dt"], mu=np.stack(mus), cov=np.stack(covs), model=np.stack(models),
               every=100)
    np.savez_compressed(os.path.join(HERE, "vel_c2.npz"), **out)
    print("vel_c2", out["mu"].shape)


if __name__ == "__main__":
    for right in (True, False):
        for name, c in CASES.items():
            make_pose(name, c, right)
    make_vel()
