#!/usr/bin/env python3
"""Per-component consistency of the synthetic C3 scenario on the CPU oracle
(diagnostic; the oracle is the checker, this measures the scenario, not the
engine): B instances from the bench's Monte-Carlo start, run in windows, and at
each checkpoint the ensemble mean of e_i^2 / P_ii for position, orientation
(side-aware log error) and velocity axes, plus the 9-DOF NEES.  A consistent
filter reads ~1 per axis.  NEES_LEFT=1: the left (nav-frame) SO3 side.
NEES_GYRO_OLD=1: the generator's gyro noise before r05i (1/dt times the modelled variance).
NEES_STRAIGHT=1: a constant-heading truth.

usage: tools/nees_components.py [B] [EPOCHS] [STEP]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import oracle_ctypes as O  # noqa: E402
from uwvk import synth  # noqa: E402
from bench import initialise  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
E = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
STEP = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
mode = os.environ.get("NEES_MODE", "C3")


RIGHT = os.environ.get("NEES_LEFT") != "1"


def qerr(q, qt):  # right side: log(qt^-1 q) (body frame); left: log(q qt^-1) (nav frame)
    w = qt[:, 0:1] * q[:, 0:1] + np.sum(qt[:, 1:] * q[:, 1:], 1, keepdims=True)
    cr = np.cross(qt[:, 1:], q[:, 1:])
    v = qt[:, 0:1] * q[:, 1:] - q[:, 0:1] * qt[:, 1:] + (-cr if RIGHT else cr)
    s = np.sign(w)
    w, v = w * s, v * s
    n = np.linalg.norm(v, axis=1, keepdims=True)
    return 2.0 * np.arctan2(n, w) * np.where(n > 0, v / np.where(n > 0, n, 1), 0)




class StraightTruth(synth.Truth):
    """NEES_STRAIGHT=1: the same truth with a constant heading (no turn, so no
    horizontal acceleration), everything derived as in synth.Truth."""

    def __init__(self, epochs, dt=1e-3, **kw):
        super().__init__(epochs, dt, **kw)
        t = self.t
        self.psi, self.r = np.zeros_like(t), np.zeros_like(t)
        self.v_nav = np.stack([self.speed * np.ones_like(t), np.zeros_like(t), np.zeros_like(t)], -1)
        self.a_nav = np.zeros((len(t), 3))
        self.pos[1:, 0] = np.cumsum(self.speed * np.ones(len(t) - 1) * dt)
        self.pos[1:, 1] = 0.0
        self.q = np.stack([np.ones_like(t), np.zeros_like(t), np.zeros_like(t), np.zeros_like(t)], -1)
        er = synth.EARTHW * np.array([np.cos(synth.LAT0), 0.0, np.sin(synth.LAT0)])
        self.gyro = np.broadcast_to(er, (len(t), 3)).copy()
        self.acc = np.broadcast_to(np.array([0, 0, self.g]), (len(t), 3)).copy()
        self.dvl = self.v_nav.copy()


if os.environ.get("NEES_STRAIGHT") == "1":
    synth.Truth = StraightTruth
cfg, uwv = synth.default_pose_config(), synth.default_uwv()
log = synth.make_pose_log(B, E, mode=mode, dof=53, cfg=cfg)
tr = log["truth"]
if os.environ.get("NEES_GYRO_OLD") == "1":
    # the pre-r05i generator's gyro noise: sd randomwalk / sqrt(dt) per sample,
    # 1/dt times the variance the filter's process noise models (PoseUKF.cpp:408,462)
    k = np.arange(1, E + 1)
    log["gyro"] = tr.gyro[k][:, None, :] + (log["gyro"] - tr.gyro[k][:, None, :]) / np.sqrt(log["dt"])
with O.so3_side(RIGHT):
    o = O.OraclePoseBatch(B, 53, timing=True)
    initialise(o, log, cfg, uwv, "mc")
    o.set_process_noise_from_config(cfg, log["dt"])
    print("epoch   pos x/y/z            ori r/p/y            vel x/y/z          NEES9")
    for e in range(0, E, STEP):
        o.run_log(log, first=e, count=min(STEP, E - e), nthreads=8)
        x, P = o.get_state()
        k = min(E, e + STEP)
        xt = tr.state(k, 53)
        ep = x[:, 0:3] - xt[0:3]
        eo = qerr(x[:, 3:7], np.broadcast_to(xt[3:7], (B, 4)))
        ev = x[:, 7:10] - xt[7:10]
        err = np.concatenate([ep, eo, ev], 1)
        Pd = P[:, :9, :9]
        nees = np.einsum("bi,bij,bj->b", err, np.linalg.inv(Pd), err)
        r = np.mean(err ** 2 / np.diagonal(Pd, axis1=1, axis2=2), 0)
        print("%5d  %s  %s  %s  %6.2f" % (k, " ".join("%6.2f" % v for v in r[0:3]), " ".join("%6.2f" % v for v in r[3:6]),
                                          " ".join("%6.2f" % v for v in r[6:9]), nees.mean()), flush=True)
