#!/usr/bin/env python3
"""Times single-call updates at batch 65,536: the BodyEfforts update
(uwvk_pose_update_efforts) on PSP (r05) and on the literal kernel, its
velocity-only form (constrainVelocity) on PSP (r05) and on the literal kernel, and the acceleration update on the dense path:
HIP events on the handle's stream around 5 calls each (each call includes its
measurement upload).  UWVK_LIB selects a variant library."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
from uwvk import engine, synth  # noqa: E402

B = 65536
cfg, uwv = synth.default_pose_config(), synth.default_uwv()
log = synth.make_pose_log(B, 2, "C3")
f = engine.PoseUKFBatch(B, 53, device=0)
f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
f.set_process_noise_from_config(cfg, log["dt"])
rng = np.random.default_rng(1)
eff = rng.normal(0, 1.0, (B, 6))
ecov = np.eye(6) * 1e2
acc = np.tile([0.0, 0.0, 9.81], (B, 1)) + rng.normal(0, 1e-3, (B, 3))
acov = np.eye(3) * 1e-4
out = {}
for name, call in (("efforts", lambda: f.update("efforts", eff, ecov, only_vel=0)),
                   ("efforts_dense", lambda: f.update("efforts", eff, ecov, only_vel=0)),
                   ("efforts_vo_psp", lambda: f.update("efforts", eff, ecov, only_vel=1)),
                   ("efforts_vo_dense", lambda: f.update("efforts", eff, ecov, only_vel=1)),
                   ("acceleration_dense", lambda: f.update("acceleration", acc, acov))):
    f.set_dense_sigma(name.endswith("_dense"))
    call()
    f.synchronize()
    f.timer_start()
    for _ in range(5):
        call()
    out[name] = f.timer_stop() / 5
print(" ".join("%s %.3f ms" % kv for kv in out.items()), "status", int((f.get_status() != 0).sum()))
