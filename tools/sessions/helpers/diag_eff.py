#!/usr/bin/env python3
"""Diagnostic: one BodyEfforts update at a small batch on each engine path
(velocity-only PSP, full PSP, full literal), reporting the HIP error behind any
UWVK_EDEVICE (uwvk_last_device_error).  usage: tools/diag_eff.py [B]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
from uwvk import engine, synth  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cfg, uwv = synth.default_pose_config(), synth.default_uwv()
log = synth.make_pose_log(B, 2, "C3")
rng = np.random.default_rng(7)
eff = 20 * rng.standard_normal((B, 6))
ecov = np.diag([25.0, 25, 25, 1, 1, 1])
ORDER = (("full_psp", False, 0), ("vo_psp", False, 1), ("full_dense", True, 0))
for name, dense, vo in ORDER:
    f = engine.PoseUKFBatch(B, 53, device=0)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    f.set_dense_sigma(dense)
    try:
        acc = f.update("efforts", eff, ecov, only_vel=vo)
        x, P = f.get_state()
        print(name, "ok", acc, "finite", bool(np.isfinite(x).all() and np.isfinite(P).all()), "status",
              f.get_status().tolist(), flush=True)
    except engine.UWVKError as e:
        print(name, "ERROR", e, flush=True)
