#!/usr/bin/env python3
"""Per-phase cycle shares of k_pose_efforts_epoch (the literal BodyEfforts
update of run_log's PSP split), diagnostic build libuwvk_stamps.so
(make -C slam-uwv_kalman_filters_amd stamps).  Runs a C4 window holding
BodyEfforts epochs and prints the s_memtime cycles per workgroup-call of each
phase of that kernel (its own translation unit, so only its stamps).
Also times the plain build's efforts launches with HIP events.
usage: python tools/efforts_stamps.py [--batch 65536]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
from uwvk import abi, engine, synth  # noqa: E402

NAMES = {4: "update: 53-col Cholesky", 5: "update: gen + h + z-mean + S", 6: "update: cross-cov C",
         7: "update: gain + Sigma -= C K^T", 10: "apply_delta (T Sigma T^T)", 11: "load mu/Sigma",
         12: "update return", 13: "store mu/Sigma"}

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
L = engine.lib(os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "libuwvk_stamps.so"))
cfg, uwv = synth.default_pose_config(), synth.default_uwv()
E = 400
log = synth.make_pose_log(a.batch, E, "C4", dropout_on=0.1, dropout_off=0.05)
eff = np.nonzero(log["flags"] & abi.EV_EFFORTS)[0]
print("efforts epochs in the window:", list(eff))
f = engine.PoseUKFBatch(a.batch)
f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
f.set_process_noise_from_config(cfg, log["dt"])
d = f.upload_log(log)
s = np.zeros(64, np.uint64)
c = np.zeros(64, np.uint64)
L.uwvk_debug_read_stamps_eff(s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p), 1)
f.run_log(d, 0, E)
L.uwvk_debug_read_stamps_eff(s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p), 1)
tot = float(s.sum())
print("%-40s %14s %8s" % ("phase", "cycles/call", "share"))
for k in range(64):
    if c[k]:
        print("%-40s %14.0f %7.1f%%" % (NAMES.get(k, str(k)), s[k] / c[k], 100.0 * s[k] / tot))
