#!/usr/bin/env python3
"""Per-phase cycle shares of the fused PoseUKF epoch kernel (diagnostic build).

Loads libuwvk_stamps.so (make -C slam-uwv_kalman_filters_amd stamps), runs C3
epochs and prints the average s_memtime cycles per workgroup-epoch per phase.
Read the SHARES, not the absolute length (stamps serialise the kernel).
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
from uwvk import engine, synth  # noqa: E402

NAMES = {0: "predict: Q' + Cholesky", 1: "predict: sigma gen + process model", 2: "predict: manifold mean",
         3: "predict: deviations + MFMA GEMM + store", 4: "update: Cholesky", 5: "update: gen + h + z-mean + S",
         6: "update: cross-cov C", 7: "update: gain + Sigma -= C K^T", 8: "apply_delta: Cholesky",
         9: "apply_delta: gen + shift", 10: "apply_delta: MFMA GEMM + store", 11: "load mu/Sigma",
         12: "epoch bookkeeping", 13: "store mu/Sigma",
         20: "psp predict: partial Cholesky + stage", 21: "psp predict: points (orientation)",
         22: "psp predict: manifold mean", 23: "psp predict: ori blocks + L Delta", 24: "psp predict: A-coupled rows",
         25: "psp predict: flat pass (decay, ori, Q')", 26: "psp predict: mean update",
         30: "psp update: partial Cholesky + stage", 31: "psp update: points + zbar + S_nl",
         32: "psp update: H, P, G", 33: "psp update: C, S, gain", 34: "psp update: Sigma -= C K^T",
         35: "psp update: apply_delta", 40: "psp load", 41: "psp epoch inputs"}

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--epochs", type=int, default=20)
ap.add_argument("--dense", action="store_true", help="literal kernels (k_pose_epoch) instead of PSP")
ap.add_argument("--so3-left", action="store_true", help="the left SO3 side (SR = 0 kernels; default right)")
a = ap.parse_args()
L = engine.lib(os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "libuwvk_stamps.so"))
cfg, uwv = synth.default_pose_config(), synth.default_uwv()
log = synth.make_pose_log(a.batch, a.epochs + 1, "C3")
f = engine.PoseUKFBatch(a.batch)
if a.dense:
    f.set_dense_sigma(True)
f.set_so3_right(not a.so3_left)
# each side's PSP translation unit has its own stamp sums (the _r reader: SR = 1)
read = L.uwvk_debug_read_stamps if a.dense else (L.uwvk_debug_read_stamps_psp if a.so3_left
                                                 else L.uwvk_debug_read_stamps_psp_r)
f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
f.set_process_noise_from_config(cfg, log["dt"])
d = f.upload_log(log)
f.run_log(d, 0, 1)
s = np.zeros(64, np.uint64)
c = np.zeros(64, np.uint64)
read(s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p), 1)
f.timer_start()
f.run_log(d, 1, a.epochs)
ms = f.timer_stop()
read(s.ctypes.data_as(C.c_void_p), c.ctypes.data_as(C.c_void_p), 1)
tot = float(s.sum())
print("diagnostic build: %.2f ms/epoch (stamped, serialised)" % (ms / a.epochs))
print("%-45s %14s %8s" % ("phase", "cycles/call", "share"))
for k in range(64):
    if c[k]:
        print("%-45s %14.0f %7.1f%%" % (NAMES.get(k, str(k)), s[k] / c[k], 100.0 * s[k] / tot))
