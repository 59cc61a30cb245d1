#!/usr/bin/env python3
"""Run the same PoseUKF workloads through two builds of libuwvk.so (one
subprocess each) and compare the results bit for bit: the default PSP path
(with its literal BodyEfforts kernel) and the literal dense path, C4 logs with
compressed drop-out cycles.
usage: python tools/diag_lib_bitwise.py LIB_A LIB_B"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out):
    sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
    from uwvk import engine, synth
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    res = {}
    for name, dof, dense, B, E in (("psp53", 53, False, 256, 800), ("dense53", 53, True, 16, 400),
                                   ("psp26", 26, False, 256, 800), ("dense26", 26, True, 16, 400)):
        log = synth.make_pose_log(B, E, "C4", dof=dof, dropout_on=0.1, dropout_off=0.05)
        f = engine.PoseUKFBatch(B, dof)
        if dense:
            f.set_dense_sigma(True)
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, log["dt"])
        f.run_log(f.upload_log(log))
        x, P = f.get_state()
        res[name + "_x"], res[name + "_P"] = x, P
    np.savez(out, **res)


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    outs = []
    for k, libp in enumerate(sys.argv[1:3]):
        out = "/tmp/diag_lib_%d.npz" % k
        env = dict(os.environ, UWVK_LIB=os.path.abspath(libp))
        subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True, timeout=600)
        outs.append(np.load(out))
    bad = 0
    for key in outs[0].files:
        a, b = outs[0][key], outs[1][key]
        same = np.array_equal(a, b)
        diff = 0.0 if same else float(np.max(np.abs(a - b) / (np.abs(a) + 1e-300)))
        print("%-10s %s  max rel diff %.3e" % (key, "bitwise equal" if same else "DIFFER", diff))
        bad += 0 if same else 1
    sys.exit(1 if bad else 0)
