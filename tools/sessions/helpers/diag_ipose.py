"""GPU diagnostic: IndirectPoseUKF test sequence step by step vs the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("slam-uwv_kalman_filters_amd/python", "oracle", "tests"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np
import oracle_ctypes as O
from uwvk.small import IndirectPoseUKFBatch
import test_small_filters as T

if 'pre' in sys.argv:
    T.test_gpu_bottom_sequence(); T.test_gpu_bottom_mask_and_errors(); print('ran bottom tests first')
B = 13
ref, p_err, q_err, marker, px = T.ipose_scene(B)
g, o = IndirectPoseUKFBatch(B), O.OracleIndirectPoseBatch(B)
ipe = np.random.default_rng(2).normal(0, 0.1, (B, 3))
for f in (g, o):
    f.init([0.1, 0.1, 0.2], [0.01, 0.01, 0.02], 20.0, ipe, [0.5, 0.5, 0.5])
    f.set_pose_reference(ref)
fcov, fpos, cm, cam, cib = T.visual_common(B)

def rep(tag):
    (xg, Pg), (xo, Po) = g.get_state(), o.get_state()
    d = np.abs(xg - xo).max(1)
    print(tag, "dx per inst", np.array2string(d, precision=2), "dP", np.abs(Pg - Po).max())
    print("   truth p_err", p_err[0], "\n   g", xg[0], "\n   o", xo[0])

rep("init")
for step in range(4):
    for f in (g, o):
        f.predict(0.1)
    rep("predict %d" % step)
    for nf in (1, 4):
        pass
    for f in (g, o):
        f.update_visual(px, fcov, fpos, marker, cm, cam, cib)
    rep("visual %d" % step)
