import sys, numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, "slam-uwv_kalman_filters_amd/python")
from helpers import cov_err, init_both, pose_setup, state_err
import oracle_ctypes as orc
from uwvk import engine as eng, abi
import test_gpu_surface as T
for path in ("psp", "dense"):
  for off, bias in ((0, False), (5e4, False), (0, True), (5e4, True)):
    B = 5
    cfg, uwv, log = pose_setup(B, 53, "C4", 600)
    o, g = orc.OraclePoseBatch(B, 53), T._mk(eng, B, 53, path)
    init_both(o, g, cfg, uwv, log)
    x, P = o.get_state()
    x[:, 0] += np.linspace(-off, off, B)
    if bias:
        x[:, 13:16] = np.array([1e-4, -2e-4, 3e-4])
    loc = abi.Location(0.925, 0.154, 0.0)
    for f in (o, g):
        f.init_from_state(x, P, loc, uwv, T._param())
    for n in (1, 10, 100, 300):
        T._run_both(o, g, log, 0 if n == 1 else prev, n - (0 if n == 1 else prev))
        prev = n
        (xo, Po), (xg, Pg) = o.get_state(), g.get_state()
        print(path, off, bias, "epochs", n, "state err per inst", np.array2string(state_err(xg, xo, Po, 53), precision=2), "cov", "%.2e" % cov_err(Pg, Po).max())
