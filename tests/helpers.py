"""Shared helpers for the parity tests (oracle vs HIP engine)."""
import numpy as np

from uwvk import abi, synth


def qlog_err(qa, qb):
    """Rotation angle (rad) between quaternion arrays [..., 4] (w, x, y, z)."""
    w = np.sum(qa * qb, axis=-1)  # (qa * conj(qb)).w
    aw, av = qa[..., :1], qa[..., 1:]
    bw, bv = qb[..., :1], qb[..., 1:]
    v = bw * av - aw * bv - np.cross(av, bv)  # vector part of qa * conj(qb)
    return 2.0 * np.arctan2(np.linalg.norm(v, axis=-1), np.abs(w))


def state_err(xa, xb, P, dof):
    """Per-instance max error of xa vs xb in units of the reference std-dev
    (orientation: rotation angle over the smallest orientation std-dev)."""
    L = abi.layout(dof)
    sd = np.sqrt(np.maximum(np.diagonal(P, axis1=-2, axis2=-1), 1e-300))
    errs = []
    for d in range(dof):
        if 3 <= d < 6:
            continue
        s = d if d < 3 else d + 1
        errs.append(np.abs(xa[:, s] - xb[:, s]) / sd[:, d])
    ang = qlog_err(xa[:, 3:7], xb[:, 3:7]) / np.min(sd[:, 3:6], axis=1)
    errs.append(ang)
    return np.max(np.stack(errs, 1), axis=1)


def cov_err(Pa, Pb):
    """max |Pa - Pb| / sqrt(diag_i diag_j) of the reference Pb."""
    d = np.sqrt(np.maximum(np.diagonal(Pb, axis1=-2, axis2=-1), 1e-300))
    return np.max(np.abs(Pa - Pb) / (d[:, :, None] * d[:, None, :]), axis=(1, 2))


def pose_setup(batch, dof=53, mode="C3", epochs=10, seed=synth.SEED):
    cfg = synth.default_pose_config()
    uwv = synth.default_uwv()
    log = synth.make_pose_log(batch, epochs, mode=mode, seed=seed, dof=dof)
    return cfg, uwv, log


def init_both(oracle, engine, cfg, uwv, log, dt=1e-3):
    for f in (oracle, engine):
        f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        f.set_process_noise_from_config(cfg, dt)


def qrot_inv(q, v):
    """conj(q) v q for arrays of unit quaternions [..., 4] (w, x, y, z) and vectors [..., 3]."""
    w, u = q[..., :1], -q[..., 1:]
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)
