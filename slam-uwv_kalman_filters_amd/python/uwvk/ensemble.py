"""Ensemble (Monte-Carlo / multi-vehicle) helpers for instance-sharded runs.

Instances are independent (no coupling anywhere in the reference: each filter
is self-contained, PoseUKF.hpp:195-205), so N ranks own contiguous instance
ranges and exchange nothing on the data path.  The one collective is the sum
of the ensemble statistics (uwvk_pose_ensemble_stats) — over RCCL on GPUs, over
gloo in the CPU tests.
"""
import numpy as np


def shard_range(rank, world, global_batch):
    """Contiguous instance range [lo, hi) owned by `rank`."""
    lo = global_batch * rank // world
    hi = global_batch * (rank + 1) // world
    return lo, hi


def _qlog_delta(q, t, right=True):
    """log(conj(t) * q) (body frame, the right SO3 side: the default,
    UWVK_OPT_SO3_RIGHT) or, right=False, log(q * conj(t)) (nav frame) for arrays of unit
    quaternions (w, x, y, z): the orientation error in the frame the filter's
    covariance is expressed in.  The two products differ only in the sign of
    the cross term."""
    w = q[..., 0] * t[0] + np.sum(q[..., 1:] * t[1:], -1)
    cr = np.cross(q[..., 1:], t[1:])
    v = t[0] * q[..., 1:] - q[..., :1] * t[1:] + (cr if right else -cr)
    sgn = np.where(w < 0, -1.0, 1.0)
    w, v = w * sgn, v * sgn[..., None]
    nv = np.linalg.norm(v, axis=-1)
    k = np.where(nv > 0, 2 * np.arctan2(nv, w) / np.where(nv > 0, nv, 1), 0.0)
    return k[..., None] * v


def ensemble_stats_host(x, P, truth, right=True):
    """Host reference of uwvk_pose_ensemble_stats (same layout of `out`);
    right: the handle's SO3 side (True, the default: the orientation error
    log(t^-1 q); False: log(q t^-1))."""
    store = x.shape[1]
    out = np.zeros(3 * store + 2)
    out[:store] = x.sum(0)
    out[store:2 * store] = (x * x).sum(0)
    e = x - truth
    e[:, 3:7] = 0.0
    r = _qlog_delta(x[:, 3:7], truth[3:7], right)
    sq = (e * e).sum(0)
    sq[3:6] += (r * r).sum(0)
    out[2 * store:3 * store] = sq
    err = np.concatenate([x[:, 0:3] - truth[0:3], r, x[:, 7:10] - truth[7:10]], 1)
    # the same exclusion rule as k_pose_stats: an instance is left out of the
    # NEES sum when its 9x9 block has a non-positive pivot or its NEES is not
    # finite (a NaN / Inf state); it is counted in out[3 * store + 1]
    sub = np.ascontiguousarray(P[:, :9, :9])
    with np.errstate(invalid="ignore", over="ignore"):
        try:  # every block positive definite: one batched factorisation
            Lc = np.linalg.cholesky(sub)
            y = np.linalg.solve(Lc, err[..., None])[..., 0]
            nees = np.sum(y * y, 1)
        except np.linalg.LinAlgError:  # some block is not: instance by instance
            nees = np.full(x.shape[0], np.nan)
            for i in range(x.shape[0]):
                try:
                    Li = np.linalg.cholesky(sub[i])
                except np.linalg.LinAlgError:
                    continue
                yi = np.linalg.solve(Li, err[i])
                nees[i] = float(yi @ yi)
    ok = np.isfinite(nees)
    out[3 * store] = float(np.sum(np.where(ok, nees, 0.0)))
    out[3 * store + 1] = float((~ok).sum())
    return out


def allreduce_stats(stats, dist, device=None):
    """Sum the per-rank statistics vectors (torch.distributed, any backend).
    Returns a new array; `stats` is left as it was."""
    import torch
    t = torch.from_numpy(np.array(stats, dtype=np.float64, copy=True))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t)
    return t.cpu().numpy()
