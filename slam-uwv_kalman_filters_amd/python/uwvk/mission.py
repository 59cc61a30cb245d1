"""Recorded-mission replay: per-sensor stamped sample streams -> the
epoch-indexed log of uwvk_pose_run_log.

The reference is driven sample by sample by its caller's stream aligner (the
Rock orogen task, outside the repository): one RotationRate +
predictionStep + Acceleration per IMU sample (PoseUKF.cpp:446-496), DVL /
pressure / ADCP / BodyEfforts integrated as their samples arrive
(PoseUKF.cpp:476-611).  `schedule()` calls the native scheduler
(uwvk_schedule_streams in libuwvk.so, host code, no GPU needed) that assigns
each lower-rate sample to its epoch; `build_pose_log()` assembles the log dict
that PoseUKFBatch.upload_log / the oracle's run_log consume.  `save()` /
`load()` keep a mission in one .npz file (plain arrays, no pickles).

Payload arrays are per instance ([samples][batch][m]) or broadcast to the batch
([samples][m]); ADCP pings carry all cells: [pings][cells][batch][2].
"""
import ctypes as C

import numpy as np

from . import abi
from .engine import _chk, lib

SENSORS = ("dvl", "pressure", "adcp", "efforts")


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def schedule(imu_t, dvl_t=None, pressure_t=None, adcp_t=None, efforts_t=None, efforts_velocity_only=None,
             dt_tolerance=0.05, time_epsilon=1e-9):
    """Native stream scheduler.  Returns dict(dt, epochs, flags, <sensor>_index, kept, dropped)."""
    imu_t = np.ascontiguousarray(imu_t, np.float64)
    E = len(imu_t)
    streams = dict(dvl=dvl_t, pressure=pressure_t, adcp=adcp_t, efforts=efforts_t)
    keep = {}
    tin = abi.StreamTimes()
    tin.imu, tin.n_imu = _p(imu_t), E
    for k in SENSORS:
        t = streams[k]
        t = np.zeros(0) if t is None else np.ascontiguousarray(t, np.float64)
        keep[k] = t
        setattr(tin, k, _p(t) if len(t) else None)
        setattr(tin, "n_" + k, len(t))
    evo = None
    if efforts_velocity_only is not None:
        evo = np.ascontiguousarray(efforts_velocity_only, np.uint8)
        tin.efforts_velocity_only = _p(evo)
    out = dict(flags=np.zeros(E, np.uint32))
    sc = abi.Schedule()
    sc.flags = _p(out["flags"])
    for k in SENSORS:
        out[k + "_index"] = np.full(E, -1, np.int32)
        setattr(sc, k + "_index", _p(out[k + "_index"]))
    _chk(lib().uwvk_schedule_streams(C.byref(tin), C.c_double(dt_tolerance), C.c_double(time_epsilon),
                                     C.byref(sc)), "uwvk_schedule_streams")
    out.update(dt=sc.dt, epochs=sc.epochs, kept=np.array(sc.kept[:]), dropped=np.array(sc.dropped[:]))
    return out


def cell_weighting(water_velocity, cells, correlation=None):
    """uwvk_adcp_cell_weighting: per-cell weight of the lower water layer and validity."""
    w = np.zeros(cells)
    v = np.zeros(cells, np.uint8)
    corr = None if correlation is None else np.ascontiguousarray(correlation, np.float64)
    _chk(lib().uwvk_adcp_cell_weighting(C.byref(water_velocity), C.c_int32(cells), _p(corr), _p(w), _p(v)),
         "uwvk_adcp_cell_weighting")
    return w, v.astype(bool)


def _per_instance(a, batch, tail):
    """[samples][*tail] broadcast or [samples][batch][*tail] -> [samples][batch][*tail]."""
    a = np.asarray(a, np.float64)
    if a.ndim == 1 + len(tail):
        a = np.broadcast_to(a[:, None], (a.shape[0], batch) + tuple(tail))
    if a.shape[1:] != (batch,) + tuple(tail):
        raise ValueError("payload shape %s does not match batch %d x %s" % (a.shape, batch, tail))
    return np.ascontiguousarray(a)


def build_pose_log(batch, imu_t, gyro, acc, acc_cov, dvl=None, pressure=None, adcp=None, efforts=None,
                   pressure_sensor_in_imu=(0.0, 0.0, 0.0), adcp_cell_weighting=None, dt_tolerance=0.05,
                   time_epsilon=1e-9):
    """Log dict of a recorded mission.

    gyro, acc: [E][batch][3] or [E][3].  dvl / pressure / efforts: (stamps, mu, cov)
    tuples, mu [n][batch][m] or [n][m].  adcp: (stamps, mu [n][cells][batch][2] or
    [n][cells][2], cov 2x2).  efforts may carry a 4th element: velocity-only flags.
    Samples the scheduler drops are removed from the payload (rows follow the
    kept samples)."""
    def stamps(s):
        return None if s is None else np.asarray(s[0], np.float64)

    sch = schedule(imu_t, stamps(dvl), stamps(pressure), stamps(adcp), stamps(efforts),
                   None if efforts is None or len(efforts) < 4 else efforts[3], dt_tolerance, time_epsilon)
    E = sch["epochs"]

    def kept_rows(name, s):
        """payload rows that the schedule placed (the leading `kept` samples
        after dropping the ones stamped before the first IMU sample)."""
        if s is None:
            return None
        t = np.asarray(s[0], np.float64)
        first = int(np.searchsorted(t, np.asarray(imu_t, np.float64)[0] - time_epsilon, side="left"))
        k = int(sch["kept"][SENSORS.index(name)])
        return slice(first, first + k)

    log = dict(mode="mission", batch=batch, epochs=E, dt=sch["dt"], flags=sch["flags"],
               gyro=_per_instance(gyro, batch, (3,)), acc=_per_instance(acc, batch, (3,)),
               acc_cov=np.asarray(acc_cov),
               kept=sch["kept"], dropped=sch["dropped"])
    if log["gyro"].shape[0] != E or log["acc"].shape[0] != E:
        raise ValueError("gyro/acc need one row per IMU stamp")
    for name, m, default_cov in (("dvl", 3, np.eye(3)), ("pressure", None, 1.0), ("efforts", 6, np.eye(6))):
        s = (locals()[name])
        log[name + "_index"] = sch[name + "_index"]
        if s is None:
            shape = (0, batch) + ((m,) if m else ())
            log[name], log[name + "_cov"] = np.zeros(shape), default_cov
            continue
        rows = kept_rows(name, s)
        mu = np.asarray(s[1], np.float64)[rows]
        log[name] = _per_instance(mu, batch, (m,) if m else ())
        if m is None:
            log[name] = log[name].reshape(-1, batch)
        log[name + "_cov"] = s[2]
    log["pressure_cov"] = float(np.asarray(log["pressure_cov"]).ravel()[0])
    log["pressure_sensor_in_imu"] = np.asarray(pressure_sensor_in_imu, np.float64)
    log["adcp_index"] = sch["adcp_index"]
    if adcp is None:
        log.update(adcp=np.zeros((0, 1, batch, 2)), adcp_cells=1, adcp_cell_weighting=np.zeros(1),
                   adcp_cov=np.eye(2))
    else:
        mu = np.asarray(adcp[1], np.float64)[kept_rows("adcp", adcp)]
        cells = mu.shape[1]
        if mu.ndim == 3:
            mu = np.broadcast_to(mu[:, :, None], (mu.shape[0], cells, batch, 2))
        if cells > 8:
            raise ValueError("at most 8 ADCP cells per ping (uwvk_pose_log.adcp_cell_weighting)")
        w = np.linspace(0.0, 1.0, cells) if adcp_cell_weighting is None else np.asarray(adcp_cell_weighting)
        log.update(adcp=np.ascontiguousarray(mu), adcp_cells=cells, adcp_cell_weighting=w,
                   adcp_cov=np.asarray(adcp[2]))
    # efforts velocity-only flags are part of `flags` (UWVK_EV_EFFORTS_VELOCITY_ONLY)
    return log


_ARRAYS = ("flags", "gyro", "acc", "acc_cov", "dvl_index", "dvl", "dvl_cov", "pressure_index", "pressure",
           "pressure_sensor_in_imu", "adcp_index", "adcp", "adcp_cell_weighting", "adcp_cov", "efforts_index",
           "efforts", "efforts_cov")
_SCALARS = ("batch", "epochs", "dt", "pressure_cov", "adcp_cells")


def save(path, log):
    """Write a (scheduled) pose log to one .npz (arrays only)."""
    d = {k: np.asarray(log[k]) for k in _ARRAYS}
    d.update({k: np.asarray(log[k]) for k in _SCALARS})
    np.savez(path, **d)


def load(path):
    """Read a log written by save() (numpy.load without pickles)."""
    with np.load(path, allow_pickle=False) as z:
        log = {k: z[k] for k in _ARRAYS}
        log.update({k: z[k].item() for k in _SCALARS})
    log["mode"] = "mission"
    return log
