"""ctypes binding of libuwvk.so — the MI355X batched UKF engine.

Mirrors the reference's class surface (PoseUKF.hpp:89-255, VelocityUKF.hpp:231-266)
in batched form: every method acts on `batch` independent filter instances held
in device memory.  There is no CPU fallback: without the HIP library or a
gfx950 device, construction raises `UWVKError` (UWVK_EDEVICE).
"""
import ctypes as C
import os

import numpy as np

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(HERE))  # slam-uwv_kalman_filters_amd/
# UWVK_LIB selects an alternative build of the same ABI (A/B performance variants)
LIB_PATH = os.environ.get("UWVK_LIB") or os.path.join(PKG, "libuwvk.so")

# every symbol include/uwvk.h declares (checked by tests/test_abi.py)
SYMBOLS = [
    "uwvk_abi_version", "uwvk_device_available", "uwvk_status_string", "uwvk_last_device_error", "uwvk_device_malloc", "uwvk_device_free",
    "uwvk_memcpy_h2d", "uwvk_memcpy_d2h", "uwvk_memcpy_h2d_on", "uwvk_memcpy_d2h_on",
    "uwvk_pose_create", "uwvk_pose_destroy", "uwvk_pose_batch", "uwvk_pose_dof", "uwvk_pose_stream",
    "uwvk_pose_synchronize", "uwvk_pose_init_from_config", "uwvk_pose_init_from_state",
    "uwvk_pose_set_process_noise_from_config", "uwvk_pose_set_process_noise", "uwvk_pose_set_rotation_rate",
    "uwvk_pose_predict", "uwvk_pose_update_acceleration", "uwvk_pose_update_velocity", "uwvk_pose_update_pressure",
    "uwvk_pose_update_water_velocity", "uwvk_pose_update_efforts", "uwvk_pose_update_xy", "uwvk_pose_update_z",
    "uwvk_pose_update_geographic", "uwvk_pose_update_delayed_xy", "uwvk_pose_reset_with_external_pose",
    "uwvk_pose_get_state", "uwvk_pose_get_rotation_rate", "uwvk_pose_get_status", "uwvk_pose_run_log",
    "uwvk_pose_ensemble_stats", "uwvk_pose_set_option", "uwvk_pose_timer_start", "uwvk_pose_timer_stop",
    "uwvk_vel_create", "uwvk_vel_destroy", "uwvk_vel_stream", "uwvk_vel_init", "uwvk_vel_setup_motion_model",
    "uwvk_vel_set_gyro", "uwvk_vel_set_efforts", "uwvk_vel_predict", "uwvk_vel_update_dvl",
    "uwvk_vel_update_pressure", "uwvk_vel_get_state", "uwvk_vel_get_model_state", "uwvk_vel_run_log",
    "uwvk_vel_set_option", "uwvk_vel_synchronize", "uwvk_vel_timer_start", "uwvk_vel_timer_stop",
    "uwvk_pose_ensemble_allreduce", "uwvk_comm_unique_id_bytes", "uwvk_comm_unique_id", "uwvk_comm_init",
    "uwvk_comm_destroy", "uwvk_comm_allreduce_sum_device", "uwvk_vel_set_process_noise",
    "uwvk_ipose_set_process_noise",
    "uwvk_schedule_streams", "uwvk_adcp_cell_weighting", "uwvk_pose_update_visual_landmark",
    "uwvk_bottom_create", "uwvk_bottom_destroy", "uwvk_bottom_stream", "uwvk_bottom_init",
    "uwvk_bottom_set_process_noise", "uwvk_bottom_set_velocity", "uwvk_bottom_predict", "uwvk_bottom_update_range",
    "uwvk_bottom_update_normal", "uwvk_bottom_get_state", "uwvk_bottom_get_status",
    "uwvk_ipose_create", "uwvk_ipose_destroy", "uwvk_ipose_stream", "uwvk_ipose_init", "uwvk_ipose_set_option",
    "uwvk_ipose_set_pose_reference", "uwvk_ipose_predict", "uwvk_ipose_update_visual",
    "uwvk_ipose_get_corrected_pose", "uwvk_ipose_get_state", "uwvk_ipose_get_status",
    "uwvk_pose_tail_chunks", "uwvk_pose_resident_slots", "uwvk_pose_epoch_qshape", "uwvk_pose_param_block", "uwvk_pose_pair_active", "uwvk_pose_timer_mark", "uwvk_pose_timer_elapsed",
    "uwvk_xcd_round_robin", "uwvk_synth_normal", "uwvk_synth_normal_at",
]

_LIB = None
ABI_VERSION = 3  # include/uwvk.h UWVK_ABI_VERSION this binding is written against
DP = C.POINTER(C.c_double)
VP = C.c_void_p


class UWVKError(RuntimeError):
    def __init__(self, code, where=""):
        self.code = code
        detail = ""
        if code == 5 and _LIB is not None:  # UWVK_EDEVICE: the HIP error behind it
            try:
                detail = (_LIB.uwvk_last_device_error() or b"").decode()
            except Exception:
                detail = ""
        super().__init__("%s%s%s" % (abi.STATUS.get(code, "UWVK_%d" % code), (" in " + where) if where else "",
                                     (" [" + detail + "]") if detail else ""))


def lib(path=None):
    """Load libuwvk.so (raises OSError if it was not built)."""
    global _LIB
    if _LIB is None or path:
        L = C.CDLL(path or LIB_PATH)
        if L.uwvk_abi_version() != ABI_VERSION:
            raise OSError("%s: ABI version %d, this binding needs %d (include/uwvk.h)"
                          % (path or LIB_PATH, L.uwvk_abi_version(), ABI_VERSION))
        L.uwvk_status_string.restype = C.c_char_p
        L.uwvk_last_device_error.restype = C.c_char_p
        L.uwvk_pose_batch.restype = C.c_int64
        L.uwvk_pose_stream.restype = VP
        L.uwvk_vel_stream.restype = VP
        L.uwvk_pose_stream.argtypes = [VP]
        L.uwvk_vel_stream.argtypes = [VP]
        L.uwvk_pose_destroy.argtypes = [VP]
        L.uwvk_vel_destroy.argtypes = [VP]
        L.uwvk_comm_destroy.argtypes = [VP]
        L.uwvk_device_free.argtypes = [VP]
        L.uwvk_pose_tail_chunks.argtypes = [C.c_int64, C.c_int64, C.c_int64]
        L.uwvk_pose_epoch_qshape.argtypes = [C.c_void_p]
        L.uwvk_pose_epoch_qshape.restype = C.c_int
        L.uwvk_pose_param_block.argtypes = [C.c_void_p]
        L.uwvk_pose_param_block.restype = C.c_int
        L.uwvk_pose_pair_active.argtypes = [C.c_void_p]
        L.uwvk_pose_pair_active.restype = C.c_int
        L.uwvk_pose_resident_slots.argtypes = [C.c_int, C.c_int]
        L.uwvk_pose_resident_slots.restype = C.c_int64
        L.uwvk_memcpy_h2d.argtypes = [VP, VP, C.c_size_t]
        L.uwvk_memcpy_d2h.argtypes = [VP, VP, C.c_size_t]
        L.uwvk_memcpy_h2d_on.argtypes = [VP, VP, C.c_size_t, VP]
        L.uwvk_memcpy_d2h_on.argtypes = [VP, VP, C.c_size_t, VP]
        L.uwvk_device_malloc.argtypes = [C.c_int, C.c_size_t, C.POINTER(VP)]
        _LIB = L
    return _LIB


def _chk(code, where=""):
    if code != 0:
        raise UWVKError(code, where)


def _f64(a):
    return None if a is None else np.ascontiguousarray(a, dtype=np.float64)


def _p(a):
    return None if a is None else a.ctypes.data_as(VP)


class DeviceBuffer:
    """A device allocation filled from a numpy array (for device-resident logs)."""

    def __init__(self, arr, device=0):
        arr = np.ascontiguousarray(arr)
        self.nbytes = max(arr.nbytes, 16)
        self.ptr = VP()
        _chk(lib().uwvk_device_malloc(device, self.nbytes, C.byref(self.ptr)), "device_malloc")
        if arr.nbytes:
            _chk(lib().uwvk_memcpy_h2d(self.ptr, arr.ctypes.data_as(VP), arr.nbytes), "memcpy_h2d")

    def read(self, dtype, shape, stream=None):
        """Copy to the host after all queued device work (stream=None), or
        ordered on one handle's stream (e.g. PoseUKFBatch.stream)."""
        out = np.empty(shape, dtype)
        if stream is None:
            _chk(lib().uwvk_memcpy_d2h(out.ctypes.data_as(VP), self.ptr, out.nbytes), "memcpy_d2h")
        else:
            _chk(lib().uwvk_memcpy_d2h_on(out.ctypes.data_as(VP), self.ptr, out.nbytes, stream), "memcpy_d2h_on")
        return out

    def free(self):
        if self.ptr:
            lib().uwvk_device_free(self.ptr)
            self.ptr = VP()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class PoseUKFBatch:
    """Batched PoseUKF (PoseUKF.hpp:89).  dof = 53 (PoseState) or 26 (kinematic subset)."""

    def __init__(self, batch, dof=53, device=0):
        self.L = lib()
        self.batch, self.dof, self.device = batch, dof, device
        self.lay = abi.layout(dof)
        self.h = VP()
        _chk(self.L.uwvk_pose_create(C.c_int64(batch), dof, device, C.byref(self.h)), "uwvk_pose_create")

    def close(self):
        if self.h:
            self.L.uwvk_pose_destroy(self.h)
            self.h = VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self):
        return self.L.uwvk_pose_stream(self.h)

    def set_dense_sigma(self, on=True):
        """Propagate all 2n+1 sigma points (literal kernels) instead of the PSP form."""
        _chk(self.L.uwvk_pose_set_option(self.h, 2, int(bool(on))), "set_option")

    def set_tail_slots(self, slots):
        """Last-generation spreading of run_log (UWVK_OPT_TAIL_SLOTS): 0 plans for
        the runtime's occupancy, > 0 for that many resident blocks per XCD, < 0 off."""
        _chk(self.L.uwvk_pose_set_option(self.h, 3, int(slots)), "set_option")

    def set_so3_right(self, on=True):
        """UWVK_OPT_SO3_RIGHT: body-frame SO3 boxplus q exp(d) (the default, MTK's
        SO3::boxplus) or, with on=False, the nav-frame exp(d) q, on every path
        (PSP, dense, literal), like the oracle's or_set_so3_right."""
        _chk(self.L.uwvk_pose_set_option(self.h, 5, int(bool(on))), "set_option")

    def set_lds_pad(self, nbytes):
        """UWVK_OPT_LDS_PAD (diagnostic): dynamic LDS bytes per PSP epoch
        workgroup, unused, to lower its occupancy (epoch-kernel occupancy sweep)."""
        _chk(self.L.uwvk_pose_set_option(self.h, 7, int(nbytes)), "set_option")

    def set_tail_chunks(self, chunks):
        """UWVK_OPT_TAIL_CHUNKS: 0 the planner's chunk count, 2..8 forced (tests)."""
        _chk(self.L.uwvk_pose_set_option(self.h, 4, int(chunks)), "set_option")

    def epoch_qshape(self):
        """The process-noise shape the PSP epoch kernel runs for: 1 simple, 2 general."""
        return int(self.L.uwvk_pose_epoch_qshape(self.h))

    def set_persist(self, on=True):
        """UWVK_OPT_PERSIST: run_log on resident workgroups that take work units
        from a ticket counter (bitwise the same results as one workgroup per instance)."""
        _chk(self.L.uwvk_pose_set_option(self.h, 6, int(bool(on))), "set_option")

    def set_wait_bound(self, sleeps):
        """UWVK_OPT_WAIT_BOUND (tests): < 0 the planner's hand-off wait bound, else
        that many ~1.7 us sleeps; 0 makes every hand-off of a spread launch time out."""
        _chk(self.L.uwvk_pose_set_option(self.h, 8, int(sleeps)), "set_option")

    def set_param_block(self, on=True):
        """UWVK_OPT_PARAM_BLOCK: run_log's launches on the parameter-decoupled
        kernel while the model-parameter block is uncoupled (default on)."""
        _chk(self.L.uwvk_pose_set_option(self.h, 9, int(bool(on))), "set_option")

    def set_pair(self, on=True):
        """UWVK_OPT_PAIR: the parameter-decoupled kernel with two instances per
        wave (persistent scheduler, even batch)."""
        _chk(self.L.uwvk_pose_set_option(self.h, 10, int(bool(on))), "set_option")

    def pair_active(self):
        """1 when the next run_log launch runs the two-instances-per-wave kernel."""
        return int(self.L.uwvk_pose_pair_active(self.h))

    def param_block(self):
        """1 when the next run_log launch runs the parameter-decoupled kernel."""
        return int(self.L.uwvk_pose_param_block(self.h))

    def set_literal_apply_delta(self, on=True):
        """ukfom's literal apply_delta re-spread instead of the exact T Sigma T^T form."""
        _chk(self.L.uwvk_pose_set_option(self.h, 1, int(bool(on))), "set_option")

    def init_from_config(self, pos, pos_cov, rot, rot_cov, cfg, uwv, imu_in_body=None):
        pos, pos_cov, rot, rot_cov, ib = map(_f64, (pos, pos_cov, rot, rot_cov, imu_in_body))
        _chk(self.L.uwvk_pose_init_from_config(self.h, _p(pos), _p(pos_cov), _p(rot), _p(rot_cov), C.byref(cfg),
                                               C.byref(uwv), _p(ib)), "init_from_config")

    def init_from_state(self, x, P, loc, uwv, param):
        x, P = _f64(x), _f64(P)
        _chk(self.L.uwvk_pose_init_from_state(self.h, _p(x), _p(P), C.byref(loc), C.byref(uwv), C.byref(param)),
             "init_from_state")

    def set_process_noise_from_config(self, cfg, dt, q_imu_in_body=None):
        q = _f64(q_imu_in_body)
        _chk(self.L.uwvk_pose_set_process_noise_from_config(self.h, C.byref(cfg), C.c_double(dt), _p(q)),
             "set_process_noise_from_config")

    def set_process_noise(self, Q):
        Q = _f64(Q)
        _chk(self.L.uwvk_pose_set_process_noise(self.h, _p(Q)), "set_process_noise")

    def set_rotation_rate(self, w, cov=None):
        w, cov = _f64(w), _f64(cov)
        _chk(self.L.uwvk_pose_set_rotation_rate(self.h, _p(w), _p(cov)), "set_rotation_rate")

    def predict(self, dt):
        _chk(self.L.uwvk_pose_predict(self.h, C.c_double(dt)), "predict")

    def update(self, kind, mu, cov, extra=None, only_vel=0, mask=None):
        """Same calling convention as the oracle wrapper: cov is m*m shared or [batch, m, m]."""
        mu = _f64(mu)
        cov = _f64(cov)
        per_inst = cov.ndim == mu.ndim + 1
        acc = np.zeros(self.batch, np.uint8)
        msk = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        args = [self.h, _p(mu), _p(cov) if per_inst else None, None if per_inst else _p(cov)]
        fn = getattr(self.L, "uwvk_pose_update_" + kind)
        if kind == "pressure":
            args.append(_p(_f64(extra if extra is not None else np.zeros(3))))
        elif kind == "water_velocity":
            cw = _f64(np.broadcast_to(np.asarray(extra, dtype=np.float64), (self.batch,)))
            args.append(_p(cw))
        elif kind == "efforts":
            args.append(C.c_int(int(only_vel)))
        elif kind == "geographic":
            args.append(_p(_f64(extra if extra is not None else np.zeros(3))))
        elif kind == "delayed_xy":
            args.append(_p(_f64(extra)))
        args += [_p(msk), _p(acc)]
        self._keep = (mu, cov, msk)
        _chk(fn(*args), "update_" + kind)
        return acc

    def update_visual(self, features, feature_cov, feature_positions, marker_pose, cov_marker_pose, camera,
                      camera_in_imu, mask=None):
        """integrateMeasurement(vector<VisualFeatureMeasurement>, ...) (PoseUKF.cpp:613-654).
        features [batch, nf, 2]; feature_cov [batch, nf, 2, 2] or [nf, 2, 2];
        feature_positions [nf, 3]; marker_pose [batch, 7] or [7]; camera (fx, fy, cx, cy)."""
        args = visual_args(self.batch, features, feature_cov, feature_positions, marker_pose, cov_marker_pose,
                           camera, camera_in_imu, mask)
        _chk(self.L.uwvk_pose_update_visual_landmark(self.h, *args[0]), "update_visual_landmark")

    def reset_with_external_pose(self, pose):
        pose = _f64(pose)
        _chk(self.L.uwvk_pose_reset_with_external_pose(self.h, _p(pose)), "reset_with_external_pose")

    def get_state(self):
        x = np.empty((self.batch, self.lay["store"]))
        P = np.empty((self.batch, self.dof, self.dof))
        _chk(self.L.uwvk_pose_get_state(self.h, _p(x), _p(P)), "get_state")
        return x, P

    def get_state_mu(self):
        """The means only (uwvk_pose_get_state with P = NULL)."""
        x = np.empty((self.batch, self.lay["store"]))
        _chk(self.L.uwvk_pose_get_state(self.h, _p(x), None), "get_state")
        return x

    def get_rotation_rate(self):
        out = np.empty((self.batch, 3))
        _chk(self.L.uwvk_pose_get_rotation_rate(self.h, _p(out)), "get_rotation_rate")
        return out

    def get_status(self, clear=False):
        out = np.zeros(self.batch, np.uint32)
        _chk(self.L.uwvk_pose_get_status(self.h, _p(out), int(clear)), "get_status")
        return out

    def synchronize(self):
        _chk(self.L.uwvk_pose_synchronize(self.h), "synchronize")

    def upload_log(self, log):
        return DevicePoseLog(log, self.device)

    def run_log(self, dlog, first=0, count=None, accept_counts=None, sync=True):
        """Queue epochs [first, first+count) on the handle's stream (PSP: one
        launch per run of epochs without BodyEfforts); sync=False leaves them in flight."""
        count = dlog.epochs - first if count is None else count
        _chk(self.L.uwvk_pose_run_log(self.h, C.byref(dlog.s), C.c_int64(first), C.c_int64(count),
                                      accept_counts.ptr if accept_counts is not None else None), "run_log")
        if sync:
            self.synchronize()

    def ensemble_stats(self, truth=None, comm=None):
        """Ensemble statistics of this handle's instances; with an RcclComm,
        summed over every rank's shard by RCCL (uwvk_pose_ensemble_allreduce)."""
        out = np.zeros(3 * self.lay["store"] + 2)
        t = _f64(truth)
        if comm is None:
            _chk(self.L.uwvk_pose_ensemble_stats(self.h, _p(t), _p(out)), "ensemble_stats")
        else:
            _chk(self.L.uwvk_pose_ensemble_allreduce(self.h, _p(t), _p(out), comm.ptr), "ensemble_allreduce")
        return out

    def timer_start(self):
        _chk(self.L.uwvk_pose_timer_start(self.h), "timer_start")

    def timer_stop(self):
        ms = C.c_float(0)
        _chk(self.L.uwvk_pose_timer_stop(self.h, C.byref(ms)), "timer_stop")
        return ms.value

    def timer_mark(self):
        """Record the stop event without waiting (uwvk_pose_timer_mark)."""
        _chk(self.L.uwvk_pose_timer_mark(self.h), "timer_mark")

    def timer_elapsed(self):
        """Wait for the event timer_mark recorded; ms since timer_start."""
        ms = C.c_float(0)
        _chk(self.L.uwvk_pose_timer_elapsed(self.h, C.byref(ms)), "timer_elapsed")
        return ms.value


class DevicePoseLog:
    """uwvk_pose_log with every array resident in device memory (HBM)."""

    def __init__(self, log, device=0):
        self.bufs = {}
        s = abi.PoseLog()
        s.epochs, s.dt = int(log["epochs"]), float(log["dt"])

        def up(name, arr, dtype):
            b = DeviceBuffer(np.ascontiguousarray(arr, dtype=dtype), device)
            self.bufs[name] = b
            return b.ptr

        s.flags = up("flags", log["flags"], np.uint32)
        s.gyro = up("gyro", log["gyro"], np.float64)
        s.acc = up("acc", log["acc"], np.float64)
        abi.fill(s.acc_cov, np.asarray(log["acc_cov"]).ravel())
        s.dvl_index = up("dvl_index", log["dvl_index"], np.int32)
        s.dvl = up("dvl", log["dvl"], np.float64)
        abi.fill(s.dvl_cov, np.asarray(log["dvl_cov"]).ravel())
        s.pressure_index = up("pressure_index", log["pressure_index"], np.int32)
        s.pressure = up("pressure", log["pressure"], np.float64)
        s.pressure_cov = float(log["pressure_cov"])
        abi.fill(s.pressure_sensor_in_imu, log["pressure_sensor_in_imu"])
        s.adcp_index = up("adcp_index", log["adcp_index"], np.int32)
        s.adcp = up("adcp", log["adcp"], np.float64)
        s.adcp_cells = int(log["adcp_cells"])
        abi.fill(s.adcp_cell_weighting, log["adcp_cell_weighting"])
        abi.fill(s.adcp_cov, np.asarray(log["adcp_cov"]).ravel())
        s.efforts_index = up("efforts_index", log["efforts_index"], np.int32)
        s.efforts = up("efforts", log["efforts"], np.float64)
        abi.fill(s.efforts_cov, np.asarray(log["efforts_cov"]).ravel())
        self.host_flags = np.ascontiguousarray(log["flags"], dtype=np.uint32)
        s.host_flags = self.host_flags.ctypes.data
        self.s = s
        self.epochs = s.epochs


class VelocityUKFBatch:
    """Batched VelocityUKF (VelocityUKF.hpp:231)."""

    def __init__(self, batch, device=0):
        self.L = lib()
        self.batch, self.device = batch, device
        self.h = VP()
        _chk(self.L.uwvk_vel_create(C.c_int64(batch), device, C.byref(self.h)), "uwvk_vel_create")

    def close(self):
        if self.h:
            self.L.uwvk_vel_destroy(self.h)
            self.h = VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init(self, x, P):
        x, P = _f64(x), _f64(P)
        _chk(self.L.uwvk_vel_init(self.h, _p(x), _p(P)), "vel_init")

    def setup_motion_model(self, uwv):
        _chk(self.L.uwvk_vel_setup_motion_model(self.h, C.byref(uwv)), "setup_motion_model")

    def set_gyro(self, w):
        w = _f64(w)
        _chk(self.L.uwvk_vel_set_gyro(self.h, _p(w), None), "set_gyro")

    def set_efforts(self, t):
        t = _f64(t)
        _chk(self.L.uwvk_vel_set_efforts(self.h, _p(t), None), "set_efforts")

    def predict(self, dt):
        _chk(self.L.uwvk_vel_predict(self.h, C.c_double(dt)), "vel_predict")

    def update_dvl(self, mu, cov):
        mu, cov = _f64(mu), _f64(cov)
        _chk(self.L.uwvk_vel_update_dvl(self.h, _p(mu), None, _p(cov), None), "update_dvl")

    def update_pressure(self, mu, cov):
        mu, cov = _f64(np.asarray(mu).reshape(-1)), _f64(np.atleast_1d(cov))
        _chk(self.L.uwvk_vel_update_pressure(self.h, _p(mu), None, _p(cov), None), "update_pressure")

    def get_state(self, model=False):
        x = np.empty((self.batch, 4))
        P = np.empty((self.batch, 4, 4))
        _chk(self.L.uwvk_vel_get_state(self.h, _p(x), _p(P)), "vel_get_state")
        if not model:
            return x, P
        ms = np.empty((self.batch, 13))
        _chk(self.L.uwvk_vel_get_model_state(self.h, _p(ms)), "vel_get_model_state")
        return x, P, ms

    def upload_log(self, log):
        return DeviceVelLog(log, self.device)

    def run_log(self, dlog, first=0, count=None, sync=True):
        count = dlog.epochs - first if count is None else count
        _chk(self.L.uwvk_vel_run_log(self.h, C.byref(dlog.s), C.c_int64(first), C.c_int64(count)), "vel_run_log")
        if sync:
            self.synchronize()

    def set_process_noise(self, Q):
        """setProcessNoiseCovariance [EXT base]: 4x4 shared by the batch."""
        Q = _f64(Q)
        _chk(self.L.uwvk_vel_set_process_noise(self.h, _p(Q)), "vel_set_process_noise")

    def set_lane_groups(self, value):
        """-1 auto, 0 one filter per lane, 1 one filter per 16 lanes (UWVK_VEL_OPT_LANE_GROUPS)."""
        _chk(self.L.uwvk_vel_set_option(self.h, 1, int(value)), "vel_set_option")

    def synchronize(self):
        _chk(self.L.uwvk_vel_synchronize(self.h), "vel_synchronize")

    def timer_start(self):
        _chk(self.L.uwvk_vel_timer_start(self.h), "vel_timer_start")

    def timer_stop(self):
        ms = C.c_float(0)
        _chk(self.L.uwvk_vel_timer_stop(self.h, C.byref(ms)), "vel_timer_stop")
        return ms.value


class DeviceVelLog:
    def __init__(self, log, device=0):
        self.bufs = {}
        s = abi.VelLog()
        s.epochs, s.dt = int(log["epochs"]), float(log["dt"])

        def up(name, arr, dtype):
            b = DeviceBuffer(np.ascontiguousarray(arr, dtype=dtype), device)
            self.bufs[name] = b
            return b.ptr

        s.flags = up("flags", log["flags"], np.uint32)
        s.gyro = up("gyro", log["gyro"], np.float64)
        s.efforts = up("efforts", log["efforts"], np.float64)
        s.dvl_index = up("dvl_index", log["dvl_index"], np.int32)
        s.dvl = up("dvl", log["dvl"], np.float64)
        abi.fill(s.dvl_cov, np.asarray(log["dvl_cov"]).ravel())
        s.pressure_index = up("pressure_index", log["pressure_index"], np.int32)
        s.pressure = up("pressure", log["pressure"], np.float64)
        s.pressure_cov = float(log["pressure_cov"])
        self.s = s
        self.epochs = s.epochs


class RcclComm:
    """An RCCL communicator made through the C ABI (uwvk_comm_*).  Rank 0 makes
    the id (RcclComm.unique_id()) and ships it to the other ranks out of band."""

    @staticmethod
    def unique_id():
        L = lib()
        n = L.uwvk_comm_unique_id_bytes()
        buf = C.create_string_buffer(n)
        _chk(L.uwvk_comm_unique_id(buf), "comm_unique_id")
        return buf.raw

    def __init__(self, nranks, uid, rank, device=0):
        self.L = lib()
        self.ptr = VP()
        _chk(self.L.uwvk_comm_init(nranks, C.c_char_p(uid), rank, device, C.byref(self.ptr)), "comm_init")

    def close(self):
        if self.ptr:
            self.L.uwvk_comm_destroy(self.ptr)
            self.ptr = VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def visual_args(batch, features, feature_cov, feature_positions, marker_pose, cov_marker_pose, camera, cam_in,
                mask=None):
    """ctypes arguments of uwvk_*_update_visual*: (args, keep-alive arrays)."""
    f = _f64(features)
    nf = f.shape[1] if f.ndim == 3 else 0
    fc = _f64(np.asarray(feature_cov, np.float64).reshape(-1, nf, 4) if nf else np.zeros(4))
    fc_pi = int(fc.shape[0] == batch and (batch > 1 or np.asarray(feature_cov).ndim == 4))
    mp = _f64(marker_pose)
    mp_pi = int(mp.ndim == 2)
    fp = _f64(np.asarray(feature_positions, np.float64).reshape(-1, 3) if nf else np.zeros(3))
    keep = [f, fc, mp, fp, _f64(cov_marker_pose), _f64(camera), _f64(cam_in)]
    msk = None if mask is None else np.ascontiguousarray(mask, np.uint8)
    keep.append(msk)
    args = [C.c_int32(nf), _p(f), _p(fc), C.c_int(fc_pi), _p(fp), _p(mp), C.c_int(mp_pi), _p(keep[4]),
            _p(keep[5]), _p(keep[6]), _p(msk)]
    return args, keep


def device_available(device=0):
    try:
        return bool(lib().uwvk_device_available(device))
    except OSError:
        return False
