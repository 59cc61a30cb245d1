"""Batched BottomUKF (BottomUKF.hpp:26-53) and IndirectPoseUKF
(IndirectPoseUKF.hpp:28-86) over the C ABI (uwvk_bottom_* / uwvk_ipose_*).

Like the rest of the package there is no CPU fallback: construction raises
UWVKError(UWVK_EDEVICE) without a gfx950 device."""
import ctypes as C

import numpy as np

from .engine import VP, _chk, _f64, _p, lib, visual_args


def _per(a, batch, tail):
    a = np.asarray(a, np.float64)
    if a.shape == tuple(tail):
        a = np.broadcast_to(a, (batch,) + tuple(tail))
    return np.ascontiguousarray(a)


class _Small:
    PREFIX = None
    STORE = DOF = None

    def __init__(self, batch, device=0):
        self.L = lib()
        self.batch, self.device = batch, device
        self.h = VP()
        getattr(self.L, self.PREFIX + "_destroy").argtypes = [VP]
        _chk(getattr(self.L, self.PREFIX + "_create")(C.c_int64(batch), device, C.byref(self.h)),
             self.PREFIX + "_create")

    def _fn(self, name):
        return getattr(self.L, "%s_%s" % (self.PREFIX, name))

    def close(self):
        if self.h:
            self._fn("destroy")(self.h)
            self.h = VP()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def get_state(self):
        x = np.empty((self.batch, self.STORE))
        P = np.empty((self.batch, self.DOF, self.DOF))
        _chk(self._fn("get_state")(self.h, _p(x), _p(P)), "get_state")
        return x, P

    def get_status(self, clear=False):
        out = np.zeros(self.batch, np.uint32)
        _chk(self._fn("get_status")(self.h, _p(out), int(clear)), "get_status")
        return out


class BottomUKFBatch(_Small):
    """Batched BottomUKF: state {distance, normal (S2)}, stored (d, nx, ny, nz)."""
    PREFIX, STORE, DOF = "uwvk_bottom", 4, 3

    def init(self, x, P):
        x, P = _f64(x), _f64(P)
        _chk(self._fn("init")(self.h, _p(x), _p(P)), "bottom_init")

    def set_process_noise(self, Q):
        Q = _f64(Q)
        _chk(self._fn("set_process_noise")(self.h, _p(Q)), "bottom_set_process_noise")

    def set_velocity(self, v):
        v = _per(v, self.batch, (3,))
        _chk(self._fn("set_velocity")(self.h, _p(v)), "bottom_set_velocity")

    def predict(self, dt):
        _chk(self._fn("predict")(self.h, C.c_double(dt)), "bottom_predict")

    def update_range(self, mu, cov, direction, origin, mask=None):
        mu = _per(mu, self.batch, ())
        cv = np.asarray(cov, np.float64)
        shared = cv.ndim == 0
        cvp = None if shared else _per(cv, self.batch, ())
        d, o = _f64(direction), _f64(origin)
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        _chk(self._fn("update_range")(self.h, _p(mu), _p(cvp), C.c_double(float(cv) if shared else 0.0), _p(d),
                                      _p(o), _p(m)), "bottom_update_range")

    def update_normal(self, mu, cov, mask=None):
        mu = _per(mu, self.batch, (3,))
        cv = np.asarray(cov, np.float64)
        shared = cv.shape == (2, 2)
        cvp = _f64(cv) if not shared else None
        sc = _f64(cv) if shared else None
        m = None if mask is None else np.ascontiguousarray(mask, np.uint8)
        _chk(self._fn("update_normal")(self.h, _p(mu), _p(cvp), _p(sc), _p(m)), "bottom_update_normal")


class IndirectPoseUKFBatch(_Small):
    """Batched IndirectPoseUKF: state {position_error, orientation_error}, stored t(3) q(4)."""
    PREFIX, STORE, DOF = "uwvk_ipose", 7, 6

    def init(self, pos_std, ori_std, tau, init_pos_err=None, init_pos_std=None):
        ipe = None if init_pos_err is None else _per(init_pos_err, self.batch, (3,))
        ips = None if init_pos_std is None else _f64(init_pos_std)
        a, b = _f64(pos_std), _f64(ori_std)
        _chk(self._fn("init")(self.h, _p(a), _p(b), C.c_double(tau), _p(ipe), _p(ips)), "ipose_init")

    def set_process_noise(self, Q):
        """setProcessNoiseCovariance [EXT base]: 6x6 shared by the batch."""
        Q = _f64(Q)
        _chk(self._fn("set_process_noise")(self.h, _p(Q)), "ipose_set_process_noise")

    def set_so3_right(self, on=True):
        """UWVK_OPT_SO3_RIGHT of the orientation_error: body frame q exp(d) (the
        default, MTK's SO3::boxplus) or, on=False, nav frame exp(d) q."""
        _chk(self._fn("set_option")(self.h, 5, int(bool(on))), "ipose_set_option")

    def set_pose_reference(self, pose):
        pose = _per(pose, self.batch, (7,))
        _chk(self._fn("set_pose_reference")(self.h, _p(pose)), "ipose_set_pose_reference")

    def predict(self, dt):
        _chk(self._fn("predict")(self.h, C.c_double(dt)), "ipose_predict")

    def update_visual(self, features, feature_cov, feature_positions, marker_pose, cov_marker_pose, camera,
                      camera_in_body, mask=None):
        args, keep = visual_args(self.batch, features, feature_cov, feature_positions, marker_pose,
                                 cov_marker_pose, camera, camera_in_body, mask)
        _chk(self._fn("update_visual")(self.h, *args), "ipose_update_visual")

    def get_corrected_pose(self):
        out = np.empty((self.batch, 7))
        _chk(self._fn("get_corrected_pose")(self.h, _p(out)), "ipose_get_corrected_pose")
        return out
