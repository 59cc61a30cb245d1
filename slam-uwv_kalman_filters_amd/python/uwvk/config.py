"""Filter configuration files: PoseUKFConfig / UWVParameters / engine options
from YAML or JSON, and back.

The reference has no file format (SURVEY.md §5 "Config / flags"): its
`PoseUKFConfig` (PoseUKFConfig.hpp:159-194) is a typelib-exported struct that
the (out-of-repo) orogen task fills from a Rock YAML configuration section.
This loader reads that section's shape: the keys are the struct's own field
names (acceleration, rotation_rate, model_noise_parameters, water_velocity,
location, visual_landmarks, hydrostatics, max_jerk, max_effort,
dynamic_model_min_depth), and an Eigen vector may be written either as a plain
list or as typelib's `{data: [...]}`.  Unknown keys, missing arrays of the
wrong length and non-numeric values are errors that name the offending path;
fields the file leaves out keep the value of the `base` config (the synthetic
defaults of `synth.default_pose_config` unless given).

A file holds up to four top-level sections:

    pose_config:  PoseUKFConfig (PoseUKFConfig.hpp:159-194)
    uwv:          the uwv_dynamic_model::UWVParameters subset the engine uses
                  (inertia_matrix, damping_matrices: 6x6 nested lists or 36
                  values row-major; weight, buoyancy, distance_body2center*)
    engine:       handle options (so3_right, dense_sigma, literal_apply_delta,
                  tail_slots, tail_chunks, persist, param_block, pair), `apply_engine_options`
    visual_landmarks may also sit at top level instead of inside pose_config.

`visual_landmarks` (VisualLandmarkConfiguration, PoseUKFConfig.hpp:111-143) is
not part of the C ABI's PoseConfig POD: the reference's PoseUKF never reads it
(only its orogen task does, to build the arguments of
integrateMeasurement(vector<VisualFeatureMeasurement>, ...), PoseUKF.cpp:613-654).
`VisualLandmarks.landmark_args(marker_id)` builds those arguments for
`PoseUKFBatch.update_visual`: feature positions = unit positions x marker_size / 2,
marker pose t(3) q(w,x,y,z) from marker_position and marker_euler_orientation,
and cov_marker_pose = diag(marker_pose_std^2).  The Euler convention is
Rock's base::getEuler order (yaw, pitch, roll), R = Rz(yaw) Ry(pitch) Rx(roll):
the task that consumed it is not in the reference, so that convention is
parity-unpinned.
"""
import ctypes as C
import json
import math

import numpy as np

from . import abi

ENGINE_OPTIONS = ("so3_right", "dense_sigma", "literal_apply_delta", "tail_slots", "tail_chunks", "persist",
                  "param_block", "pair")


class ConfigError(ValueError):
    pass


def _is_array(t):
    return isinstance(t, type) and issubclass(t, C.Array)


def _is_struct(t):
    return isinstance(t, type) and issubclass(t, C.Structure)


def _num(v, path):
    if isinstance(v, bool) or not isinstance(v, (int, float)):
        raise ConfigError("%s: expected a number, got %r" % (path, v))
    v = float(v)
    if math.isnan(v):
        raise ConfigError("%s: NaN" % path)
    return v


def _flat(v, path):
    """A list, nested lists (matrices, row-major) or typelib's {data: [...]}."""
    if isinstance(v, dict):
        if set(v) != {"data"}:
            raise ConfigError("%s: an array is a list or {data: [...]}, got keys %s" % (path, sorted(v)))
        v = v["data"]
    if not isinstance(v, (list, tuple)):
        raise ConfigError("%s: expected a list, got %r" % (path, v))
    out = []
    for i, x in enumerate(v):
        if isinstance(x, (list, tuple)):
            out.extend(_flat(x, "%s[%d]" % (path, i)))
        else:
            out.append(_num(x, "%s[%d]" % (path, i)))
    return out


def _fill_array(arr, v, path):
    et = arr._type_
    if _is_array(et):  # array of arrays (damping_matrices): one entry per sub-array
        if not isinstance(v, (list, tuple)) or len(v) != len(arr):
            raise ConfigError("%s: expected %d entries" % (path, len(arr)))
        for i, x in enumerate(v):
            _fill_array(arr[i], x, "%s[%d]" % (path, i))
        return
    vals = _flat(v, path)
    if len(vals) != len(arr):
        raise ConfigError("%s: expected %d values, got %d" % (path, len(arr), len(vals)))
    for i, x in enumerate(vals):
        arr[i] = x


def fill_struct(s, d, path=""):
    """Write the mapping d into the ctypes structure s (in place), strictly."""
    if not isinstance(d, dict):
        raise ConfigError("%s: expected a mapping, got %r" % (path or "<root>", d))
    types = dict(s._fields_)
    for k, v in d.items():
        p = "%s.%s" % (path, k) if path else k
        if k not in types:
            raise ConfigError("%s: unknown field (known: %s)" % (p, ", ".join(types)))
        t = types[k]
        if _is_struct(t):
            fill_struct(getattr(s, k), v, p)
        elif _is_array(t):
            _fill_array(getattr(s, k), v, p)
        else:
            setattr(s, k, _num(v, p))
    return s


def struct_to_dict(s):
    out = {}
    for k, t in s._fields_:
        v = getattr(s, k)
        if _is_struct(t):
            out[k] = struct_to_dict(v)
        elif _is_array(t):
            out[k] = [list(x) for x in v] if _is_array(t._type_) else list(v)
        else:
            out[k] = float(v)
    return out


def _copy(s):
    n = type(s)()
    C.memmove(C.addressof(n), C.addressof(s), C.sizeof(s))
    return n


def euler_to_quat(euler):
    """(yaw, pitch, roll) -> q(w, x, y, z) of Rz(yaw) Ry(pitch) Rx(roll)."""
    y, p, r = (0.5 * float(a) for a in euler)
    cy, sy, cp, sp, cr, sr = math.cos(y), math.sin(y), math.cos(p), math.sin(p), math.cos(r), math.sin(r)
    return np.array([cy * cp * cr + sy * sp * sr, cy * cp * sr - sy * sp * cr,
                     cy * sp * cr + sy * cp * sr, sy * cp * cr - cy * sp * sr])


class VisualLandmarks:
    """VisualLandmarkConfiguration (PoseUKFConfig.hpp:111-143)."""

    FIELDS = ("camera_config", "feature_std", "unit_feature_positions", "landmarks")
    LANDMARK = ("marker_id", "marker_size", "marker_position", "marker_euler_orientation", "marker_pose_std")

    def __init__(self, d, path="visual_landmarks"):
        if not isinstance(d, dict):
            raise ConfigError("%s: expected a mapping" % path)
        for k in d:
            if k not in self.FIELDS:
                raise ConfigError("%s.%s: unknown field (known: %s)" % (path, k, ", ".join(self.FIELDS)))
        cam = d.get("camera_config", {})
        for k in cam:
            if k not in ("fx", "fy", "cx", "cy"):
                raise ConfigError("%s.camera_config.%s: unknown field" % (path, k))
        self.camera = np.array([_num(cam.get(k, 0.0), "%s.camera_config.%s" % (path, k))
                                for k in ("fx", "fy", "cx", "cy")])
        fs = _flat(d.get("feature_std", [1.0, 1.0]), path + ".feature_std")
        if len(fs) != 2:
            raise ConfigError("%s.feature_std: expected 2 values" % path)
        self.feature_std = np.array(fs)
        ufp = d.get("unit_feature_positions", [])
        self.unit_feature_positions = np.array([_flat(v, "%s.unit_feature_positions[%d]" % (path, i))
                                                for i, v in enumerate(ufp)]).reshape(-1, 3)
        self.landmarks = {}
        for i, lm in enumerate(d.get("landmarks", [])):
            p = "%s.landmarks[%d]" % (path, i)
            if not isinstance(lm, dict):
                raise ConfigError("%s: expected a mapping" % p)
            for k in lm:
                if k not in self.LANDMARK:
                    raise ConfigError("%s.%s: unknown field" % (p, k))
            mid = str(lm.get("marker_id", ""))
            if not mid or mid in self.landmarks:
                raise ConfigError("%s.marker_id: missing or duplicate %r" % (p, mid))
            e = dict(marker_size=_num(lm.get("marker_size", 0.0), p + ".marker_size"))
            for k, n in (("marker_position", 3), ("marker_euler_orientation", 3), ("marker_pose_std", 6)):
                v = _flat(lm.get(k, [0.0] * n), "%s.%s" % (p, k))
                if len(v) != n:
                    raise ConfigError("%s.%s: expected %d values, got %d" % (p, k, n, len(v)))
                e[k] = np.array(v)
            self.landmarks[mid] = e

    def feature_cov(self):
        """[nf, 4]: diag(feature_std^2) per feature (px^2)."""
        nf = len(self.unit_feature_positions)
        c = np.diag(self.feature_std ** 2).ravel()
        return np.tile(c, (nf, 1))

    def landmark_args(self, marker_id):
        """feature_positions [nf, 3], marker_pose [7], cov_marker_pose [36], camera [4]."""
        if marker_id not in self.landmarks:
            raise KeyError("unknown marker_id %r (known: %s)" % (marker_id, ", ".join(self.landmarks)))
        lm = self.landmarks[marker_id]
        fp = self.unit_feature_positions * (0.5 * lm["marker_size"])
        pose = np.concatenate([lm["marker_position"], euler_to_quat(lm["marker_euler_orientation"])])
        cov = np.diag(lm["marker_pose_std"] ** 2).ravel()
        return fp, pose, cov, self.camera.copy()

    def to_dict(self):
        return {
            "camera_config": dict(zip(("fx", "fy", "cx", "cy"), map(float, self.camera))),
            "feature_std": self.feature_std.tolist(),
            "unit_feature_positions": self.unit_feature_positions.tolist(),
            "landmarks": [dict(marker_id=k, marker_size=v["marker_size"],
                               **{f: v[f].tolist() for f in self.LANDMARK[2:]}) for k, v in self.landmarks.items()],
        }


class FilterConfig:
    """The parsed file: pose (abi.PoseConfig), uwv (abi.UWVParams), engine
    options (dict) and visual (VisualLandmarks or None)."""

    def __init__(self, pose, uwv, engine=None, visual=None):
        self.pose, self.uwv, self.engine, self.visual = pose, uwv, dict(engine or {}), visual

    def to_dict(self):
        d = {"pose_config": struct_to_dict(self.pose), "uwv": struct_to_dict(self.uwv)}
        if self.visual is not None:
            d["pose_config"]["visual_landmarks"] = self.visual.to_dict()
        if self.engine:
            d["engine"] = dict(self.engine)
        return d


def from_dict(d, base_pose=None, base_uwv=None):
    from . import synth
    if not isinstance(d, dict):
        raise ConfigError("<root>: expected a mapping")
    for k in d:
        if k not in ("pose_config", "uwv", "engine", "visual_landmarks"):
            raise ConfigError("%s: unknown section (known: pose_config, uwv, engine, visual_landmarks)" % k)
    pose = _copy(base_pose) if base_pose is not None else synth.default_pose_config()
    uwv = _copy(base_uwv) if base_uwv is not None else synth.default_uwv()
    pc = dict(d.get("pose_config") or {})
    vis = pc.pop("visual_landmarks", None)
    if "visual_landmarks" in d:
        if vis is not None:
            raise ConfigError("visual_landmarks: given both at top level and in pose_config")
        vis = d["visual_landmarks"]
    fill_struct(pose, pc, "pose_config")
    fill_struct(uwv, d.get("uwv") or {}, "uwv")
    eng = dict(d.get("engine") or {})
    for k, v in eng.items():
        if k not in ENGINE_OPTIONS:
            raise ConfigError("engine.%s: unknown option (known: %s)" % (k, ", ".join(ENGINE_OPTIONS)))
        if k in ("so3_right", "dense_sigma", "literal_apply_delta", "param_block", "pair"):
            if not isinstance(v, bool):
                raise ConfigError("engine.%s: expected true / false, got %r" % (k, v))
        elif k == "persist":
            # UWVK_OPT_PERSIST is 0 / 1 (a boolean in YAML reads the same)
            if not (isinstance(v, bool) or (isinstance(v, int) and v in (0, 1))):
                raise ConfigError("engine.persist: expected 0 / 1 or true / false, got %r" % (v,))
            eng[k] = int(v)
        elif k == "tail_slots":
            # UWVK_OPT_TAIL_SLOTS: 0 runtime occupancy, > 0 blocks per XCD, < 0 (-1) no tail spreading
            if isinstance(v, bool) or not isinstance(v, int) or v < -1:
                raise ConfigError("engine.tail_slots: expected an integer >= -1, got %r" % (v,))
        elif isinstance(v, bool) or not isinstance(v, int) or v < 0:
            raise ConfigError("engine.%s: expected a non-negative integer, got %r" % (k, v))
    return FilterConfig(pose, uwv, eng, VisualLandmarks(vis) if vis is not None else None)


def loads(text, fmt="yaml", **kw):
    if fmt == "json":
        d = json.loads(text)
    else:
        import yaml
        d = yaml.safe_load(text)  # plain data only: no tags, no object construction
    return from_dict(d or {}, **kw)


def load(path, **kw):
    """YAML (.yaml / .yml) or JSON (.json) file -> FilterConfig."""
    with open(path) as f:
        text = f.read()
    return loads(text, "json" if str(path).endswith(".json") else "yaml", **kw)


def dump(cfg, path):
    d = cfg.to_dict()
    with open(path, "w") as f:
        if str(path).endswith(".json"):
            json.dump(d, f, indent=1)
        else:
            import yaml
            yaml.safe_dump(d, f, sort_keys=False)


def apply_engine_options(batch, opts):
    """Engine options on a PoseUKFBatch (each maps to a uwvk_pose_set_option).
    Applied after the caller's own settings, so an option the file sets wins
    over the same option set on the command line (bench.py warns when both
    are given and differ)."""
    for k, v in opts.items():
        if k == "so3_right":
            batch.set_so3_right(v)
        elif k == "dense_sigma":
            batch.set_dense_sigma(v)
        elif k == "literal_apply_delta":
            batch.set_literal_apply_delta(v)
        elif k == "tail_slots":
            batch.set_tail_slots(v)
        elif k == "tail_chunks":
            batch.set_tail_chunks(v)
        elif k == "persist":
            batch.set_persist(int(v))
        elif k == "param_block":
            batch.set_param_block(bool(v))
        elif k == "pair":
            batch.set_pair(bool(v))
        else:
            raise ConfigError("engine.%s: unknown option" % k)
