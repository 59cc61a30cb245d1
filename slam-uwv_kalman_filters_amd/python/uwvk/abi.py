"""ctypes mirror of include/uwvk.h (the C ABI of the batched UKF engine).

Only plain data types live here; `uwvk.engine` binds the HIP library and the
test-only oracle wrapper (oracle/oracle_ctypes.py) binds the CPU restatement.
Struct field order must match include/uwvk.h exactly.
"""
import ctypes as C

D = C.c_double


def _arr(t, n):
    return t * n


class InertialNoise(C.Structure):  # PoseUKFConfig.hpp:50-63
    _fields_ = [("randomwalk", _arr(D, 3)), ("bias_offset", _arr(D, 3)),
                ("bias_instability", _arr(D, 3)), ("bias_tau", D)]


class ModelNoise(C.Structure):  # PoseUKFConfig.hpp:65-97
    _fields_ = [("body_efforts_std", _arr(D, 6)), ("inertia_instability", _arr(D, 9)),
                ("lin_damping_instability", _arr(D, 9)), ("quad_damping_instability", _arr(D, 9)),
                ("inertia_tau", D), ("lin_damping_tau", D), ("quad_damping_tau", D)]


class WaterVelocity(C.Structure):  # PoseUKFConfig.hpp:20-48
    _fields_ = [("tau", D), ("limits", D), ("measurement_std", _arr(D, 3)), ("scale", D),
                ("cell_size", D), ("first_cell_blank", D), ("minimum_correlation", D),
                ("adcp_bias_tau", D), ("adcp_bias_limits", D)]


class Location(C.Structure):  # PoseUKFConfig.hpp:99-109
    _fields_ = [("latitude", D), ("longitude", D), ("altitude", D)]


class Hydrostatics(C.Structure):  # PoseUKFConfig.hpp:145-157
    _fields_ = [("water_density", D), ("water_density_limits", D), ("water_density_tau", D),
                ("atmospheric_pressure", D), ("pressure_std", D)]


class PoseConfig(C.Structure):  # PoseUKFConfig.hpp:159-194
    _fields_ = [("acceleration", InertialNoise), ("rotation_rate", InertialNoise),
                ("model_noise_parameters", ModelNoise), ("water_velocity", WaterVelocity),
                ("location", Location), ("hydrostatics", Hydrostatics),
                ("max_jerk", _arr(D, 3)), ("max_effort", _arr(D, 6)), ("dynamic_model_min_depth", D)]


class UWVParams(C.Structure):  # [EXT] uwv_dynamic_model::UWVParameters subset
    _fields_ = [("inertia_matrix", _arr(D, 36)), ("damping_matrices", _arr(_arr(D, 36), 2)),
                ("weight", D), ("buoyancy", D),
                ("distance_body2centerofgravity", _arr(D, 3)),
                ("distance_body2centerofbuoyancy", _arr(D, 3))]


class PoseParameter(C.Structure):  # PoseUKF.hpp:46-76
    _fields_ = [("imu_in_body", _arr(D, 3)), ("gyro_bias_offset", _arr(D, 3)), ("gyro_bias_tau", D),
                ("acc_bias_offset", _arr(D, 3)), ("acc_bias_tau", D), ("inertia_tau", D),
                ("lin_damping_tau", D), ("quad_damping_tau", D), ("water_velocity_tau", D),
                ("water_velocity_limits", D), ("water_velocity_scale", D), ("adcp_bias_tau", D),
                ("atmospheric_pressure", D), ("water_density_tau", D)]


P = C.c_void_p


class PoseLog(C.Structure):  # uwvk_pose_log (device pointers)
    _fields_ = [("epochs", C.c_int64), ("dt", D), ("flags", P), ("gyro", P), ("acc", P),
                ("acc_cov", _arr(D, 9)), ("dvl_index", P), ("dvl", P), ("dvl_cov", _arr(D, 9)),
                ("pressure_index", P), ("pressure", P), ("pressure_cov", D),
                ("pressure_sensor_in_imu", _arr(D, 3)), ("adcp_index", P), ("adcp", P),
                ("adcp_cells", C.c_int32), ("adcp_cell_weighting", _arr(D, 8)), ("adcp_cov", _arr(D, 4)),
                ("efforts_index", P), ("efforts", P), ("efforts_cov", _arr(D, 36)),
                ("host_flags", P)]


class VelLog(C.Structure):  # uwvk_vel_log (device pointers)
    _fields_ = [("epochs", C.c_int64), ("dt", D), ("flags", P), ("gyro", P), ("efforts", P),
                ("dvl_index", P), ("dvl", P), ("dvl_cov", _arr(D, 9)),
                ("pressure_index", P), ("pressure", P), ("pressure_cov", D)]


class StreamTimes(C.Structure):  # uwvk_stream_times (host pointers)
    _fields_ = [("imu", P), ("n_imu", C.c_int64), ("dvl", P), ("n_dvl", C.c_int64),
                ("pressure", P), ("n_pressure", C.c_int64), ("adcp", P), ("n_adcp", C.c_int64),
                ("efforts", P), ("n_efforts", C.c_int64), ("efforts_velocity_only", P)]


class Schedule(C.Structure):  # uwvk_schedule (host pointers)
    _fields_ = [("flags", P), ("dvl_index", P), ("pressure_index", P), ("adcp_index", P),
                ("efforts_index", P), ("dt", D), ("epochs", C.c_int64),
                ("kept", _arr(C.c_int64, 4)), ("dropped", _arr(C.c_int64, 4))]


# event flags (include/uwvk.h)
EV_ACC = 0x1
EV_DVL = 0x2
EV_PRESSURE = 0x4
EV_ADCP = 0x8
EV_EFFORTS = 0x10
EV_EFFORTS_VELOCITY_ONLY = 0x20

STATUS = {0: "UWVK_OK", 1: "UWVK_EINVAL", 2: "UWVK_ENAN", 3: "UWVK_ENOTPD", 4: "UWVK_ENOMODEL",
          5: "UWVK_EDEVICE", 6: "UWVK_ENOMEM", 7: "UWVK_ENOTINIT", 8: "UWVK_ESCHEDULE"}

# storage / tangent layout of PoseState (PoseState.hpp:29-45)
FULL = dict(dof=53, store=54, s_pos=0, s_quat=3, s_vel=7, s_acc=10, s_bg=13, s_ba=16, s_grav=19,
            s_inertia=20, s_lin=29, s_quad=38, s_wv=47, s_wvb=49, s_badcp=51, s_rho=53,
            d_pos=0, d_ori=3, d_vel=6, d_acc=9, d_bg=12, d_ba=15, d_grav=18, d_inertia=19, d_lin=28,
            d_quad=37, d_wv=46, d_wvb=48, d_badcp=50, d_rho=52)
KIN = dict(dof=26, store=27, s_pos=0, s_quat=3, s_vel=7, s_acc=10, s_bg=13, s_ba=16, s_grav=19,
           s_inertia=None, s_lin=None, s_quad=None, s_wv=20, s_wvb=22, s_badcp=24, s_rho=26,
           d_pos=0, d_ori=3, d_vel=6, d_acc=9, d_bg=12, d_ba=15, d_grav=18, d_inertia=None, d_lin=None,
           d_quad=None, d_wv=19, d_wvb=21, d_badcp=23, d_rho=25)


def layout(dof):
    return FULL if dof == 53 else KIN


def fill(arr, values):
    for i, v in enumerate(values):
        arr[i] = float(v)
