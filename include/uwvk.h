/*
 * uwvk.h — C ABI of the MI355X-native batched UKF engine (PoseUKF / VelocityUKF).
 *
 * This is the drop-in boundary for the predict / measurement-update hot path of
 * tomcreutz/slam-uwv_kalman_filters.  The reference exposes single-instance C++
 * classes (src/PoseUKF.hpp:89-255, src/VelocityUKF.hpp:231-266) that derive from
 * pose_estimation::UnscentedKalmanFilter<State> [EXT].  Each entry point below
 * names the reference member it replaces (file:line).  Every call works on a
 * BATCH of independent filter instances held in device memory by the handle;
 * batch = 1 is the reference's single-instance case.
 *
 * Conventions
 *  - Plain C types only.  Host arrays passed in are borrowed for the duration
 *    of the call (copied to the device before it returns).
 *  - Arrays are instance-major: element [i][k] of a per-instance array of width
 *    K lives at index i*K + k.  Matrices are row-major, n x n.
 *  - Quaternions are stored (w, x, y, z).
 *  - One handle owns one HIP stream and is NOT thread-safe (the reference is
 *    not re-entrant either: PoseUKF.cpp:173, VelocityUKF.cpp:18).
 *  - Errors are returned as uwvk_status codes; the C++ facade
 *    (slam-uwv_kalman_filters_amd/include/uwv_kalman_filters_amd/PoseUKF.hpp)
 *    maps them to std::runtime_error like the reference's checkMeasurment [EXT]
 *    (PoseUKF.cpp:478) and the missing-model throw (VelocityUKF.cpp:117-118).
 *  - There is NO CPU fallback: without a usable gfx950 device every create call
 *    returns UWVK_EDEVICE.
 */
#ifndef UWVK_H_
#define UWVK_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  A caller checks uwvk_abi_version() == UWVK_ABI_VERSION of the
 * header it was built against (the Python binding and the C++ facade do).
 *   1  round 1.
 *   2  uwvk_pose_ensemble_stats / _allreduce write 3*store+2 doubles (was
 *      3*store+1: the count of instances left out of the NEES sum was added);
 *      uwvk_pose_init_from_state reads only the lower triangle of P;
 *      uwvk_memcpy_h2d / _d2h wait for the buffer's own device only.
 *   3  (r05/r06) the default UWVK_OPT_SO3_RIGHT of pose and ipose handles is 1
 *      (body-frame SO3 [+], MTK's SO3::boxplus; was 0, nav frame): a caller
 *      that wants the old convention sets the option to 0;
 *      new entry points uwvk_last_device_error, uwvk_synth_normal_at,
 *      uwvk_ipose_set_option;
 *      a tail-chunk hand-off that timed out is an error of the API, not only
 *      the instances' UWVK_ST_SCHEDULE bit: the next uwvk_pose_synchronize
 *      or uwvk_pose_run_log on the handle after the launch has completed
 *      returns UWVK_ESCHEDULE (once); new option UWVK_OPT_WAIT_BOUND;
 *      UWVK_OPT_PERSIST defaults to 1 (no dispatch-order assumption). */
#define UWVK_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------ */
typedef enum uwvk_status {
  UWVK_OK = 0,
  UWVK_EINVAL = 1,   /* bad argument (null handle, wrong size, unsupported layout) */
  UWVK_ENAN = 2,     /* NaN/Inf in a measurement mean or covariance (checkMeasurment [EXT]) */
  UWVK_ENOTPD = 3,   /* covariance not positive definite in at least one instance */
  UWVK_ENOMODEL = 4, /* VelocityUKF predict without setupMotionModel (VelocityUKF.cpp:117-118) */
  UWVK_EDEVICE = 5,  /* no gfx950 device / HIP runtime error */
  UWVK_ENOMEM = 6,
  UWVK_ENOTINIT = 7, /* state or process noise not initialised */
  UWVK_ESCHEDULE = 8 /* a run_log tail-chunk hand-off timed out (instances flagged UWVK_ST_SCHEDULE);
                        returned by the next uwvk_pose_synchronize / uwvk_pose_run_log */
} uwvk_status;

/* per-instance status bits (uwvk_pose_get_status / uwvk_vel_get_status) */
#define UWVK_ST_NOTPD 0x1u    /* Cholesky of Sigma failed (non-positive pivot) */
#define UWVK_ST_NAN 0x2u      /* non-finite measurement skipped for this instance */
#define UWVK_ST_NONFINITE 0x4u/* non-finite state after a step */
/* UWVK_ST_SCHEDULE: engine fault, a tail-chunk hand-off timed out (see
 * UWVK_OPT_TAIL_SLOTS; never observed outside forced tests).  The instance's
 * state is then INVALID, not merely late: the chunks after the lost hand-off
 * did not run, and the late predecessor may have left Sigma in the kernel's
 * time-scaled (unfolded) form.  Re-initialise a flagged instance
 * (uwvk_pose_init_from_state with a state of the caller's choosing) before
 * using it again. */
#define UWVK_ST_SCHEDULE 0x8u

/* ---- PoseState layout (src/PoseState.hpp:29-45) ------------------------ */
/* Full layout: 53 DOF, 54 stored scalars (SO3 as a quaternion).           */
/* Kinematic layout: the same without inertia / lin_damping / quad_damping */
/* (26 DOF, 27 stored scalars) — the "~30-dim" config of BASELINE.json.     */
#define UWVK_POSE_DOF_FULL 53
#define UWVK_POSE_STORE_FULL 54
#define UWVK_POSE_DOF_KIN 26
#define UWVK_POSE_STORE_KIN 27
/* storage offsets, full layout */
#define UWVK_S_POS 0
#define UWVK_S_QUAT 3
#define UWVK_S_VEL 7
#define UWVK_S_ACC 10
#define UWVK_S_BIAS_GYRO 13
#define UWVK_S_BIAS_ACC 16
#define UWVK_S_GRAVITY 19
#define UWVK_S_INERTIA 20      /* 3x3 column-major (PoseState.hpp:37) */
#define UWVK_S_LIN_DAMPING 29  /* 3x3 column-major */
#define UWVK_S_QUAD_DAMPING 38 /* 3x3 column-major */
#define UWVK_S_WATER_VEL 47
#define UWVK_S_WATER_VEL_BELOW 49
#define UWVK_S_BIAS_ADCP 51
#define UWVK_S_WATER_DENSITY 53

/* ---- configuration PODs (Eigen-free mirrors of PoseUKFConfig.hpp) ------ */
typedef struct uwvk_inertial_noise { /* InertialNoiseParameters, PoseUKFConfig.hpp:50-63 */
  double randomwalk[3];
  double bias_offset[3];
  double bias_instability[3];
  double bias_tau;
} uwvk_inertial_noise;

typedef struct uwvk_model_noise { /* DynamicModelNoiseParameters, PoseUKFConfig.hpp:65-97 */
  double body_efforts_std[6];
  double inertia_instability[9];
  double lin_damping_instability[9];
  double quad_damping_instability[9];
  double inertia_tau;
  double lin_damping_tau;
  double quad_damping_tau;
} uwvk_model_noise;

typedef struct uwvk_water_velocity { /* WaterVelocityParameters, PoseUKFConfig.hpp:20-48 */
  double tau;
  double limits;
  double measurement_std[3];
  double scale;
  double cell_size;
  double first_cell_blank;
  double minimum_correlation;
  double adcp_bias_tau;
  double adcp_bias_limits;
} uwvk_water_velocity;

typedef struct uwvk_location { /* LocationConfiguration, PoseUKFConfig.hpp:99-109 */
  double latitude;  /* rad */
  double longitude; /* rad */
  double altitude;  /* m */
} uwvk_location;

typedef struct uwvk_hydrostatics { /* HydrostaticConfiguration, PoseUKFConfig.hpp:145-157 */
  double water_density;
  double water_density_limits;
  double water_density_tau;
  double atmospheric_pressure;
  double pressure_std;
} uwvk_hydrostatics;

typedef struct uwvk_pose_config { /* PoseUKFConfig, PoseUKFConfig.hpp:159-194 (visual-landmark config: passed per call) */
  uwvk_inertial_noise acceleration;
  uwvk_inertial_noise rotation_rate;
  uwvk_model_noise model_noise_parameters;
  uwvk_water_velocity water_velocity;
  uwvk_location location;
  uwvk_hydrostatics hydrostatics;
  double max_jerk[3];
  double max_effort[6];
  double dynamic_model_min_depth;
} uwvk_pose_config;

/* [EXT] uwv_dynamic_model::UWVParameters, the subset the hot path reads
 * (PoseUKF.cpp:159-171, VelocityUKF.cpp:60-74).  6x6 matrices row-major.
 * Forces/torques follow M*nu_dot + C(nu)*nu + D_l*nu + D_q*|nu|*nu + g(q) = tau. */
typedef struct uwvk_uwv_params {
  double inertia_matrix[36];
  double damping_matrices[2][36]; /* [0] linear, [1] quadratic */
  double weight;
  double buoyancy;
  double distance_body2centerofgravity[3];
  double distance_body2centerofbuoyancy[3];
} uwvk_uwv_params;

/* PoseUKF::PoseUKFParameter, PoseUKF.hpp:46-76 */
typedef struct uwvk_pose_parameter {
  double imu_in_body[3];
  double gyro_bias_offset[3];
  double gyro_bias_tau;
  double acc_bias_offset[3];
  double acc_bias_tau;
  double inertia_tau;
  double lin_damping_tau;
  double quad_damping_tau;
  double water_velocity_tau;
  double water_velocity_limits;
  double water_velocity_scale;
  double adcp_bias_tau;
  double atmospheric_pressure;
  double water_density_tau;
} uwvk_pose_parameter;

/* ---- library ------------------------------------------------------------ */
int uwvk_abi_version(void);
/* 1 when a gfx950 device is visible and the kernels' code object loads. */
int uwvk_device_available(int device);
const char* uwvk_status_string(uwvk_status s);
/* The HIP error (name, message, failing entry point) behind the calling host
 * thread's most recent UWVK_EDEVICE, "" if none (diagnostics). */
const char* uwvk_last_device_error(void);

/* device memory helpers for device-resident logs (bench / run_log).
 * uwvk_memcpy_h2d / _d2h are synchronous with all work on the device that owns
 * the device-side buffer (they make that device current, wait for every
 * stream on it, the handles' non-blocking ones included, then copy); work
 * queued on OTHER devices is not waited for.
 * uwvk_memcpy_*_on are ordered on one stream (a handle's uwvk_*_stream) and
 * return once the copy has completed. */
uwvk_status uwvk_device_malloc(int device, size_t bytes, void** out);
uwvk_status uwvk_device_free(void* p);
uwvk_status uwvk_memcpy_h2d(void* dst, const void* src, size_t bytes);
uwvk_status uwvk_memcpy_d2h(void* dst, const void* src, size_t bytes);
uwvk_status uwvk_memcpy_h2d_on(void* dst, const void* src, size_t bytes, void* stream);
uwvk_status uwvk_memcpy_d2h_on(void* dst, const void* src, size_t bytes, void* stream);

/* Synthetic-log noise (host only, no device work): out[j * count + k] is the
 * k-th standard normal variate of stream `stream` (< 256) of global instance
 * first_instance + j, a pure function of (seed, instance, stream, k):
 * Philox4x32-10 blocks, Box-Muller (csrc/uwvk_synth.cpp).  Instance-sharded
 * runs therefore draw bitwise the rows of the full batch. */
uwvk_status uwvk_synth_normal(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream, int64_t count,
                              double* out);
/* The variates [offset, offset + count) of the same per-(instance, stream)
 * sequences (uwvk_synth_normal is offset 0, group 0).  group 0: out[batch][count];
 * group g > 0 (count a multiple of g): record-major out[count / g][batch][g],
 * the logs' [epoch][instance][component] layout. */
uwvk_status uwvk_synth_normal_at(uint64_t seed, int64_t first_instance, int64_t batch, uint32_t stream,
                                 int64_t offset, int64_t count, int32_t group, double* out);

/* ======================================================================== */
/* PoseUKF                                                                   */
/* ======================================================================== */
typedef struct uwvk_pose uwvk_pose;

/* dof = 53 (PoseState) or 26 (kinematic subset).  Allocates device state. */
uwvk_status uwvk_pose_create(int64_t batch, int dof, int device, uwvk_pose** out);
void uwvk_pose_destroy(uwvk_pose* h);
int64_t uwvk_pose_batch(const uwvk_pose* h);
int uwvk_pose_dof(const uwvk_pose* h);
/* hipStream_t of the handle (as void*), for event timing by the caller. */
void* uwvk_pose_stream(const uwvk_pose* h);
uwvk_status uwvk_pose_synchronize(uwvk_pose* h);

/* Both init calls are the reference's constructors: every instance becomes a
 * NEW filter, so the process noise is zero until set again and the stored
 * rotation rate is zero (PoseUKF.cpp:380).
 *
 * PoseUKF::PoseUKF(pos, pos_cov, rot, rot_cov, cfg, uwv, imu_in_body)
 * (PoseUKF.hpp:100-103, PoseUKF.cpp:288-372).  Per instance: pos[3],
 * pos_cov[9], rot[4] (w,x,y,z), rot_cov[9].  imu_in_body = {tx,ty,tz,qw,qx,qy,qz}
 * (NULL = identity), shared by the batch. */
uwvk_status uwvk_pose_init_from_config(uwvk_pose* h, const double* pos, const double* pos_cov,
                                       const double* rot, const double* rot_cov,
                                       const uwvk_pose_config* cfg, const uwvk_uwv_params* uwv,
                                       const double imu_in_body[7]);
/* PoseUKF::PoseUKF(state, cov, location, uwv, param) (PoseUKF.hpp:113-115,
 * PoseUKF.cpp:374-391).  x: batch*store, P: batch*dof*dof. */
uwvk_status uwvk_pose_init_from_state(uwvk_pose* h, const double* x, const double* P,
                                      const uwvk_location* location, const uwvk_uwv_params* uwv,
                                      const uwvk_pose_parameter* param);
/* setProcessNoiseFromConfig (PoseUKF.hpp:126-127, PoseUKF.cpp:393-439);
 * q_imu_in_body (w,x,y,z) may be NULL (identity). */
uwvk_status uwvk_pose_set_process_noise_from_config(uwvk_pose* h, const uwvk_pose_config* cfg,
                                                    double imu_delta_t, const double q_imu_in_body[4]);
/* setProcessNoiseCovariance [EXT base]: dof*dof, shared by the batch. */
uwvk_status uwvk_pose_set_process_noise(uwvk_pose* h, const double* Q);

/* integrateMeasurement(RotationRate) (PoseUKF.cpp:492-496): stores omega.
 * w: batch*3, cov: batch*9 (checked for NaN only, may be NULL). */
uwvk_status uwvk_pose_set_rotation_rate(uwvk_pose* h, const double* w, const double* cov);
/* predictionStep(dt) -> predictionStepImpl (PoseUKF.cpp:446-474). */
uwvk_status uwvk_pose_predict(uwvk_pose* h, double dt);

/* Measurement updates.  mu: batch*m, cov: batch*m*m (NULL = shared_cov),
 * shared_cov: m*m used when cov == NULL.  mask: batch bytes, 0 = skip this
 * instance (NULL = all).  accepted (out, nullable): batch bytes, 1 when the
 * innovation gate passed and the state was updated. */
/* integrateMeasurement(Acceleration) (PoseUKF.cpp:484-490), m = 3 */
uwvk_status uwvk_pose_update_acceleration(uwvk_pose* h, const double* mu, const double* cov,
                                          const double* shared_cov, const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(Velocity) (PoseUKF.cpp:476-482), m = 3, DVL in IMU frame */
uwvk_status uwvk_pose_update_velocity(uwvk_pose* h, const double* mu, const double* cov,
                                      const double* shared_cov, const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(Pressure, sensor_in_imu) (PoseUKF.cpp:559-565), m = 1 */
uwvk_status uwvk_pose_update_pressure(uwvk_pose* h, const double* mu, const double* cov,
                                      const double* shared_cov, const double sensor_in_imu[3],
                                      const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(WaterVelocityMeasurement, cell_weighting)
 * (PoseUKF.cpp:604-611), m = 2, d2p95 gate.  cell_weighting: batch doubles. */
uwvk_status uwvk_pose_update_water_velocity(uwvk_pose* h, const double* mu, const double* cov,
                                            const double* shared_cov, const double* cell_weighting,
                                            const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(BodyEffortsMeasurement, only_affect_velocity)
 * (PoseUKF.cpp:581-602), m = 6. */
uwvk_status uwvk_pose_update_efforts(uwvk_pose* h, const double* mu, const double* cov,
                                     const double* shared_cov, int only_affect_velocity,
                                     const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(XY_Position) (PoseUKF.cpp:506-512), m = 2 */
uwvk_status uwvk_pose_update_xy(uwvk_pose* h, const double* mu, const double* cov,
                                const double* shared_cov, const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(Z_Position) (PoseUKF.cpp:498-504), m = 1 */
uwvk_status uwvk_pose_update_z(uwvk_pose* h, const double* mu, const double* cov,
                               const double* shared_cov, const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(GeographicPosition, gps_in_body) (PoseUKF.cpp:567-579),
 * m = 2 (lat, lon in rad), d2p95 gate. */
uwvk_status uwvk_pose_update_geographic(uwvk_pose* h, const double* mu, const double* cov,
                                        const double* shared_cov, const double gps_in_body[3],
                                        const uint8_t* mask, uint8_t* accepted);
/* integrateDelayedPositionMeasurement (PoseUKF.cpp:514-527): delayed_xy batch*2 */
uwvk_status uwvk_pose_update_delayed_xy(uwvk_pose* h, const double* mu, const double* cov,
                                        const double* shared_cov, const double* delayed_xy,
                                        const uint8_t* mask, uint8_t* accepted);
/* integrateMeasurement(vector<VisualFeatureMeasurement>, feature_positions, marker_pose,
 * cov_marker_pose, camera_config, camera_in_IMU) (PoseUKF.cpp:613-654): the state is
 * augmented with the marker pose (PoseStateWithMarker, :221-229), one S2-valued
 * update per feature (measurementVisualLandmark, :231-244; accept any Mahalanobis
 * distance), then reset to the leading block.  Per instance n_features features:
 *   features           [batch][nf][2] undistorted image coordinates (px)
 *   feature_cov        [batch][nf][4] (feature_cov_per_instance) or [nf][4], px^2
 *   feature_positions  [nf][3] in the marker frame (shared)
 *   marker_pose        [batch][7] (marker_pose_per_instance) or [7]: t(3), q(w,x,y,z)
 *   cov_marker_pose    [36] (shared), camera {fx, fy, cx, cy}, camera_in_imu t(3) q(4)
 * A NaN feature fails the whole call with UWVK_ENAN and changes nothing (the
 * reference throws before its ukf.reset). */
uwvk_status uwvk_pose_update_visual_landmark(uwvk_pose* h, int32_t n_features, const double* features,
                                             const double* feature_cov, int feature_cov_per_instance,
                                             const double* feature_positions, const double* marker_pose,
                                             int marker_pose_per_instance, const double cov_marker_pose[36],
                                             const double camera[4], const double camera_in_imu[7],
                                             const uint8_t* mask);
/* resetFilterWithExternalPose (PoseUKF.cpp:685-691): pose batch*7 {t, q(w,x,y,z)} */
uwvk_status uwvk_pose_reset_with_external_pose(uwvk_pose* h, const double* pose);

/* getCurrentState / ukf->mu(), ukf->sigma() [EXT]: x batch*store, P batch*dof*dof (nullable) */
uwvk_status uwvk_pose_get_state(uwvk_pose* h, double* x, double* P);
/* getRotationRate (PoseUKF.cpp:693-699): batch*3 */
uwvk_status uwvk_pose_get_rotation_rate(uwvk_pose* h, double* out);
/* per-instance status words (UWVK_ST_*), batch uint32; clear = 1 resets them */
uwvk_status uwvk_pose_get_status(uwvk_pose* h, uint32_t* status, int clear);

/* ---- device-resident measurement log (persistent multi-epoch path) ----- */
/* Event flags per epoch (what the out-of-repo driver would call, §3 of SURVEY):
 * every epoch: RotationRate -> predictionStep(dt) -> Acceleration update;
 * then, when flagged: Velocity (DVL), Pressure, ADCP cells, BodyEfforts. */
#define UWVK_EV_ACC 0x1u
#define UWVK_EV_DVL 0x2u
#define UWVK_EV_PRESSURE 0x4u
#define UWVK_EV_ADCP 0x8u
#define UWVK_EV_EFFORTS 0x10u
#define UWVK_EV_EFFORTS_VELOCITY_ONLY 0x20u

typedef struct uwvk_pose_log {
  /* ALL pointers are DEVICE pointers (uwvk_device_malloc) unless noted. */
  int64_t epochs;
  double dt;                 /* predict step, seconds (host value) */
  const uint32_t* flags;     /* [epochs] UWVK_EV_* */
  const double* gyro;        /* [epochs][batch][3] */
  const double* acc;         /* [epochs][batch][3] */
  double acc_cov[9];         /* host value, shared */
  const int32_t* dvl_index;  /* [epochs] row into dvl (valid when EV_DVL) */
  const double* dvl;         /* [n_dvl][batch][3] */
  double dvl_cov[9];
  const int32_t* pressure_index;
  const double* pressure;    /* [n_pressure][batch] */
  double pressure_cov;
  double pressure_sensor_in_imu[3];
  const int32_t* adcp_index;
  const double* adcp;        /* [n_adcp][cells][batch][2] */
  int32_t adcp_cells;
  double adcp_cell_weighting[8]; /* host values, per cell */
  double adcp_cov[4];
  const int32_t* efforts_index;
  const double* efforts;     /* [n_efforts][batch][6] */
  double efforts_cov[36];
  /* HOST copy of flags (nullable): lets run_log plan its launches without a
   * device->host read of `flags`.  It must equal `flags`: run_log also picks
   * each launch's kernel from it (a launch whose host flags hold no pressure or
   * ADCP event runs a kernel without those updates). */
  const uint32_t* host_flags;
} uwvk_pose_log;

/* Runs epochs [first, first+count) of the log.  Default (PSP) path: one launch
 * per run of epochs, each instance's Sigma resident in LDS across the run;
 * BodyEfforts epochs run through the literal kernel (one launch per epoch).
 * UWVK_OPT_DENSE_SIGMA = 1: one literal fused launch per epoch.
 * accept_counts (device, nullable): [batch][4] uint32 accepted DVL/pressure/ADCP/efforts. */
uwvk_status uwvk_pose_run_log(uwvk_pose* h, const uwvk_pose_log* log, int64_t first, int64_t count,
                              uint32_t* accept_counts);

/* Ensemble statistics over the batch (for Monte-Carlo runs):
 * out[0..store)        = sum_i x_i (orientation quaternion summed componentwise)
 * out[store..2*store)  = sum_i x_i^2
 * out[2*store..3*store)= sum_i (x_i - truth)^2 (orientation: rotation-vector error, 3 entries used)
 * out[3*store]         = sum_i NEES_i over (position, orientation, velocity) (9 DOF),
 *                        over the instances whose 9x9 covariance block is positive definite
 * out[3*store+1]       = number of instances left out of that NEES sum (not positive definite / NaN)
 * truth: host store-vector (nullable -> zeros).  out: host doubles, 3*store+2. */
uwvk_status uwvk_pose_ensemble_stats(uwvk_pose* h, const double* truth, double* out);

/* Multi-GPU ensembles: one process (or thread) per GPU owns a
 * contiguous instance range; the only collective is this statistics sum over
 * RCCL.  `comm` is an RCCL communicator (ncclComm_t) as void*, from
 * uwvk_comm_init or the caller's own RCCL setup; NULL = this handle only (same
 * as uwvk_pose_ensemble_stats).  The sum runs on the handle's stream. */
uwvk_status uwvk_pose_ensemble_allreduce(uwvk_pose* h, const double* truth, double* out, void* comm);
/* RCCL communicator helpers (no RCCL headers needed by the caller): rank 0
 * calls uwvk_comm_unique_id and ships the uwvk_comm_unique_id_bytes() bytes to
 * the other ranks out of band; every rank then calls uwvk_comm_init. */
int uwvk_comm_unique_id_bytes(void);
uwvk_status uwvk_comm_unique_id(char* id);
uwvk_status uwvk_comm_init(int nranks, const char* id, int rank, int device, void** comm);
void uwvk_comm_destroy(void* comm);
uwvk_status uwvk_comm_allreduce_sum_device(void* comm, double* d_buf, int64_t n, void* stream);

/* Engine options (not part of the reference surface).
 * UWVK_OPT_LITERAL_APPLY_DELTA: 0 (default) applies ukfom's apply_delta through
 *   its exact nav-frame identity mu <- mu [+] d, Sigma <- T Sigma T^T
 *   (T rotates the orientation block by exp(d)); 1 runs the literal re-spread
 *   (Cholesky + sigma points + covariance GEMM).  Results agree to rounding. */
#define UWVK_OPT_LITERAL_APPLY_DELTA 1
/* UWVK_OPT_DENSE_SIGMA: 0 (default) evaluates ukfom's unscented transform in
 *   partitioned form (PSP): sigma points only along the Cholesky columns a model
 *   is non-affine in, the affine remainder in closed form (A Sigma A^T, H Sigma
 *   H^T); equal to the literal spread up to rounding.
 *   1 propagates all 2n+1 sigma points (MFMA covariance GEMM).  Setting
 *   UWVK_OPT_LITERAL_APPLY_DELTA also selects the literal kernels. */
#define UWVK_OPT_DENSE_SIGMA 2
/* UWVK_OPT_TAIL_SLOTS: last-generation spreading of the PSP run_log launch.
 *   When batch / 8 instances per XCD leave a partial last generation of the
 *   XCD's resident blocks, those tail instances run as a few epoch chunks
 *   handed from block to block (Sigma~ and its time scale unfolded, so the
 *   result is bitwise the one-block run), spread over the slots that would
 *   idle.  0 (default): plan for the occupancy the runtime reports; > 0: plan
 *   for that many resident blocks per XCD (tests); < 0: off.  Needs
 *   batch % 8 == 0. */
#define UWVK_OPT_TAIL_SLOTS 3
/* UWVK_OPT_TAIL_CHUNKS: 0 (default) the planner picks the chunk count; 2..8
 *   forces that many chunks per tail instance whenever the launch allows it
 *   (chunks x slots <= batch / 8, chunks <= epochs), for tests.  Spreading of
 *   any kind runs only where uwvk_xcd_round_robin(device) is 1. */
#define UWVK_OPT_TAIL_CHUNKS 4
/* UWVK_OPT_SO3_RIGHT: the side of the SO3 [+] / [-] [EXT MTK], SURVEY 8(c)
 *   item 5, the largest unpinned semantic.  1 (default since r05): body frame
 *   (right), q [+] d = q exp(d), MTK's published SO3::boxplus, through which the
 *   reference's orientation.boxplus runs (mtkwrap<MTK::SO3<double>>,
 *   PoseState.hpp:15; PoseUKF.cpp:32), in every orientation [+] / [-]: sigma
 *   points, processModel's orientation step, manifold mean, apply_delta, the
 *   visual update's filter and marker orientations and the ensemble
 *   statistics' orientation error (log(t^-1 q)).  0: nav frame (left),
 *   q [+] d = exp(d) q, an option (the convention SURVEY 8(c) had inferred
 *   from PoseUKF.cpp:31 / :451).  Every engine path runs either side (the PSP
 *   kernels are instantiated per side, SR); the oracle's or_set_so3_right is
 *   the same switch. */
#define UWVK_OPT_SO3_RIGHT 5
/* UWVK_OPT_PERSIST: scheduling of the PSP run_log launch.  1 (default since
 *   r06): persistent workgroups, as many as are resident, run their own unit
 *   first and then take work units (whole instances, then the epoch chunks of
 *   the last chunks x resident-slots instances) from a ticket counter: faster
 *   XCDs and CUs take more units, no workgroup dispatch between units, and a
 *   chunk's hand-off waits only on a unit a running workgroup holds (no
 *   placement or dispatch-order assumption).  0: one workgroup per instance
 *   (plus UWVK_OPT_TAIL_SLOTS spreading, which relies on the round-robin XCD
 *   placement of uwvk_xcd_round_robin and in-order dispatch; without the
 *   placement the launch falls back to the persistent form).  Results are
 *   bitwise the same.  (MI355X, C3 batch 65,536, four interleaved rounds: tie,
 *   200.6 against 200.9 M steps/s over 20 epochs, 219.2 against 219.1 M over
 *   200) */
#define UWVK_OPT_PERSIST 6
/* UWVK_OPT_LDS_PAD (diagnostic, r05): bytes of dynamic LDS requested per PSP
 *   epoch workgroup on top of its static 12.8 KB, unused by the kernel: it only
 *   lowers the resident workgroups per CU (12 -> 9 / 6 / 4 ...), to measure the
 *   epoch kernel's rate against occupancy.  0 default,
 *   at most 160 KiB minus the static 12.8 KB (else UWVK_EINVAL); a non-zero pad
 *   turns tail spreading off (the planners assume the unpadded occupancy). */
#define UWVK_OPT_LDS_PAD 7
/* UWVK_OPT_WAIT_BOUND (tests, r06): sleeps of ~1.7 us a tail chunk waits for
 *   its predecessor's hand-off before it gives up (UWVK_ST_SCHEDULE, and
 *   the next synchronize / run_log returns UWVK_ESCHEDULE).  < 0 (default): the planner's
 *   bound (~2 s plus 64-128 sleeps per epoch); 0 forces every hand-off of a
 *   spread launch to time out. */
#define UWVK_OPT_WAIT_BOUND 8
/* UWVK_OPT_PARAM_BLOCK (r06): 1 (default) runs run_log's PSP epoch launches of
 *   a 53-DOF handle on the parameter-decoupled kernel while the 27 model-
 *   parameter DOFs (inertia, linear / quadratic damping) are uncoupled: their
 *   rows of Sigma zero off the diagonal (as PoseUKF.cpp:333-335 make P0; checked
 *   on the host at init) and Q diagonal there (PoseUKF.cpp:417-422).  That
 *   kernel keeps the other 26 DOFs in the 26-DOF layout with the 53-DOF
 *   sigma-point weights and evolves each parameter alone; the results are the
 *   53-DOF kernel's.  The full BodyEfforts update (and
 *   any literal-kernel step) couples the block: the handle then runs the
 *   general kernel until it is re-initialised.  0: always the general kernel.
 *   uwvk_pose_param_block says which the next launch runs. */
#define UWVK_OPT_PARAM_BLOCK 9
/* UWVK_OPT_PAIR (r06, default 1): run_log runs two instances per wave (each on
 *   32 lanes; uwvk_psp_pair.hip) for 53-DOF handles while the parameter-
 *   decoupled kernel applies and for 26-DOF handles, on the persistent
 *   scheduler, an even batch and the lane-resident Q.  The pressure update's
 *   39 sigma points do not fit a half-wave: a launch is split around its
 *   pressure epochs (those run one instance per wave) when the runs between
 *   them are at least 48 epochs long.  The results agree with the one-instance
 *   kernel to rounding (the rank-M update sums in another order), gate
 *   decisions bitwise.  0: one instance per wave. */
#define UWVK_OPT_PAIR 10
uwvk_status uwvk_pose_set_option(uwvk_pose* h, int option, int value);
/* Host-only query (no device work): the chunks per tail instance the
 * UWVK_OPT_TAIL_SLOTS planner picks for one XCD's instances over its resident
 * blocks in an epochs-long launch; 1 = no spreading. */
int uwvk_pose_tail_chunks(int64_t instances_per_xcd, int64_t slots_per_xcd, int64_t epochs);
/* Resident PSP epoch-kernel blocks per XCD the runtime reports for this dof on
 * device (occupancy x CUs / 8; what UWVK_OPT_TAIL_SLOTS = 0 plans for), 0 if
 * unknown. */
int64_t uwvk_pose_resident_slots(int dof, int device);
/* Host-only query: the process-noise shape the PSP epoch kernel is
 * instantiated for on this handle's current Q: 1 = the lane-resident simple
 * shape (no coupling of the rewritten rows < 9, band <= 2; the default
 * configuration's), 2 = general (psp_predict QM). */
int uwvk_pose_epoch_qshape(const uwvk_pose* h);
/* Host-only query: 1 when the next run_log PSP launch runs the
 * parameter-decoupled kernel (UWVK_OPT_PARAM_BLOCK), else 0. */
int uwvk_pose_param_block(uwvk_pose* h);
/* Host-only query: 1 when run_log's launches (their epochs without a pressure
 * update) run the two-instances-per-wave form (UWVK_OPT_PAIR). */
int uwvk_pose_pair_active(uwvk_pose* h);
/* 1 when a probe grid on device showed round-robin workgroup placement over 8
 * XCCs (block b on the XCC of block b % 8, read from the hardware XCC_ID
 * register): the placement tail spreading's hand-off order relies on.  0 on a
 * partitioned device (or any other placement): spreading is then off.  The
 * probe runs once per device and process. */
int uwvk_xcd_round_robin(int device);

/* Kernel-timing helper: HIP events recorded on the handle's stream. */
uwvk_status uwvk_pose_timer_start(uwvk_pose* h);
uwvk_status uwvk_pose_timer_stop(uwvk_pose* h, float* elapsed_ms);
/* Split form of uwvk_pose_timer_stop: _mark records the stop event without
 * waiting, so work queued after it (the ensemble statistics) follows the
 * timed launches with no host round trip; _elapsed waits for that event and
 * returns the time since uwvk_pose_timer_start. */
uwvk_status uwvk_pose_timer_mark(uwvk_pose* h);
uwvk_status uwvk_pose_timer_elapsed(uwvk_pose* h, float* elapsed_ms);

/* ---- recorded-mission ingestion (host only, no device needed) ---------- */
/* The reference is driven by its caller's stream aligner (Rock orogen task,
 * outside the repository): RotationRate + predictionStep +
 * Acceleration per IMU sample (PoseUKF.cpp:446-496), the lower-rate sensors
 * integrated as their samples arrive (PoseUKF.cpp:476-611).  This turns the
 * per-sensor sample stamps of a recording into the epoch-indexed flags and
 * row indices of uwvk_pose_log (the payload arrays keep sample order).
 * Semantics: DESIGN.md §11 (fixed-step replay, lag < dt, per-sensor queue). */
typedef struct uwvk_stream_times { /* seconds, ascending per sensor; NULL when n = 0 */
  const double* imu;      int64_t n_imu;  /* one epoch per IMU sample */
  const double* dvl;      int64_t n_dvl;
  const double* pressure; int64_t n_pressure;
  const double* adcp;     int64_t n_adcp;  /* one sample = all cells of one ADCP ping */
  const double* efforts;  int64_t n_efforts;
  const uint8_t* efforts_velocity_only;    /* [n_efforts], nullable: only_affect_velocity */
} uwvk_stream_times;

typedef struct uwvk_schedule {
  /* caller-allocated HOST arrays of n_imu entries (index arrays may be NULL
   * when that sensor has no samples) */
  uint32_t* flags;         /* UWVK_EV_* per epoch */
  int32_t* dvl_index;      /* row of the sample integrated at that epoch, -1 = none */
  int32_t* pressure_index;
  int32_t* adcp_index;
  int32_t* efforts_index;
  /* outputs */
  double dt;               /* mean IMU interval (0 for a single sample) */
  int64_t epochs;
  int64_t kept[4];         /* DVL, pressure, ADCP, efforts samples placed */
  int64_t dropped[4];      /* before the first IMU stamp / queued past the last epoch */
} uwvk_schedule;

/* dt_tolerance: allowed |interval - dt| / dt of the IMU stream (non-uniform ->
 * UWVK_EINVAL); time_epsilon: stamp slack in seconds. */
uwvk_status uwvk_schedule_streams(const uwvk_stream_times* in, double dt_tolerance, double time_epsilon,
                                  uwvk_schedule* out);

/* ADCP cell weighting for integrateMeasurement(WaterVelocityMeasurement,
 * cell_weighting) (PoseUKF.cpp:133-151,604-611) from cell_size and
 * first_cell_blank (PoseUKFConfig.hpp:34-38): 0 at the nearest cell centre,
 * 1 at the farthest, linear in range.  valid[i] (nullable) = correlation[i] >=
 * minimum_correlation (PoseUKFConfig.hpp:40-41), all 1 when correlation is NULL. */
uwvk_status uwvk_adcp_cell_weighting(const uwvk_water_velocity* wv, int32_t cells, const double* correlation,
                                     double* weighting, uint8_t* valid);

/* ======================================================================== */
/* VelocityUKF (src/VelocityUKF.hpp:231-266)                                 */
/* ======================================================================== */
#define UWVK_VEL_DOF 4
typedef struct uwvk_vel uwvk_vel;

uwvk_status uwvk_vel_create(int64_t batch, int device, uwvk_vel** out);
void uwvk_vel_destroy(uwvk_vel* h);
void* uwvk_vel_stream(const uwvk_vel* h);
/* VelocityUKF(state, cov) (VelocityUKF.cpp:49-56): x batch*4 {v, z}, P batch*16 */
uwvk_status uwvk_vel_init(uwvk_vel* h, const double* x, const double* P);
/* setupMotionModel (VelocityUKF.cpp:58-77) */
uwvk_status uwvk_vel_setup_motion_model(uwvk_vel* h, const uwvk_uwv_params* uwv);
/* GyroMeasurement (VelocityUKF.cpp:87-98): batch*3 */
uwvk_status uwvk_vel_set_gyro(uwvk_vel* h, const double* w, const double* cov);
/* BodyEffortsMeasurement (VelocityUKF.cpp:100-104): batch*6 */
uwvk_status uwvk_vel_set_efforts(uwvk_vel* h, const double* tau, const double* cov);
/* predictionStep -> predictionStepImpl (VelocityUKF.cpp:114-130) */
uwvk_status uwvk_vel_predict(uwvk_vel* h, double dt);
/* DVLMeasurement (VelocityUKF.cpp:79-85), m = 3 */
uwvk_status uwvk_vel_update_dvl(uwvk_vel* h, const double* mu, const double* cov, const double* shared_cov,
                                const uint8_t* mask);
/* PressureMeasurement (z) (VelocityUKF.cpp:106-112), m = 1 */
uwvk_status uwvk_vel_update_pressure(uwvk_vel* h, const double* mu, const double* cov, const double* shared_cov,
                                     const uint8_t* mask);
uwvk_status uwvk_vel_get_state(uwvk_vel* h, double* x, double* P);
/* motion-model side state: batch*13 {p(3), q(4: w,x,y,z), v(3), w(3)} */
uwvk_status uwvk_vel_get_model_state(uwvk_vel* h, double* out);

typedef struct uwvk_vel_log {
  int64_t epochs;
  double dt;
  const uint32_t* flags;    /* UWVK_EV_DVL / UWVK_EV_PRESSURE */
  const double* gyro;       /* [epochs][batch][3] */
  const double* efforts;    /* [epochs][batch][6] */
  const int32_t* dvl_index;
  const double* dvl;        /* [n_dvl][batch][3] */
  double dvl_cov[9];
  const int32_t* pressure_index;
  const double* pressure;   /* [n_pressure][batch] (z position) */
  double pressure_cov;
} uwvk_vel_log;
/* Runs epochs [first, first + count): one launch per 4096 epochs, state in
 * registers across the launch.  Asynchronous on the handle's stream (the
 * getters and uwvk_vel_synchronize wait). */
uwvk_status uwvk_vel_run_log(uwvk_vel* h, const uwvk_vel_log* log, int64_t first, int64_t count);
/* UWVK_VEL_OPT_LANE_GROUPS: -1 (default) auto by batch size, 0 one filter per
 * lane (9 sigma points in one lane's registers), 1 one filter per 16-lane DPP
 * row (one sigma point per lane; fills the chip at small batches, e.g. C2's 4096);
 * 2 (diagnostic, r05) the 16-lane kernel with each filter duplicated in a second
 * row that stores nothing: twice the waves, the same per-wave work. */
#define UWVK_VEL_OPT_LANE_GROUPS 1
uwvk_status uwvk_vel_set_option(uwvk_vel* h, int option, int value);
/* setProcessNoiseCovariance [EXT pose_estimation base]: 4x4, shared by the
 * batch (default: VelocityUKF.cpp:54-55, velocity diag 1e-4); predict adds dt * Q. */
uwvk_status uwvk_vel_set_process_noise(uwvk_vel* h, const double Q[16]);
uwvk_status uwvk_vel_synchronize(uwvk_vel* h);
/* HIP events on the handle's stream around queued work (bench timing) */
uwvk_status uwvk_vel_timer_start(uwvk_vel* h);
uwvk_status uwvk_vel_timer_stop(uwvk_vel* h, float* elapsed_ms);

/* ======================================================================== */
/* BottomUKF (src/BottomUKF.hpp:26-53, BottomUKF.cpp:1-71)                  */
/* State {distance, normal}: 3 DOF, stored as 4 scalars {d, nx, ny, nz}      */
/* (the normal is an MTK::S2 unit vector).             */
/* ======================================================================== */
#define UWVK_BOTTOM_DOF 3
typedef struct uwvk_bottom uwvk_bottom;
uwvk_status uwvk_bottom_create(int64_t batch, int device, uwvk_bottom** out);
void uwvk_bottom_destroy(uwvk_bottom* h);
void* uwvk_bottom_stream(const uwvk_bottom* h);
/* BottomUKF(initial_state, state_cov) (BottomUKF.cpp:40-46): x batch*4 (normal
 * normalised here, as MTK::S2 does), P batch*9; process noise = identity. */
uwvk_status uwvk_bottom_init(uwvk_bottom* h, const double* x, const double* P);
/* setProcessNoiseCovariance [EXT base]: 3x3, shared by the batch */
uwvk_status uwvk_bottom_set_process_noise(uwvk_bottom* h, const double Q[9]);
/* setVelocity (BottomUKF.cpp:69-72): batch*3 */
uwvk_status uwvk_bottom_set_velocity(uwvk_bottom* h, const double* velocity);
/* predictionStep -> predictionStepImpl (BottomUKF.cpp:48-54) */
uwvk_status uwvk_bottom_predict(uwvk_bottom* h, double dt);
/* integrateMeasurement(RangeMeasurement, unit_direction, origin) (BottomUKF.cpp:56-61):
 * mu batch, cov batch (NULL = shared_cov); beam direction / origin shared. */
uwvk_status uwvk_bottom_update_range(uwvk_bottom* h, const double* mu, const double* cov, double shared_cov,
                                     const double unit_direction[3], const double origin[3], const uint8_t* mask);
/* integrateMeasurement(NormalType, cov) (BottomUKF.cpp:63-67): mu batch*3 (normalised),
 * cov batch*4 (NULL = shared_cov[4]) */
uwvk_status uwvk_bottom_update_normal(uwvk_bottom* h, const double* mu, const double* cov, const double* shared_cov,
                                      const uint8_t* mask);
uwvk_status uwvk_bottom_get_state(uwvk_bottom* h, double* x, double* P);
uwvk_status uwvk_bottom_get_status(uwvk_bottom* h, uint32_t* status, int clear);

/* ======================================================================== */
/* IndirectPoseUKF (src/IndirectPoseUKF.hpp:28-86, IndirectPoseUKF.cpp:1-147) */
/* State {position_error, orientation_error}: 6 DOF, stored t(3) q(w,x,y,z).  */
/* ======================================================================== */
#define UWVK_IPOSE_DOF 6
typedef struct uwvk_ipose uwvk_ipose;
uwvk_status uwvk_ipose_create(int64_t batch, int device, uwvk_ipose** out);
void uwvk_ipose_destroy(uwvk_ipose* h);
void* uwvk_ipose_stream(const uwvk_ipose* h);
/* UWVK_OPT_SO3_RIGHT only: the side of the orientation_error [+] / [-] (an
 * MTK::SO3, IndirectPoseUKF.hpp:21), 1 (default) body frame q exp(d), 0 nav
 * frame exp(d) q, as uwvk_pose_set_option; the oracle's or_set_so3_right. */
uwvk_status uwvk_ipose_set_option(uwvk_ipose* h, int option, int value);
/* IndirectPoseUKF(position_error_std, orientation_error_std, orientation_error_tau,
 * initial_position_error, initial_position_error_std) (IndirectPoseUKF.cpp:53-78):
 * stds shared; initial_position_error batch*3 (NULL = zero); initial std NULL = ones. */
uwvk_status uwvk_ipose_init(uwvk_ipose* h, const double position_error_std[3], const double orientation_error_std[3],
                            double orientation_error_tau, const double* initial_position_error,
                            const double initial_position_error_std[3]);
/* setProcessNoiseCovariance [EXT pose_estimation base]: 6x6, shared by the
 * batch (uwvk_ipose_init sets diag(position_error_std^2, orientation_error_std^2),
 * IndirectPoseUKF.cpp:72-77); predict shapes it as predictionStepImpl (:80-92). */
uwvk_status uwvk_ipose_set_process_noise(uwvk_ipose* h, const double Q[36]);
/* updatePoseReference (IndirectPoseUKF.cpp:144-147): batch*7 body in world, t(3) q(4) */
uwvk_status uwvk_ipose_set_pose_reference(uwvk_ipose* h, const double* pose);
/* predictionStep -> predictionStepImpl (IndirectPoseUKF.cpp:80-92) */
uwvk_status uwvk_ipose_predict(uwvk_ipose* h, double dt);
/* integrateMeasurement(marker_features, feature_positions, marker_pose, cov_marker_pose,
 * camera_config, camera_in_body) (IndirectPoseUKF.cpp:94-135); arrays as for
 * uwvk_pose_update_visual_landmark. */
uwvk_status uwvk_ipose_update_visual(uwvk_ipose* h, int32_t n_features, const double* features,
                                     const double* feature_cov, int feature_cov_per_instance,
                                     const double* feature_positions, const double* marker_pose,
                                     int marker_pose_per_instance, const double cov_marker_pose[36],
                                     const double camera[4], const double camera_in_body[7], const uint8_t* mask);
/* getCorrectedPose (IndirectPoseUKF.cpp:137-142): pose_ref * pose_error, batch*7 */
uwvk_status uwvk_ipose_get_corrected_pose(uwvk_ipose* h, double* out);
uwvk_status uwvk_ipose_get_state(uwvk_ipose* h, double* x, double* P);
uwvk_status uwvk_ipose_get_status(uwvk_ipose* h, uint32_t* status, int clear);

#ifdef __cplusplus
}
#endif
#endif /* UWVK_H_ */
