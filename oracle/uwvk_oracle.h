/*
 * uwvk_oracle.h — CPU fp64 restatement of the PoseUKF / VelocityUKF hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library.  The product path
 * (libuwvk.so) never links or calls it.
 *
 * PARITY STATUS: UNPINNED against the reference binary.  The reference
 * (tomcreutz/slam-uwv_kalman_filters) cannot be built here: its UKF arithmetic
 * lives in ukfom/MTK, pose_estimation and uwv_dynamic_model, none of which are
 * in /root/reference or in this image, and it ships zero tests or golden
 * vectors.  This oracle restates the reference's own
 * files line by line (citations inline) and the [EXT] library semantics from
 * their published designs, frozen as the written spec in DESIGN.md §3.  It is
 * cross-checked by an independently written numpy twin (oracle/numpy_twin.py)
 * and by closed-form known-answer tests (tests/test_oracle_kat.py).
 */
#ifndef UWVK_ORACLE_H_
#define UWVK_ORACLE_H_
#include <stdint.h>
#include "../include/uwvk.h"

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAXN 53
#define OR_MAXS 54

/* state layout descriptor (PoseState.hpp:29-45; kinematic subset without the
 * three 3x3 model-parameter blocks) */
typedef struct or_layout {
  int dof, store, has_params, has_quat;
  /* storage offsets (-1 = absent) */
  int s_pos, s_quat, s_vel, s_acc, s_bg, s_ba, s_grav, s_inertia, s_lin, s_quad, s_wv, s_wvb, s_badcp, s_rho;
  /* tangent offsets */
  int d_pos, d_ori, d_vel, d_acc, d_bg, d_ba, d_grav, d_inertia, d_lin, d_quad, d_wv, d_wvb, d_badcp, d_rho;
} or_layout;

void or_layout_init(or_layout* L, int dof);

/* One PoseUKF instance (members of PoseUKF.hpp:195-205 + the base filter). */
typedef struct or_pose {
  or_layout L;
  double mu[OR_MAXS];
  double sigma[OR_MAXN * OR_MAXN];
  double Q[OR_MAXN * OR_MAXN]; /* process_noise_cov */
  double rotation_rate[3];
  uwvk_pose_parameter param;
  double inertia_offset[9], lin_damping_offset[9], quad_damping_offset[9], water_density_offset;
  uwvk_location location;
  uwvk_uwv_params uwv;       /* dynamic_model parameters (mutated by the efforts update, PoseUKF.cpp:173) */
  int last_mean_iterations;  /* diagnostics: manifold-mean iterations of the last predict */
} or_pose;

/* ---- math primitives exposed for the known-answer tests ---------------- */
void or_quat_mul(const double a[4], const double b[4], double out[4]);
void or_quat_rotate(const double q[4], const double v[3], double out[3]);
void or_quat_rotate_inv(const double q[4], const double v[3], double out[3]);
void or_quat_to_matrix(const double q[4], double R[9]);
void or_so3_exp(const double v[3], double out[4]);
void or_so3_log(const double q[4], double out[3]);
int or_cholesky(int n, const double* A, double* L); /* 0 ok, -1 not PD */
void or_nav_to_world(const uwvk_location* loc, double x, double y, double* lat, double* lon);
void or_world_to_nav(const uwvk_location* loc, double lat, double lon, double* x, double* y);
double or_wgs84_gravity(double latitude, double altitude);
void or_calc_efforts(const uwvk_uwv_params* p, const double acc6[6], const double vel6[6], const double q[4],
                     double tau[6]);
void or_boxplus(const or_layout* L, const double* x, const double* delta, double scale, double* out);
void or_boxminus(const or_layout* L, const double* a, const double* b, double* out);
/* SO3 [+] side, process-wide: 1 = body-frame/right, q exp(d)
 * (default since r05: MTK's SO3::boxplus, through which PoseUKF.cpp:32 runs),
 * 0 = nav-frame/left, exp(d) q (option).  The HIP engine's UWVK_OPT_SO3_RIGHT. */
void or_set_so3_right(int on);
int or_get_so3_right(void);

/* ---- PoseUKF ------------------------------------------------------------ */
int or_pose_init_from_config(or_pose* f, int dof, const double pos[3], const double pos_cov[9], const double rot[4],
                             const double rot_cov[9], const uwvk_pose_config* cfg, const uwvk_uwv_params* uwv,
                             const double imu_in_body[7]);
int or_pose_init_from_state(or_pose* f, int dof, const double* x, const double* P, const uwvk_location* loc,
                            const uwvk_uwv_params* uwv, const uwvk_pose_parameter* param);
void or_pose_set_process_noise_from_config(or_pose* f, const uwvk_pose_config* cfg, double imu_dt,
                                           const double q_imu_in_body[4]);
void or_pose_set_process_noise(or_pose* f, const double* Q);
int or_pose_set_rotation_rate(or_pose* f, const double w[3], const double* cov);
int or_pose_predict(or_pose* f, double dt); /* 0 ok, UWVK_ENOTPD */
/* returns uwvk_status; *accepted = gate result */
int or_pose_update_acceleration(or_pose* f, const double mu[3], const double cov[9], int* accepted);
int or_pose_update_velocity(or_pose* f, const double mu[3], const double cov[9], int* accepted);
int or_pose_update_pressure(or_pose* f, const double mu[1], const double cov[1], const double sensor_in_imu[3],
                            int* accepted);
int or_pose_update_water_velocity(or_pose* f, const double mu[2], const double cov[4], double cell_weighting,
                                  int* accepted);
int or_pose_update_efforts(or_pose* f, const double mu[6], const double cov[36], int only_affect_velocity,
                           int* accepted);
int or_pose_update_xy(or_pose* f, const double mu[2], const double cov[4], int* accepted);
int or_pose_update_z(or_pose* f, const double mu[1], const double cov[1], int* accepted);
int or_pose_update_geographic(or_pose* f, const double mu[2], const double cov[4], const double gps_in_body[3],
                              int* accepted);
int or_pose_update_delayed_xy(or_pose* f, const double mu[2], const double cov[4], const double delayed_xy[2],
                              int* accepted);
void or_pose_reset_with_external_pose(or_pose* f, const double pose[7]);
void or_pose_get_rotation_rate(const or_pose* f, double out[3]);

/* ---- VelocityUKF -------------------------------------------------------- */
typedef struct or_vel {
  double mu[4];
  double sigma[16];
  double Q[16];
  double gyro[3];
  double efforts[6];
  int has_model;
  uwvk_uwv_params uwv;
  double Minv[36];
  double model_state[13]; /* motion_model pose: p(3) q(4) v(3) w(3) */
} or_vel;

void or_vel_init(or_vel* f, const double x[4], const double P[16]);
void or_vel_setup_motion_model(or_vel* f, const uwvk_uwv_params* uwv);
int or_vel_set_gyro(or_vel* f, const double w[3], const double* cov);
int or_vel_set_efforts(or_vel* f, const double tau[6], const double* cov);
int or_vel_predict(or_vel* f, double dt);
void or_vel_set_process_noise(or_vel* f, const double Q[16]);
int or_vel_update_dvl(or_vel* f, const double mu[3], const double cov[9]);
int or_vel_update_pressure(or_vel* f, const double mu[1], const double cov[1]);
/* one RK4 step of the [EXT] ModelSimulation (state: p q v w), exposed for tests */
void or_model_rk4(const uwvk_uwv_params* p, const double Minv[36], const double tau[6], double dt,
                  const double s_in[13], double s_out[13]);
int or_invert(int n, const double* A, double* Ainv);

/* ---- BottomUKF / IndirectPoseUKF / visual landmarks (uwvk_small_oracle.c) */
typedef struct or_bottom {  /* BottomUKF.hpp:15-53: {distance, normal (S2, unit 3-vector)} */
  double mu[4];
  double sigma[9];
  double Q[9];
  double velocity[3];
} or_bottom;
void or_bottom_init(or_bottom* f, const double x[4], const double P[9]);
void or_bottom_set_process_noise(or_bottom* f, const double Q[9]);
void or_bottom_set_velocity(or_bottom* f, const double v[3]);
int or_bottom_predict(or_bottom* f, double dt);
int or_bottom_update_range(or_bottom* f, double mu, double cov, const double dir[3], const double origin[3]);
int or_bottom_update_normal(or_bottom* f, const double mu[3], const double cov[4]);
size_t or_bottom_sizeof(void);

typedef struct or_ipose {  /* IndirectPoseUKF.hpp:18-86: {position_error, orientation_error} */
  double mu[7];
  double sigma[36];
  double Q[36];
  double pose_ref[7]; /* t(3), q(4) */
  double tau;
} or_ipose;
void or_ipose_init(or_ipose* f, const double pos_std[3], const double ori_std[3], double tau,
                   const double init_pos_err[3], const double init_pos_std[3]);
void or_ipose_set_pose_reference(or_ipose* f, const double pose[7]);
void or_ipose_set_process_noise(or_ipose* f, const double Q[36]);
int or_ipose_predict(or_ipose* f, double dt);
int or_ipose_update_visual(or_ipose* f, int nf, const double* features, const double* feature_cov,
                           const double* feature_pos, const double marker_pose[7], const double cov_marker[36],
                           const double cam_cfg[4], const double cam_in_body[7]);
void or_ipose_get_corrected_pose(const or_ipose* f, double out[7]);
size_t or_ipose_sizeof(void);
int or_pose_update_visual(or_pose* f, int nf, const double* features, const double* feature_cov,
                          const double* feature_pos, const double marker_pose[7], const double cov_marker[36],
                          const double cam_cfg[4], const double cam_in_imu[7]);
void or_s2_boxplus(const double x[3], const double d[2], double s, double o[3]);
void or_s2_boxminus(const double y[3], const double x[3], double o[2]);
void or_s2_from_vector(const double v[3], double o[3]);

/* ---- batched log runners (cpu_baseline leg + golden fixtures) ----------- */
/* Host-array version of uwvk_pose_log; arrays are host pointers. */
typedef struct or_pose_run_args {
  int64_t batch, epochs;
  double dt;
  const uint32_t* flags;
  const double* gyro; /* [epochs][batch][3] */
  const double* acc;
  double acc_cov[9];
  const int32_t* dvl_index;
  const double* dvl;
  double dvl_cov[9];
  const int32_t* pressure_index;
  const double* pressure;
  double pressure_cov;
  double pressure_sensor_in_imu[3];
  const int32_t* adcp_index;
  const double* adcp;
  int32_t adcp_cells;
  double adcp_cell_weighting[8];
  double adcp_cov[4];
  const int32_t* efforts_index;
  const double* efforts;
  double efforts_cov[36];
} or_pose_run_args;

/* Runs `count` epochs starting at `first` on filters[0..batch) with nthreads
 * pthreads.  accept_counts nullable: [batch][4].  Returns 0 or first error. */
int or_pose_run_log(or_pose* filters, const or_pose_run_args* a, int64_t first, int64_t count, int nthreads,
                    uint32_t* accept_counts);
size_t or_pose_sizeof(void);
/* VelocityUKF log (config C2), host arrays; layout as uwvk_vel_log */
typedef struct or_vel_run_args {
  int64_t batch, epochs;
  double dt;
  const uint32_t* flags;
  const double* gyro;    /* [epochs][batch][3] */
  const double* efforts; /* [epochs][batch][6] */
  const int32_t* dvl_index;
  const double* dvl;
  double dvl_cov[9];
  const int32_t* pressure_index;
  const double* pressure;
  double pressure_cov;
} or_vel_run_args;
/* VelocityUKF driver loop per epoch (gyro, efforts, predict, DVL, pressure),
 * instances split over nthreads pthreads.  Returns 0 or the first error. */
int or_vel_run_log(or_vel* filters, const or_vel_run_args* a, int64_t first, int64_t count, int nthreads);
void or_pose_get_state(const or_pose* f, double* x, double* P);
void or_vel_get_state(const or_vel* f, double* x, double* P, double* model_state);
size_t or_vel_sizeof(void);

#ifdef __cplusplus
}
#endif
#endif
