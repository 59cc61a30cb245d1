// uwvk_host.hpp — host-side (init-time) helpers of the engine: initial state
// and covariance from PoseUKFConfig, process noise, offsets.  These run once
// per handle on the CPU, exactly where the reference runs them (constructor /
// setProcessNoiseFromConfig); the per-step hot path is on the GPU.
#pragma once
#include <cmath>
#include <cstring>

#include "../../include/uwvk.h"

namespace uwvk {

// the last HIP error a uwvk_* call turned into UWVK_EDEVICE on this host
// thread (uwvk_last_device_error); HIPCHK records it
void note_hip_error(int err, const char* where);
namespace host {

inline void wgs84_radii(double lat0, double* rm, double* rn) {  // [EXT] GeographicProjection
  const double a = 6378137.0, f = 1.0 / 298.257223563;
  const double e2 = f * (2.0 - f);
  const double s = std::sin(lat0);
  const double den = 1.0 - e2 * s * s;
  const double sq = std::sqrt(den);
  *rn = a / sq;
  *rm = a * (1.0 - e2) / (den * sq);
}

inline double wgs84_gravity(double lat, double alt) {  // [EXT] GravitationalModel::WGS_84
  const double s2 = std::sin(lat) * std::sin(lat);
  return 9.7803253359 * (1.0 + 0.00193185265241 * s2) / std::sqrt(1.0 - 0.00669437999013 * s2) - 3.086e-6 * alt;
}

inline void quat_matrix(const double q[4], double R[9]) {
  const double w = q[0], x = q[1], y = q[2], z = q[3];
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w;
  const double txx = tx * x, txy = ty * x, txz = tz * x;
  const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

struct Offs {  // storage / tangent offsets of PoseState (PoseState.hpp:29-45)
  int has_params, s_inertia, s_lin, s_quad, s_wv, s_wvb, s_badcp, s_rho;
  int d_inertia, d_lin, d_quad, d_wv, d_wvb, d_badcp, d_rho;
};
inline Offs offsets(int dof) {
  if (dof == 53) return Offs{1, 20, 29, 38, 47, 49, 51, 53, 19, 28, 37, 46, 48, 50, 52};
  return Offs{0, -1, -1, -1, 20, 22, 24, 26, -1, -1, -1, 19, 21, 23, 25};
}

static const int kIdx[3] = {0, 1, 5};  // (surge, sway, yaw), PoseUKF.cpp:160-171

// PoseUKF::PoseUKF(pose, config, uwv, imu_in_body), PoseUKF.cpp:288-372
inline void pose_initial_state(int n, const double pos[3], const double pos_cov[9], const double rot[4],
                               const double rot_cov[9], const uwvk_pose_config& cfg, const uwvk_uwv_params& uwv,
                               const double* imu_in_body, double* x, double* P, uwvk_pose_parameter* par) {
  const Offs o = offsets(n);
  double qb[4] = {1, 0, 0, 0}, tb[3] = {0, 0, 0}, Mb[9];
  if (imu_in_body) {
    std::memcpy(tb, imu_in_body, 3 * sizeof(double));
    std::memcpy(qb, imu_in_body + 3, 4 * sizeof(double));
  }
  quat_matrix(qb, Mb);
  std::memcpy(x, pos, 3 * sizeof(double));
  std::memcpy(x + 3, rot, 4 * sizeof(double));
  for (int i = 0; i < 3; i++) {
    x[7 + i] = 0.0;
    x[10 + i] = 0.0;
    double sg = 0, sa = 0;
    for (int k = 0; k < 3; k++) {
      sg += Mb[i * 3 + k] * cfg.rotation_rate.bias_offset[k];
      sa += Mb[i * 3 + k] * cfg.acceleration.bias_offset[k];
    }
    x[13 + i] = sg;
    x[16 + i] = sa;
  }
  x[19] = wgs84_gravity(cfg.location.latitude, cfg.location.altitude);
  if (o.has_params)
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        x[o.s_inertia + a + 3 * b] = uwv.inertia_matrix[kIdx[a] * 6 + kIdx[b]];
        x[o.s_lin + a + 3 * b] = uwv.damping_matrices[0][kIdx[a] * 6 + kIdx[b]];
        x[o.s_quad + a + 3 * b] = uwv.damping_matrices[1][kIdx[a] * 6 + kIdx[b]];
      }
  for (int i = 0; i < 2; i++) x[o.s_wv + i] = x[o.s_wvb + i] = x[o.s_badcp + i] = 0.0;
  x[o.s_rho] = cfg.hydrostatics.water_density;

  for (int i = 0; i < n * n; i++) P[i] = 0.0;
  auto pb = [&](int d0, int r, int c, double v) { P[(d0 + r) * n + d0 + c] = v; };
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      pb(0, r, c, pos_cov[r * 3 + c]);
      pb(3, r, c, rot_cov[r * 3 + c]);
      pb(6, r, c, r == c ? 1.0 : 0.0);
      pb(9, r, c, r == c ? 10.0 : 0.0);
      double sg = 0, sa = 0;
      for (int k = 0; k < 3; k++) {
        const double bg = cfg.rotation_rate.bias_instability[k], ba = cfg.acceleration.bias_instability[k];
        sg += Mb[r * 3 + k] * (bg * bg) * Mb[c * 3 + k];
        sa += Mb[r * 3 + k] * (ba * ba) * Mb[c * 3 + k];
      }
      pb(12, r, c, sg);
      pb(15, r, c, sa);
    }
  pb(18, 0, 0, std::pow(0.05, 2.));
  if (o.has_params)
    for (int k = 0; k < 9; k++) {
      const double a = cfg.model_noise_parameters.inertia_instability[k];
      const double b = cfg.model_noise_parameters.lin_damping_instability[k];
      const double c = cfg.model_noise_parameters.quad_damping_instability[k];
      pb(o.d_inertia, k, k, a * a);
      pb(o.d_lin, k, k, b * b);
      pb(o.d_quad, k, k, c * c);
    }
  const double wl = std::pow(cfg.water_velocity.limits, 2), al = std::pow(cfg.water_velocity.adcp_bias_limits, 2);
  for (int k = 0; k < 2; k++) {
    pb(o.d_wv, k, k, wl);
    pb(o.d_wvb, k, k, wl);
    pb(o.d_badcp, k, k, al);
  }
  pb(o.d_rho, 0, 0, std::pow(cfg.hydrostatics.water_density_limits, 2.));

  uwvk_pose_parameter& p = *par;
  std::memcpy(p.imu_in_body, tb, 3 * sizeof(double));
  p.acc_bias_tau = cfg.acceleration.bias_tau;
  std::memcpy(p.acc_bias_offset, x + 16, 3 * sizeof(double));
  p.gyro_bias_tau = cfg.rotation_rate.bias_tau;
  std::memcpy(p.gyro_bias_offset, x + 13, 3 * sizeof(double));
  p.inertia_tau = cfg.model_noise_parameters.inertia_tau;
  p.lin_damping_tau = cfg.model_noise_parameters.lin_damping_tau;
  p.quad_damping_tau = cfg.model_noise_parameters.quad_damping_tau;
  p.water_velocity_tau = cfg.water_velocity.tau;
  p.water_velocity_limits = cfg.water_velocity.limits;
  p.water_velocity_scale = cfg.water_velocity.scale;
  p.adcp_bias_tau = cfg.water_velocity.adcp_bias_tau;
  p.atmospheric_pressure = cfg.hydrostatics.atmospheric_pressure;
  p.water_density_tau = cfg.hydrostatics.water_density_tau;
}

// inertia / lin / quad offsets (col-major 9 each) + density offset (PoseUKF.cpp:346-349)
inline void pose_offsets(int n, const double* x, double* off) {
  const Offs o = offsets(n);
  for (int k = 0; k < 28; k++) off[k] = 0.0;
  if (o.has_params)
    for (int k = 0; k < 9; k++) {
      off[k] = x[o.s_inertia + k];
      off[9 + k] = x[o.s_lin + k];
      off[18 + k] = x[o.s_quad + k];
    }
  off[27] = x[o.s_rho];
}

// the (surge, sway, yaw) blocks of the base UWV model (col-major 3x3 each)
inline void model_blocks(const uwvk_uwv_params& u, double* m) {
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) {
      m[a + 3 * b] = u.inertia_matrix[kIdx[a] * 6 + kIdx[b]];
      m[9 + a + 3 * b] = u.damping_matrices[0][kIdx[a] * 6 + kIdx[b]];
      m[18 + a + 3 * b] = u.damping_matrices[1][kIdx[a] * 6 + kIdx[b]];
    }
}

// setProcessNoiseFromConfig, PoseUKF.cpp:393-439
inline void pose_process_noise(int n, const uwvk_pose_config& cfg, double dt, const double* q_imu_in_body, double* Q) {
  const Offs o = offsets(n);
  double qb[4] = {1, 0, 0, 0}, M[9];
  if (q_imu_in_body) std::memcpy(qb, q_imu_in_body, 4 * sizeof(double));
  quat_matrix(qb, M);
  for (int i = 0; i < n * n; i++) Q[i] = 0.0;
  auto qb_ = [&](int d0, int r, int c, double v) { Q[(d0 + r) * n + d0 + c] = v; };
  for (int r = 0; r < 3; r++) {
    const double j = cfg.max_jerk[r];
    const double jp = (1. / 6.) * 0.25 * j, jv = 0.5 * 0.25 * j, ja = 0.25 * j;
    qb_(0, r, r, 1.5 * (std::pow(dt, 4.0) * (jp * jp)));
    qb_(6, r, r, 1.5 * (std::pow(dt, 2.0) * (jv * jv)));
    qb_(9, r, r, ja * ja);
  }
  const double kg = 2. / (cfg.rotation_rate.bias_tau * dt), ka = 2. / (cfg.acceleration.bias_tau * dt);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double so = 0, sg = 0, sa = 0;
      for (int k = 0; k < 3; k++) {
        const double rw = cfg.rotation_rate.randomwalk[k];
        const double bg = cfg.rotation_rate.bias_instability[k], ba = cfg.acceleration.bias_instability[k];
        so += M[r * 3 + k] * (rw * rw) * M[c * 3 + k];
        sg += M[r * 3 + k] * (kg * (bg * bg)) * M[c * 3 + k];
        sa += M[r * 3 + k] * (ka * (ba * ba)) * M[c * 3 + k];
      }
      qb_(3, r, c, so);
      qb_(12, r, c, sg);
      qb_(15, r, c, sa);
    }
  qb_(18, 0, 0, 1.e-12);
  if (o.has_params) {
    const uwvk_model_noise& mn = cfg.model_noise_parameters;
    for (int k = 0; k < 9; k++) {
      qb_(o.d_inertia, k, k, (2. / (mn.inertia_tau * dt)) * (mn.inertia_instability[k] * mn.inertia_instability[k]));
      qb_(o.d_lin, k, k,
          (2. / (mn.lin_damping_tau * dt)) * (mn.lin_damping_instability[k] * mn.lin_damping_instability[k]));
      qb_(o.d_quad, k, k,
          (2. / (mn.quad_damping_tau * dt)) * (mn.quad_damping_instability[k] * mn.quad_damping_instability[k]));
    }
  }
  const double qwv = (2. / (cfg.water_velocity.tau * dt)) * std::pow(cfg.water_velocity.limits, 2);
  const double qad = (2. / (cfg.water_velocity.adcp_bias_tau * dt)) * std::pow(cfg.water_velocity.adcp_bias_limits, 2);
  for (int k = 0; k < 2; k++) {
    qb_(o.d_wv, k, k, qwv);
    qb_(o.d_wvb, k, k, qwv);
    qb_(o.d_badcp, k, k, qad);
  }
  qb_(o.d_rho, 0, 0,
      (2. / (cfg.hydrostatics.water_density_tau * dt)) * std::pow(cfg.hydrostatics.water_density_limits, 2.));
}

// 6x6 inverse by Gauss-Jordan with partial pivoting (M^-1 of the UWV model)
inline bool invert6(const double* A, double* X) {
  double M[6][12];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 12; j++) M[i][j] = j < 6 ? A[i * 6 + j] : (j - 6 == i ? 1.0 : 0.0);
  for (int c = 0; c < 6; c++) {
    int p = c;
    for (int r = c + 1; r < 6; r++)
      if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
    if (M[p][c] == 0.0) return false;
    if (p != c)
      for (int j = 0; j < 12; j++) std::swap(M[c][j], M[p][j]);
    const double ip = 1.0 / M[c][c];
    for (int j = 0; j < 12; j++) M[c][j] *= ip;
    for (int r = 0; r < 6; r++) {
      if (r == c) continue;
      const double f = M[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 12; j++) M[r][j] -= f * M[c][j];
    }
  }
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) X[i * 6 + j] = M[i][6 + j];
  return true;
}

}  // namespace host
}  // namespace uwvk
