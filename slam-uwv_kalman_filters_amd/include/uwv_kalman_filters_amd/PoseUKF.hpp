// PoseUKF.hpp — C++ host facade over the batched C ABI (include/uwvk.h).
//
// Mirrors the reference's class interface (src/PoseUKF.hpp:40-205,
// src/VelocityUKF.hpp:33-62) in two call forms on the same object:
//
//  * the REFERENCE form (a drop-in for a caller written against the reference):
//    the batch-1 constructors in the reference's parameter order, the nested
//    MEASUREMENT types (PoseUKF::Velocity, ::WaterVelocityMeasurement, ...,
//    VelocityUKF::BodyEffortsMeasurement) with Eigen-style .mu / .cov, State /
//    Covariance, integrateMeasurement(adcp, cell_weighting),
//    resetFilterWithExternalPose(Affine3d), getRotationRate() -> Mu,
//    getCurrentState(State&[, Covariance&]).  The value types are Eigen's
//    where Eigen is installed, else the small stand-ins of linalg.hpp.  On an
//    object with batch > 1 a single measurement is applied to every instance
//    and the single-filter getters read instance 0 (or the one named);
//  * the BATCHED form: each object owns a batch of independent filters on one
//    gfx950 device; measurements carry one row per instance (namespace
//    `batch`, e.g. batch::Velocity), with per-instance masks and gate results.
//
// Errors the reference reports by throwing (NaN measurements, non-PD
// covariance, no motion model) throw here as well (uwvk::Error carries the
// uwvk_status).  Header-only; link with libuwvk.so.  No HIP types in the
// interface.  <uwv_kalman_filters/PoseUKF.hpp> includes this header under the
// reference's include path and namespace.
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/uwvk.h"
#include "linalg.hpp"
#include "reference_types.hpp"

namespace uwv_kalman_filters_amd {

struct Error : std::runtime_error {
  uwvk_status code;
  Error(uwvk_status c, const std::string& where)
      : std::runtime_error(where + ": " + uwvk_status_string(c)), code(c) {}
};

inline void check(uwvk_status s, const char* where) {
  if (s != UWVK_OK) throw Error(s, where);
}

// the library must implement the ABI this header describes (include/uwvk.h)
inline void check_abi() {
  if (uwvk_abi_version() != UWVK_ABI_VERSION)
    throw std::runtime_error("libuwvk.so ABI version " + std::to_string(uwvk_abi_version()) +
                             ", this facade needs " + std::to_string(UWVK_ABI_VERSION));
}

// ---- batched measurements: one row per instance ----------------------------
namespace batch {
// One measurement for every instance of the batch (reference: MEASUREMENT(Name, M)
// = {mu, cov}, PoseUKF.hpp:79-88).  cov holds batch*M*M values, or is empty to use
// shared_cov for all instances.  mask (optional, batch bytes) skips instances.
template <int M>
struct BatchMeasurement {
  static constexpr int dim = M;
  std::vector<double> mu;
  std::vector<double> cov;
  std::array<double, M * M> shared_cov{};
  std::vector<uint8_t> mask;
};
struct GeographicPosition : BatchMeasurement<2> {};
struct XY_Position : BatchMeasurement<2> {};
struct Z_Position : BatchMeasurement<1> {};
struct Pressure : BatchMeasurement<1> {};
struct RotationRate : BatchMeasurement<3> {};
struct Acceleration : BatchMeasurement<3> {};
struct Velocity : BatchMeasurement<3> {};
struct BodyEffortsMeasurement : BatchMeasurement<6> {};
struct WaterVelocityMeasurement : BatchMeasurement<2> {};
// VisualFeatureMeasurement (PoseUKF.hpp:88, IndirectPoseUKF.hpp:35): ONE feature
// for every instance: mu batch*2 undistorted image coordinates (px), cov
// batch*4 (px^2) or empty for shared_cov.
struct VisualFeatureMeasurement : BatchMeasurement<2> {};
// VelocityUKF's (VelocityUKF.hpp:36-39)
struct DVLMeasurement : BatchMeasurement<3> {};
struct GyroMeasurement : BatchMeasurement<3> {};
struct VelBodyEffortsMeasurement : BatchMeasurement<6> {};
struct PressureMeasurement : BatchMeasurement<1> {};
}  // namespace batch
// the batched types under their earlier namespace-scope names
using batch::BatchMeasurement;
using batch::GeographicPosition;
using batch::XY_Position;
using batch::Z_Position;
using batch::Pressure;
using batch::RotationRate;
using batch::Acceleration;
using batch::Velocity;
using batch::BodyEffortsMeasurement;
using batch::WaterVelocityMeasurement;
using batch::VisualFeatureMeasurement;
using batch::DVLMeasurement;
using batch::GyroMeasurement;
using batch::VelBodyEffortsMeasurement;
using batch::PressureMeasurement;

// Affine3d as {t, q(w, x, y, z)} for the batched calls
struct Pose7 {
  std::array<double, 3> t{};
  std::array<double, 4> q{{1.0, 0.0, 0.0, 0.0}};
};

namespace detail {
// Packs a reference-style feature list into the C ABI's [batch][nf][...] arrays.
struct VisualPack {
  std::vector<double> features, fcov, fpos, marker, cam_in;
  int fcov_pi = 0, marker_pi = 0, nf = 0;
  double cam[4] = {0, 0, 0, 0};
  VisualPack(int64_t batch, const std::vector<batch::VisualFeatureMeasurement>& f,
             const std::vector<std::array<double, 3>>& positions, const std::vector<Pose7>& marker_pose,
             const CameraConfiguration& cc, const Pose7& cam_in_body) {
    if (f.size() != positions.size())
      throw std::invalid_argument("integrateMeasurement(VisualFeature): features / positions size mismatch");
    if (marker_pose.size() != 1 && marker_pose.size() != (size_t)batch)
      throw std::invalid_argument("integrateMeasurement(VisualFeature): marker_pose size");
    nf = (int)f.size();
    const size_t B = (size_t)batch;
    fcov_pi = 0;
    for (const auto& m : f) {
      if (m.mu.size() != B * 2) throw std::invalid_argument("VisualFeatureMeasurement: mu size");
      if (!m.cov.empty()) fcov_pi = 1;
    }
    features.assign(B * nf * 2, 0.0);
    fcov.assign(fcov_pi ? B * nf * 4 : (size_t)nf * 4, 0.0);
    for (int i = 0; i < nf; i++) {
      for (size_t b = 0; b < B; b++) {
        features[(b * nf + i) * 2] = f[i].mu[b * 2];
        features[(b * nf + i) * 2 + 1] = f[i].mu[b * 2 + 1];
        if (fcov_pi)
          for (int k = 0; k < 4; k++) fcov[(b * nf + i) * 4 + k] = f[i].cov.empty() ? f[i].shared_cov[k] : f[i].cov.at(b * 4 + k);
      }
      if (!fcov_pi)
        for (int k = 0; k < 4; k++) fcov[(size_t)i * 4 + k] = f[i].shared_cov[k];
      for (int k = 0; k < 3; k++) fpos.push_back(positions[i][k]);
    }
    marker_pi = marker_pose.size() == B && B > 1;
    for (size_t b = 0; b < (marker_pi ? B : 1); b++) {
      for (int k = 0; k < 3; k++) marker.push_back(marker_pose[b].t[k]);
      for (int k = 0; k < 4; k++) marker.push_back(marker_pose[b].q[k]);
    }
    cam[0] = cc.fx; cam[1] = cc.fy; cam[2] = cc.cx; cam[3] = cc.cy;
    for (int k = 0; k < 3; k++) cam_in.push_back(cam_in_body.t[k]);
    for (int k = 0; k < 4; k++) cam_in.push_back(cam_in_body.q[k]);
  }
};

inline Pose7 pose7(const Affine3d& a) {
  double p[7];
  pose7_of(a, p);
  Pose7 r;
  for (int k = 0; k < 3; k++) r.t[k] = p[k];
  for (int k = 0; k < 4; k++) r.q[k] = p[3 + k];
  return r;
}

// one single-filter vector repeated for every instance of the batch
template <class V>
std::vector<double> repeat(const V& v, int64_t batch) {
  const int n = (int)v.size();
  std::vector<double> r((size_t)batch * n);
  for (int64_t b = 0; b < batch; b++)
    for (int k = 0; k < n; k++) r[(size_t)b * n + k] = v(k);
  return r;
}
inline std::vector<double> repeat(const std::vector<double>& v, int64_t batch) {
  std::vector<double> r;
  r.reserve((size_t)batch * v.size());
  for (int64_t b = 0; b < batch; b++) r.insert(r.end(), v.begin(), v.end());
  return r;
}
template <class M>
std::vector<double> rowmajor(const M& m) {
  std::vector<double> r((size_t)m.rows() * m.cols());
  put_rowmajor(m, r.data());
  return r;
}
}  // namespace detail

// PoseUKF::PoseUKFParameter (PoseUKF.hpp:46-76), Eigen-typed like the reference's
struct PoseUKFParameter {
  Vector3d imu_in_body = Vector3d::Zero();
  Vector3d gyro_bias_offset = Vector3d::Zero();
  double gyro_bias_tau = 0;
  Vector3d acc_bias_offset = Vector3d::Zero();
  double acc_bias_tau = 0;
  double inertia_tau = 0;
  double lin_damping_tau = 0;
  double quad_damping_tau = 0;
  double water_velocity_tau = 0;
  double water_velocity_limits = 0;
  double water_velocity_scale = 0;
  double adcp_bias_tau = 0;
  double atmospheric_pressure = 0;
  double water_density_tau = 0;

  uwvk_pose_parameter to_c() const {
    uwvk_pose_parameter p{};
    for (int k = 0; k < 3; k++) {
      p.imu_in_body[k] = imu_in_body(k);
      p.gyro_bias_offset[k] = gyro_bias_offset(k);
      p.acc_bias_offset[k] = acc_bias_offset(k);
    }
    p.gyro_bias_tau = gyro_bias_tau;
    p.acc_bias_tau = acc_bias_tau;
    p.inertia_tau = inertia_tau;
    p.lin_damping_tau = lin_damping_tau;
    p.quad_damping_tau = quad_damping_tau;
    p.water_velocity_tau = water_velocity_tau;
    p.water_velocity_limits = water_velocity_limits;
    p.water_velocity_scale = water_velocity_scale;
    p.adcp_bias_tau = adcp_bias_tau;
    p.atmospheric_pressure = atmospheric_pressure;
    p.water_density_tau = water_density_tau;
    return p;
  }
};

class PoseUKF {
 public:
  // ---- the reference's nested types (PoseUKF.hpp:46-88) ----
  using PoseUKFParameter = ::uwv_kalman_filters_amd::PoseUKFParameter;
  struct GeographicPosition : Measurement<2> {};
  struct XY_Position : Measurement<2> {};
  struct Z_Position : Measurement<1> {};
  struct Pressure : Measurement<1> {};
  struct RotationRate : Measurement<3> {};
  struct Acceleration : Measurement<3> {};
  struct Velocity : Measurement<3> {};
  struct BodyEffortsMeasurement : Measurement<6> {};
  struct WaterVelocityMeasurement : Measurement<2> {};
  struct VisualFeatureMeasurement : Measurement<2> {};
  typedef PoseState State;
  typedef Matrix<PoseState::DOF, PoseState::DOF> Covariance;

  // ---- reference constructors (batch = 1) ----
  // PoseUKF(imu_in_nwu_pos, pos_cov, rot, rot_cov, config, model, imu_in_body) (PoseUKF.hpp:100-103)
  PoseUKF(const Vector3d& imu_in_nwu_pos, const Matrix3d& imu_in_nwu_pos_cov, const Quaterniond& imu_in_nwu_rot,
          const Matrix3d& imu_in_nwu_rot_cov, const PoseUKFConfig& pose_filter_config,
          const UWVParameters& model_parameters, const Affine3d& imu_in_body = Affine3d::Identity())
      : h_(create(1, PoseState::DOF, 0)) {
    guard([&] {
      double pos[3], pc[9], rot[4], rc[9], ib[7];
      for (int k = 0; k < 3; k++) pos[k] = imu_in_nwu_pos(k);
      detail::put_rowmajor(imu_in_nwu_pos_cov, pc);
      detail::put_rowmajor(imu_in_nwu_rot_cov, rc);
      rot[0] = imu_in_nwu_rot.w(); rot[1] = imu_in_nwu_rot.x(); rot[2] = imu_in_nwu_rot.y(); rot[3] = imu_in_nwu_rot.z();
      detail::pose7_of(imu_in_body, ib);
      const uwvk_pose_config c = pose_filter_config.to_c();
      const uwvk_uwv_params m = model_parameters.to_c();
      check(uwvk_pose_init_from_config(h_, pos, pc, rot, rc, &c, &m, ib), "PoseUKF");
    });
  }
  // PoseUKF(initial_state, state_cov, location, model, filter_parameter) (PoseUKF.hpp:113-115)
  PoseUKF(const State& initial_state, const Covariance& state_cov, const LocationConfiguration& location,
          const UWVParameters& model_parameters, const PoseUKFParameter& filter_parameter)
      : h_(create(1, PoseState::DOF, 0)) {
    guard([&] {
      double x[UWVK_POSE_STORE_FULL];
      initial_state.to_store(x);
      const std::vector<double> P = detail::rowmajor(state_cov);
      const uwvk_uwv_params m = model_parameters.to_c();
      const uwvk_pose_parameter p = filter_parameter.to_c();
      check(uwvk_pose_init_from_state(h_, x, P.data(), &location, &m, &p), "PoseUKF");
    });
  }

  // ---- batched constructors ----
  // per instance pos[3], pos_cov[9], rot[4] (w,x,y,z), rot_cov[9]; imu_in_body {t, q} or null
  PoseUKF(int64_t batch, const std::vector<double>& pos, const std::vector<double>& pos_cov,
          const std::vector<double>& rot, const std::vector<double>& rot_cov, const uwvk_pose_config& cfg,
          const uwvk_uwv_params& model, const double* imu_in_body = nullptr, int dof = 53, int device = 0)
      : h_(create(batch, dof, device)) {
    guard([&] {
      need(pos, 3, "pos"); need(pos_cov, 9, "pos_cov"); need(rot, 4, "rot"); need(rot_cov, 9, "rot_cov");
      check(uwvk_pose_init_from_config(h_, pos.data(), pos_cov.data(), rot.data(), rot_cov.data(), &cfg, &model,
                                       imu_in_body),
            "PoseUKF");
    });
  }
  PoseUKF(int64_t batch, const std::vector<double>& pos, const std::vector<double>& pos_cov,
          const std::vector<double>& rot, const std::vector<double>& rot_cov, const PoseUKFConfig& cfg,
          const UWVParameters& model, const Affine3d& imu_in_body = Affine3d::Identity(), int dof = 53,
          int device = 0)
      : h_(create(batch, dof, device)) {
    guard([&] {
      need(pos, 3, "pos"); need(pos_cov, 9, "pos_cov"); need(rot, 4, "rot"); need(rot_cov, 9, "rot_cov");
      double ib[7];
      detail::pose7_of(imu_in_body, ib);
      const uwvk_pose_config c = cfg.to_c();
      const uwvk_uwv_params m = model.to_c();
      check(uwvk_pose_init_from_config(h_, pos.data(), pos_cov.data(), rot.data(), rot_cov.data(), &c, &m, ib),
            "PoseUKF");
    });
  }
  // per instance state[store], cov[dof*dof] (row-major, lower triangle read)
  PoseUKF(int64_t batch, const std::vector<double>& state, const std::vector<double>& cov,
          const LocationConfiguration& location, const uwvk_uwv_params& model, const uwvk_pose_parameter& param,
          int dof = 53, int device = 0)
      : h_(create(batch, dof, device)) {
    guard([&] {
      need(state, store(), "state"); need(cov, (size_t)dof * dof, "cov");
      check(uwvk_pose_init_from_state(h_, state.data(), cov.data(), &location, &model, &param), "PoseUKF");
    });
  }
  PoseUKF(const PoseUKF&) = delete;
  PoseUKF& operator=(const PoseUKF&) = delete;
  PoseUKF(PoseUKF&& o) noexcept : h_(std::exchange(o.h_, nullptr)) {}
  virtual ~PoseUKF() { uwvk_pose_destroy(h_); }

  int64_t batch() const { return uwvk_pose_batch(h_); }
  int dof() const { return uwvk_pose_dof(h_); }
  size_t store() const { return dof() == 53 ? 54 : 27; }
  uwvk_pose* handle() { return h_; }

  // setProcessNoiseFromConfig (PoseUKF.hpp:126-127)
  void setProcessNoiseFromConfig(const PoseUKFConfig& cfg, double imu_delta_t,
                                 const Quaterniond& imu_in_body = Quaterniond::Identity()) {
    const uwvk_pose_config c = cfg.to_c();
    const double q[4] = {imu_in_body.w(), imu_in_body.x(), imu_in_body.y(), imu_in_body.z()};
    check(uwvk_pose_set_process_noise_from_config(h_, &c, imu_delta_t, q), "setProcessNoiseFromConfig");
  }
  void setProcessNoiseFromConfig(const uwvk_pose_config& cfg, double imu_delta_t,
                                 const double* q_imu_in_body = nullptr) {
    check(uwvk_pose_set_process_noise_from_config(h_, &cfg, imu_delta_t, q_imu_in_body),
          "setProcessNoiseFromConfig");
  }
  // setProcessNoiseCovariance [EXT pose_estimation base]
  void setProcessNoiseCovariance(const Covariance& Q) {
    if (dof() != PoseState::DOF) throw std::invalid_argument("setProcessNoiseCovariance: 53-DOF filter only");
    const std::vector<double> q = detail::rowmajor(Q);
    check(uwvk_pose_set_process_noise(h_, q.data()), "setProcessNoiseCovariance");
  }
  void setProcessNoiseCovariance(const std::vector<double>& Q) {
    if (Q.size() != (size_t)dof() * dof()) throw std::invalid_argument("setProcessNoiseCovariance: size");
    check(uwvk_pose_set_process_noise(h_, Q.data()), "setProcessNoiseCovariance");
  }
  // predictionStep(dt) [EXT base] -> predictionStepImpl (PoseUKF.cpp:446-474)
  void predictionStep(double delta_t) { check(uwvk_pose_predict(h_, delta_t), "predictionStep"); }

  // ---- reference integrateMeasurement overloads (PoseUKF.hpp:137-177) ----
  void integrateMeasurement(const GeographicPosition& m, const Vector3d& gps_in_body = Vector3d::Zero()) {
    const double g[3] = {gps_in_body(0), gps_in_body(1), gps_in_body(2)};
    single(m, "GeographicPosition", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_geographic(h_, mu, nullptr, cov, g, nullptr, acc());
    });
  }
  void integrateMeasurement(const XY_Position& m) {
    single(m, "XY_Position", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_xy(h_, mu, nullptr, cov, nullptr, acc());
    });
  }
  void integrateDelayedPositionMeasurement(const XY_Position& m, const Vector2d& delayed_position) {
    const std::vector<double> d = detail::repeat(delayed_position, batch());
    single(m, "XY_Position", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_delayed_xy(h_, mu, nullptr, cov, d.data(), nullptr, acc());
    });
  }
  void integrateMeasurement(const Z_Position& m) {
    single(m, "Z_Position", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_z(h_, mu, nullptr, cov, nullptr, acc());
    });
  }
  void integrateMeasurement(const Pressure& m, const Vector3d& pressure_sensor_in_imu = Vector3d::Zero()) {
    const double s[3] = {pressure_sensor_in_imu(0), pressure_sensor_in_imu(1), pressure_sensor_in_imu(2)};
    single(m, "Pressure", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_pressure(h_, mu, nullptr, cov, s, nullptr, acc());
    });
  }
  // stored only, the predict's input (PoseUKF.cpp:492-496)
  void integrateMeasurement(const RotationRate& m) {
    const std::vector<double> mu = detail::repeat(m.mu, batch());
    const std::vector<double> cov = detail::repeat(detail::rowmajor(m.cov), batch());
    check(uwvk_pose_set_rotation_rate(h_, mu.data(), cov.data()), "integrateMeasurement(RotationRate)");
  }
  void integrateMeasurement(const Acceleration& m) {
    single(m, "Acceleration", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_acceleration(h_, mu, nullptr, cov, nullptr, acc());
    });
  }
  void integrateMeasurement(const Velocity& m) {
    single(m, "Velocity", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_velocity(h_, mu, nullptr, cov, nullptr, acc());
    });
  }
  void integrateMeasurement(const BodyEffortsMeasurement& m, bool only_affect_velocity = false) {
    single(m, "BodyEffortsMeasurement", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_efforts(h_, mu, nullptr, cov, only_affect_velocity ? 1 : 0, nullptr, acc());
    });
  }
  void integrateMeasurement(const WaterVelocityMeasurement& m, double cell_weighting) {
    const std::vector<double> w((size_t)batch(), cell_weighting);
    single(m, "WaterVelocityMeasurement", [&](const double* mu, const double* cov) {
      return uwvk_pose_update_water_velocity(h_, mu, nullptr, cov, w.data(), nullptr, acc());
    });
  }
  // the visual-marker update (PoseUKF.hpp:174-177, PoseUKF.cpp:613-654)
  void integrateMeasurement(const std::vector<VisualFeatureMeasurement>& marker_features,
                            const std::vector<Vector3d>& feature_positions, const Affine3d& marker_pose,
                            const Matrix<6, 6> cov_marker_pose, const CameraConfiguration& camera_config,
                            const Affine3d& camera_in_IMU) {
    const int64_t B = batch();
    std::vector<batch::VisualFeatureMeasurement> f(marker_features.size());
    for (size_t i = 0; i < f.size(); i++) {
      f[i].mu = detail::repeat(marker_features[i].mu, B);
      f[i].cov = detail::repeat(detail::rowmajor(marker_features[i].cov), B);
    }
    std::vector<std::array<double, 3>> p(feature_positions.size());
    for (size_t i = 0; i < p.size(); i++)
      for (int k = 0; k < 3; k++) p[i][k] = feature_positions[i](k);
    std::array<double, 36> cm;
    detail::put_rowmajor(cov_marker_pose, cm.data());
    integrateMeasurement(f, p, std::vector<Pose7>{detail::pose7(marker_pose)}, cm, camera_config,
                         detail::pose7(camera_in_IMU));
  }
  // resetFilterWithExternalPose (PoseUKF.hpp:187, PoseUKF.cpp:685-691)
  void resetFilterWithExternalPose(const Affine3d& imu_in_nav) {
    double p[7];
    detail::pose7_of(imu_in_nav, p);
    std::vector<double> v((size_t)batch() * 7);
    for (size_t b = 0; b < (size_t)batch(); b++)
      for (int k = 0; k < 7; k++) v[b * 7 + k] = p[k];
    check(uwvk_pose_reset_with_external_pose(h_, v.data()), "resetFilterWithExternalPose");
  }
  // getRotationRate (PoseUKF.hpp:190, PoseUKF.cpp:693-699): IMU-frame rate of one instance
  RotationRate::Mu getRotationRate(int64_t instance = 0) {
    const std::vector<double> w = getRotationRateBatch();
    at(instance, "getRotationRate");
    RotationRate::Mu r;
    for (int k = 0; k < 3; k++) r(k) = w[(size_t)instance * 3 + k];
    return r;
  }
  // The inherited getters of pose_estimation::UnscentedKalmanFilter<State> [EXT]
  // (used at VelocityUKF.cpp:70: `if (getCurrentState(current_state))`): true once initialised.
  bool getCurrentState(State& state, int64_t instance = 0) {
    if (dof() != PoseState::DOF) throw std::invalid_argument("getCurrentState(State&): 53-DOF filter only");
    std::vector<double> x;
    getState(x);
    at(instance, "getCurrentState");
    state.from_store(&x[(size_t)instance * store()]);
    return true;
  }
  bool getCurrentState(State& state, Covariance& covariance, int64_t instance = 0) {
    if (dof() != PoseState::DOF) throw std::invalid_argument("getCurrentState(State&): 53-DOF filter only");
    std::vector<double> x, P;
    getState(x, &P);
    at(instance, "getCurrentState");
    state.from_store(&x[(size_t)instance * store()]);
    detail::get_rowmajor(&P[(size_t)instance * PoseState::DOF * PoseState::DOF], covariance);
    return true;
  }

  // ---- batched integrateMeasurement overloads: one row per instance ----
  void integrateMeasurement(const batch::RotationRate& m) {
    need(m.mu, 3, "RotationRate");
    check(uwvk_pose_set_rotation_rate(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()),
          "integrateMeasurement(RotationRate)");
  }
  void integrateMeasurement(const batch::Acceleration& m) { upd(m, uwvk_pose_update_acceleration, "Acceleration"); }
  void integrateMeasurement(const batch::Velocity& m) { upd(m, uwvk_pose_update_velocity, "Velocity"); }
  void integrateMeasurement(const batch::XY_Position& m) { upd(m, uwvk_pose_update_xy, "XY_Position"); }
  void integrateMeasurement(const batch::Z_Position& m) { upd(m, uwvk_pose_update_z, "Z_Position"); }
  void integrateMeasurement(const batch::Pressure& m, const std::array<double, 3>& pressure_sensor_in_imu = {}) {
    prep(m, "Pressure");
    check(uwvk_pose_update_pressure(h_, m.mu.data(), covp(m), m.shared_cov.data(), pressure_sensor_in_imu.data(),
                                    maskp(m), acc()),
          "integrateMeasurement(Pressure)");
  }
  void integrateMeasurement(const batch::GeographicPosition& m, const std::array<double, 3>& gps_in_body = {}) {
    prep(m, "GeographicPosition");
    check(uwvk_pose_update_geographic(h_, m.mu.data(), covp(m), m.shared_cov.data(), gps_in_body.data(),
                                      maskp(m), acc()),
          "integrateMeasurement(GeographicPosition)");
  }
  void integrateMeasurement(const batch::BodyEffortsMeasurement& m, bool only_affect_velocity = false) {
    prep(m, "BodyEffortsMeasurement");
    check(uwvk_pose_update_efforts(h_, m.mu.data(), covp(m), m.shared_cov.data(), only_affect_velocity ? 1 : 0,
                                   maskp(m), acc()),
          "integrateMeasurement(BodyEffortsMeasurement)");
  }
  // cell_weighting: one value per instance, or a single value for all
  void integrateMeasurement(const batch::WaterVelocityMeasurement& m, const std::vector<double>& cell_weighting) {
    prep(m, "WaterVelocityMeasurement");
    std::vector<double> w = cell_weighting.size() == 1 ? std::vector<double>((size_t)batch(), cell_weighting[0])
                                                       : cell_weighting;
    need(w, 1, "cell_weighting");
    check(uwvk_pose_update_water_velocity(h_, m.mu.data(), covp(m), m.shared_cov.data(), w.data(), maskp(m),
                                          acc()),
          "integrateMeasurement(WaterVelocityMeasurement)");
  }
  void integrateMeasurement(const batch::WaterVelocityMeasurement& m, double cell_weighting) {
    integrateMeasurement(m, std::vector<double>{cell_weighting});
  }
  // integrateDelayedPositionMeasurement (PoseUKF.hpp:143): delayed_position batch*2
  void integrateDelayedPositionMeasurement(const batch::XY_Position& m, const std::vector<double>& delayed_position) {
    prep(m, "XY_Position");
    need(delayed_position, 2, "delayed_position");
    check(uwvk_pose_update_delayed_xy(h_, m.mu.data(), covp(m), m.shared_cov.data(), delayed_position.data(),
                                      maskp(m), acc()),
          "integrateDelayedPositionMeasurement");
  }
  // marker_pose: one pose shared by the batch, or one per instance
  void integrateMeasurement(const std::vector<batch::VisualFeatureMeasurement>& marker_features,
                            const std::vector<std::array<double, 3>>& feature_positions,
                            const std::vector<Pose7>& marker_pose, const std::array<double, 36>& cov_marker_pose,
                            const CameraConfiguration& camera_config, const Pose7& camera_in_IMU,
                            const std::vector<uint8_t>& mask = {}) {
    detail::VisualPack v(batch(), marker_features, feature_positions, marker_pose, camera_config, camera_in_IMU);
    check(uwvk_pose_update_visual_landmark(h_, v.nf, v.features.data(), v.fcov.data(), v.fcov_pi, v.fpos.data(),
                                           v.marker.data(), v.marker_pi, cov_marker_pose.data(), v.cam,
                                           v.cam_in.data(), mask.empty() ? nullptr : mask.data()),
          "integrateMeasurement(VisualFeatureMeasurement)");
  }
  // per instance {tx,ty,tz,qw,qx,qy,qz}
  void resetFilterWithExternalPose(const std::vector<double>& imu_in_nav) {
    need(imu_in_nav, 7, "imu_in_nav");
    check(uwvk_pose_reset_with_external_pose(h_, imu_in_nav.data()), "resetFilterWithExternalPose");
  }
  // batch*3
  std::vector<double> getRotationRateBatch() {
    std::vector<double> w((size_t)batch() * 3);
    check(uwvk_pose_get_rotation_rate(h_, w.data()), "getRotationRate");
    return w;
  }
  // batch*store (x) and batch*dof*dof (P, full symmetric, row-major)
  void getState(std::vector<double>& x, std::vector<double>* P = nullptr) {
    x.resize((size_t)batch() * store());
    if (P) P->resize((size_t)batch() * dof() * dof());
    check(uwvk_pose_get_state(h_, x.data(), P ? P->data() : nullptr), "getState");
  }
  bool getCurrentState(std::vector<double>& state) {
    getState(state);
    return true;
  }
  bool getCurrentState(std::vector<double>& state, std::vector<double>& covariance) {
    getState(state, &covariance);
    return true;
  }
  // the ukf's mu() / sigma() (PoseUKF.cpp:448,453,516), batched
  std::vector<double> mu() {
    std::vector<double> x;
    getState(x);
    return x;
  }
  std::vector<double> sigma() {
    std::vector<double> x, P;
    getState(x, &P);
    return P;
  }
  // Ensemble statistics (layout: uwvk_pose_ensemble_stats); with an RCCL
  // communicator (uwvk_comm_init, void* ncclComm_t) summed over all ranks.
  std::vector<double> ensembleStats(const double* truth = nullptr, void* comm = nullptr) {
    std::vector<double> out(3 * store() + 2);
    check(uwvk_pose_ensemble_allreduce(h_, truth, out.data(), comm), "ensembleStats");
    return out;
  }
  // Gate decisions of the last update (1 = accepted), one byte per instance.
  const std::vector<uint8_t>& lastAccepted() const { return accepted_; }
  std::vector<uint32_t> status(bool clear = false) {
    std::vector<uint32_t> s((size_t)batch());
    check(uwvk_pose_get_status(h_, s.data(), clear ? 1 : 0), "status");
    return s;
  }
  // Multi-epoch path (uwvk_pose_run_log): one PSP k_psp_epoch launch per run of
  // epochs, split after each BodyEfforts epoch, whose efforts update then runs
  // alone on k_psp_efforts; UWVK_OPT_DENSE_SIGMA: one literal launch per epoch.
  void runLog(const uwvk_pose_log& log, int64_t first, int64_t count, uint32_t* accept_counts = nullptr) {
    check(uwvk_pose_run_log(h_, &log, first, count, accept_counts), "runLog");
  }
  void synchronize() { check(uwvk_pose_synchronize(h_), "synchronize"); }

 private:
  static uwvk_pose* create(int64_t batch, int dof, int device) {
    check_abi();
    uwvk_pose* h = nullptr;
    check(uwvk_pose_create(batch, dof, device, &h), "uwvk_pose_create");
    return h;
  }
  // a constructor body: the handle is released if it throws (no destructor runs then)
  template <class F>
  void guard(F f) {
    try {
      f();
    } catch (...) {
      uwvk_pose_destroy(h_);
      h_ = nullptr;
      throw;
    }
  }
  void at(int64_t instance, const char* what) const {
    if (instance < 0 || instance >= batch()) throw std::out_of_range(std::string(what) + ": instance");
  }
  void need(const std::vector<double>& v, size_t per, const char* what) const {
    if (v.size() != (size_t)batch() * per) throw std::invalid_argument(std::string(what) + ": wrong size");
  }
  // a single-filter measurement, repeated for every instance; cov shared
  template <int M, class F>
  void single(const Measurement<M>& m, const char* what, F fn) {
    const std::vector<double> mu = detail::repeat(m.mu, batch());
    double cov[M * M];
    detail::put_rowmajor(m.cov, cov);
    check(fn(mu.data(), cov), (std::string("integrateMeasurement(") + what + ")").c_str());
  }
  template <int M>
  void prep(const batch::BatchMeasurement<M>& m, const char* what) {
    need(m.mu, M, what);
    if (!m.cov.empty()) need(m.cov, (size_t)M * M, what);
    if (!m.mask.empty() && m.mask.size() != (size_t)batch()) throw std::invalid_argument("mask: wrong size");
  }
  template <int M>
  static const double* covp(const batch::BatchMeasurement<M>& m) { return m.cov.empty() ? nullptr : m.cov.data(); }
  template <int M>
  static const uint8_t* maskp(const batch::BatchMeasurement<M>& m) { return m.mask.empty() ? nullptr : m.mask.data(); }
  uint8_t* acc() {
    accepted_.assign((size_t)batch(), 0);
    return accepted_.data();
  }
  template <int M, class F>
  void upd(const batch::BatchMeasurement<M>& m, F fn, const char* what) {
    prep(m, what);
    check(fn(h_, m.mu.data(), covp(m), m.shared_cov.data(), maskp(m), acc()),
          (std::string("integrateMeasurement(") + what + ")").c_str());
  }

  uwvk_pose* h_ = nullptr;
  std::vector<uint8_t> accepted_;
};

// VelocityUKF (src/VelocityUKF.hpp:33-62): 4-DOF {v, z}.
class VelocityUKF {
 public:
  // ---- the reference's nested types (VelocityUKF.hpp:36-39) ----
  struct DVLMeasurement : Measurement<3> {};
  struct GyroMeasurement : Measurement<3> {};
  struct BodyEffortsMeasurement : Measurement<6> {};
  struct PressureMeasurement : Measurement<1> {};
  typedef VelocityState State;
  typedef Matrix<VelocityState::DOF, VelocityState::DOF> Covariance;

  // VelocityUKF(initial_state, state_cov) (VelocityUKF.hpp:42, VelocityUKF.cpp:49-56), batch = 1
  VelocityUKF(const State& initial_state, const Covariance& state_cov, int device = 0) : batch_(1) {
    check_abi();
    check(uwvk_vel_create(1, device, &h_), "uwvk_vel_create");
    guard([&] {
      double x[4];
      initial_state.to_store(x);
      const std::vector<double> P = detail::rowmajor(state_cov);
      check(uwvk_vel_init(h_, x, P.data()), "VelocityUKF");
    });
  }
  // batched: state batch*4 {v, z}, cov batch*16
  VelocityUKF(int64_t batch, const std::vector<double>& state, const std::vector<double>& cov, int device = 0)
      : batch_(batch) {
    check_abi();
    check(uwvk_vel_create(batch, device, &h_), "uwvk_vel_create");
    guard([&] {
      if (state.size() != (size_t)batch * 4 || cov.size() != (size_t)batch * 16)
        throw std::invalid_argument("VelocityUKF: wrong size");
      check(uwvk_vel_init(h_, state.data(), cov.data()), "VelocityUKF");
    });
  }
  VelocityUKF(const VelocityUKF&) = delete;
  VelocityUKF& operator=(const VelocityUKF&) = delete;
  virtual ~VelocityUKF() { uwvk_vel_destroy(h_); }

  int64_t batch() const { return batch_; }
  // setupMotionModel (VelocityUKF.hpp:46, VelocityUKF.cpp:58-77)
  bool setupMotionModel(const UWVParameters& p) {
    const uwvk_uwv_params c = p.to_c();
    return setupMotionModel(c);
  }
  bool setupMotionModel(const uwvk_uwv_params& p) {
    check(uwvk_vel_setup_motion_model(h_, &p), "setupMotionModel");
    return true;
  }
  // setProcessNoiseCovariance [EXT pose_estimation base]: 4x4 shared by the batch
  void setProcessNoiseCovariance(const Covariance& Q) {
    double q[16];
    detail::put_rowmajor(Q, q);
    check(uwvk_vel_set_process_noise(h_, q), "setProcessNoiseCovariance");
  }
  void setProcessNoiseCovariance(const std::array<double, 16>& Q) {
    check(uwvk_vel_set_process_noise(h_, Q.data()), "setProcessNoiseCovariance");
  }
  void predictionStep(double dt) { check(uwvk_vel_predict(h_, dt), "predictionStep"); }

  // ---- reference overloads (VelocityUKF.hpp:49-58), one measurement for every instance ----
  void integrateMeasurement(const GyroMeasurement& m) {
    const std::vector<double> mu = detail::repeat(m.mu, batch_), cov = detail::repeat(detail::rowmajor(m.cov), batch_);
    check(uwvk_vel_set_gyro(h_, mu.data(), cov.data()), "integrateMeasurement(Gyro)");
  }
  void integrateMeasurement(const BodyEffortsMeasurement& m) {
    const std::vector<double> mu = detail::repeat(m.mu, batch_), cov = detail::repeat(detail::rowmajor(m.cov), batch_);
    check(uwvk_vel_set_efforts(h_, mu.data(), cov.data()), "integrateMeasurement(BodyEfforts)");
  }
  void integrateMeasurement(const DVLMeasurement& m) {
    const std::vector<double> mu = detail::repeat(m.mu, batch_);
    double cov[9];
    detail::put_rowmajor(m.cov, cov);
    check(uwvk_vel_update_dvl(h_, mu.data(), nullptr, cov, nullptr), "integrateMeasurement(DVL)");
  }
  void integrateMeasurement(const PressureMeasurement& m) {
    const std::vector<double> mu = detail::repeat(m.mu, batch_);
    const double cov[1] = {m.cov(0, 0)};
    check(uwvk_vel_update_pressure(h_, mu.data(), nullptr, cov, nullptr), "integrateMeasurement(Pressure)");
  }
  bool getCurrentState(State& state, int64_t instance = 0) {
    std::vector<double> x;
    getState(x);
    at(instance);
    state.from_store(&x[(size_t)instance * 4]);
    return true;
  }
  bool getCurrentState(State& state, Covariance& covariance, int64_t instance = 0) {
    std::vector<double> x, P;
    getState(x, &P);
    at(instance);
    state.from_store(&x[(size_t)instance * 4]);
    detail::get_rowmajor(&P[(size_t)instance * 16], covariance);
    return true;
  }

  // ---- batched overloads ----
  void integrateMeasurement(const batch::GyroMeasurement& m) {
    check(uwvk_vel_set_gyro(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()), "integrateMeasurement(Gyro)");
  }
  void integrateMeasurement(const batch::VelBodyEffortsMeasurement& m) {
    check(uwvk_vel_set_efforts(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()),
          "integrateMeasurement(BodyEfforts)");
  }
  void integrateMeasurement(const batch::DVLMeasurement& m) {
    check(uwvk_vel_update_dvl(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(), m.shared_cov.data(),
                              m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(DVL)");
  }
  void integrateMeasurement(const batch::PressureMeasurement& m) {
    check(uwvk_vel_update_pressure(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(), m.shared_cov.data(),
                                   m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(Pressure)");
  }
  void getState(std::vector<double>& x, std::vector<double>* P = nullptr) {
    x.resize((size_t)batch_ * 4);
    if (P) P->resize((size_t)batch_ * 16);
    check(uwvk_vel_get_state(h_, x.data(), P ? P->data() : nullptr), "getState");
  }
  // inherited getters [EXT] (VelocityUKF.cpp:70), batched
  bool getCurrentState(std::vector<double>& state) {
    getState(state);
    return true;
  }
  bool getCurrentState(std::vector<double>& state, std::vector<double>& covariance) {
    getState(state, &covariance);
    return true;
  }
  std::vector<double> mu() {
    std::vector<double> x;
    getState(x);
    return x;
  }
  std::vector<double> sigma() {
    std::vector<double> x, P;
    getState(x, &P);
    return P;
  }

 private:
  template <class F>
  void guard(F f) {
    try {
      f();
    } catch (...) {
      uwvk_vel_destroy(h_);
      h_ = nullptr;
      throw;
    }
  }
  void at(int64_t instance) const {
    if (instance < 0 || instance >= batch_) throw std::out_of_range("getCurrentState: instance");
  }
  int64_t batch_;
  uwvk_vel* h_ = nullptr;
};

#if UWVK_FACADE_EIGEN
// Eigen copies of a batched object's state (dynamic sizes)
inline Eigen::VectorXd state_eigen(PoseUKF& f) {
  const std::vector<double> x = f.mu();
  return Eigen::Map<const Eigen::VectorXd>(x.data(), (Eigen::Index)x.size());
}
inline Eigen::MatrixXd covariance_eigen(PoseUKF& f) {
  const std::vector<double> P = f.sigma();
  const Eigen::Index n = f.dof();
  return Eigen::Map<const Eigen::Matrix<double, Eigen::Dynamic, Eigen::Dynamic, Eigen::RowMajor>>(P.data(), n, n);
}
#endif

}  // namespace uwv_kalman_filters_amd
