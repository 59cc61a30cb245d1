// PoseUKF.hpp — C++ host facade over the batched C ABI (include/uwvk.h).
//
// Mirrors the reference's class interface (src/PoseUKF.hpp:40-205,
// src/VelocityUKF.hpp:33-62): same method names and argument meaning, but each
// object owns a BATCH of independent filters resident on one gfx950 device, so
// every measurement carries one row per instance.  Errors the reference reports
// by throwing (NaN measurements, non-PD covariance, no motion model) throw
// std::runtime_error here as well (uwvk::Error carries the uwvk_status).
//
// Header-only; link with libuwvk.so.  No Eigen / HIP types in the interface.
#pragma once
#include <array>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/uwvk.h"

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
// CameraConfiguration (PoseUKFConfig.hpp:125-131)
struct CameraConfiguration {
  double fx = 0, fy = 0, cx = 0, cy = 0;
};
// Affine3d stand-in: translation + quaternion (w, x, y, z)
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
  VisualPack(int64_t batch, const std::vector<VisualFeatureMeasurement>& f,
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
          for (int k = 0; k < 4; k++)
            fcov[(b * nf + i) * 4 + k] = f[i].cov.empty() ? f[i].shared_cov[k] : f[i].cov.at(b * 4 + k);
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
}  // namespace detail

using PoseUKFConfig = uwvk_pose_config;
using UWVParameters = uwvk_uwv_params;
using LocationConfiguration = uwvk_location;
using PoseUKFParameter = uwvk_pose_parameter;

class PoseUKF {
 public:
  // PoseUKF(imu_in_nwu_pos, pos_cov, rot, rot_cov, config, model, imu_in_body)
  // (PoseUKF.hpp:100-103): per instance pos[3], pos_cov[9], rot[4] (w,x,y,z), rot_cov[9].
  PoseUKF(int64_t batch, const std::vector<double>& pos, const std::vector<double>& pos_cov,
          const std::vector<double>& rot, const std::vector<double>& rot_cov, const PoseUKFConfig& cfg,
          const UWVParameters& model, const double* imu_in_body = nullptr, int dof = 53, int device = 0)
      : h_(create(batch, dof, device)) {
    need(pos, 3, "pos"); need(pos_cov, 9, "pos_cov"); need(rot, 4, "rot"); need(rot_cov, 9, "rot_cov");
    check(uwvk_pose_init_from_config(h_, pos.data(), pos_cov.data(), rot.data(), rot_cov.data(), &cfg, &model,
                                     imu_in_body),
          "PoseUKF");
  }
  // PoseUKF(state, cov, location, model, filter_parameter) (PoseUKF.hpp:113-115)
  PoseUKF(int64_t batch, const std::vector<double>& state, const std::vector<double>& cov,
          const LocationConfiguration& location, const UWVParameters& model, const PoseUKFParameter& param,
          int dof = 53, int device = 0)
      : h_(create(batch, dof, device)) {
    need(state, store(), "state"); need(cov, (size_t)dof * dof, "cov");
    check(uwvk_pose_init_from_state(h_, state.data(), cov.data(), &location, &model, &param), "PoseUKF");
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
                                 const double* q_imu_in_body = nullptr) {
    check(uwvk_pose_set_process_noise_from_config(h_, &cfg, imu_delta_t, q_imu_in_body),
          "setProcessNoiseFromConfig");
  }
  // setProcessNoiseCovariance [EXT pose_estimation base]
  void setProcessNoiseCovariance(const std::vector<double>& Q) {
    if (Q.size() != (size_t)dof() * dof()) throw std::invalid_argument("setProcessNoiseCovariance: size");
    check(uwvk_pose_set_process_noise(h_, Q.data()), "setProcessNoiseCovariance");
  }
  // predictionStep(dt) [EXT base] -> predictionStepImpl (PoseUKF.cpp:446-474)
  void predictionStep(double delta_t) { check(uwvk_pose_predict(h_, delta_t), "predictionStep"); }

  void integrateMeasurement(const RotationRate& m) {
    need(m.mu, 3, "RotationRate");
    check(uwvk_pose_set_rotation_rate(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()),
          "integrateMeasurement(RotationRate)");
  }
  void integrateMeasurement(const Acceleration& m) { upd(m, uwvk_pose_update_acceleration, "Acceleration"); }
  void integrateMeasurement(const Velocity& m) { upd(m, uwvk_pose_update_velocity, "Velocity"); }
  void integrateMeasurement(const XY_Position& m) { upd(m, uwvk_pose_update_xy, "XY_Position"); }
  void integrateMeasurement(const Z_Position& m) { upd(m, uwvk_pose_update_z, "Z_Position"); }
  void integrateMeasurement(const Pressure& m, const std::array<double, 3>& pressure_sensor_in_imu = {}) {
    prep(m, "Pressure");
    check(uwvk_pose_update_pressure(h_, m.mu.data(), covp(m), m.shared_cov.data(), pressure_sensor_in_imu.data(),
                                    maskp(m), acc()),
          "integrateMeasurement(Pressure)");
  }
  void integrateMeasurement(const GeographicPosition& m, const std::array<double, 3>& gps_in_body = {}) {
    prep(m, "GeographicPosition");
    check(uwvk_pose_update_geographic(h_, m.mu.data(), covp(m), m.shared_cov.data(), gps_in_body.data(),
                                      maskp(m), acc()),
          "integrateMeasurement(GeographicPosition)");
  }
  void integrateMeasurement(const BodyEffortsMeasurement& m, bool only_affect_velocity = false) {
    prep(m, "BodyEffortsMeasurement");
    check(uwvk_pose_update_efforts(h_, m.mu.data(), covp(m), m.shared_cov.data(), only_affect_velocity ? 1 : 0,
                                   maskp(m), acc()),
          "integrateMeasurement(BodyEffortsMeasurement)");
  }
  // cell_weighting: one value per instance, or a single value for all
  void integrateMeasurement(const WaterVelocityMeasurement& m, const std::vector<double>& cell_weighting) {
    prep(m, "WaterVelocityMeasurement");
    std::vector<double> w = cell_weighting.size() == 1 ? std::vector<double>((size_t)batch(), cell_weighting[0])
                                                       : cell_weighting;
    need(w, 1, "cell_weighting");
    check(uwvk_pose_update_water_velocity(h_, m.mu.data(), covp(m), m.shared_cov.data(), w.data(), maskp(m),
                                          acc()),
          "integrateMeasurement(WaterVelocityMeasurement)");
  }
  void integrateMeasurement(double cell_weighting, const WaterVelocityMeasurement& m) {
    integrateMeasurement(m, std::vector<double>{cell_weighting});
  }
  // integrateDelayedPositionMeasurement (PoseUKF.hpp:143): delayed_position batch*2
  void integrateDelayedPositionMeasurement(const XY_Position& m, const std::vector<double>& delayed_position) {
    prep(m, "XY_Position");
    need(delayed_position, 2, "delayed_position");
    check(uwvk_pose_update_delayed_xy(h_, m.mu.data(), covp(m), m.shared_cov.data(), delayed_position.data(),
                                      maskp(m), acc()),
          "integrateDelayedPositionMeasurement");
  }
  // integrateMeasurement(marker_features, feature_positions, marker_pose, cov_marker_pose,
  // camera_config, camera_in_IMU) (PoseUKF.hpp:174-177, PoseUKF.cpp:613-654).
  // marker_pose: one pose shared by the batch, or one per instance.
  void integrateMeasurement(const std::vector<VisualFeatureMeasurement>& marker_features,
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
  // resetFilterWithExternalPose (PoseUKF.hpp:187): per instance {tx,ty,tz,qw,qx,qy,qz}
  void resetFilterWithExternalPose(const std::vector<double>& imu_in_nav) {
    need(imu_in_nav, 7, "imu_in_nav");
    check(uwvk_pose_reset_with_external_pose(h_, imu_in_nav.data()), "resetFilterWithExternalPose");
  }
  // getRotationRate (PoseUKF.hpp:190): batch*3
  std::vector<double> getRotationRate() {
    std::vector<double> w((size_t)batch() * 3);
    check(uwvk_pose_get_rotation_rate(h_, w.data()), "getRotationRate");
    return w;
  }
  // batch*store (x) and batch*dof*dof (P, full symmetric)
  void getState(std::vector<double>& x, std::vector<double>* P = nullptr) {
    x.resize((size_t)batch() * store());
    if (P) P->resize((size_t)batch() * dof() * dof());
    check(uwvk_pose_get_state(h_, x.data(), P ? P->data() : nullptr), "getState");
  }
  // The inherited getters of pose_estimation::UnscentedKalmanFilter<State> [EXT]
  // (used at VelocityUKF.cpp:70: `if (getCurrentState(current_state))`) and the
  // ukf's mu() / sigma() (PoseUKF.cpp:448,453,516): true once initialised.
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
  // alone on k_pose_efforts_epoch; UWVK_OPT_DENSE_SIGMA: one literal launch per epoch.
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
  void need(const std::vector<double>& v, size_t per, const char* what) const {
    if (v.size() != (size_t)batch() * per) throw std::invalid_argument(std::string(what) + ": wrong size");
  }
  template <int M>
  void prep(const BatchMeasurement<M>& m, const char* what) {
    need(m.mu, M, what);
    if (!m.cov.empty()) need(m.cov, (size_t)M * M, what);
    if (!m.mask.empty() && m.mask.size() != (size_t)batch()) throw std::invalid_argument("mask: wrong size");
  }
  template <int M>
  static const double* covp(const BatchMeasurement<M>& m) { return m.cov.empty() ? nullptr : m.cov.data(); }
  template <int M>
  static const uint8_t* maskp(const BatchMeasurement<M>& m) { return m.mask.empty() ? nullptr : m.mask.data(); }
  uint8_t* acc() {
    accepted_.assign((size_t)batch(), 0);
    return accepted_.data();
  }
  template <int M, class F>
  void upd(const BatchMeasurement<M>& m, F fn, const char* what) {
    prep(m, what);
    check(fn(h_, m.mu.data(), covp(m), m.shared_cov.data(), maskp(m), acc()),
          (std::string("integrateMeasurement(") + what + ")").c_str());
  }

  uwvk_pose* h_ = nullptr;
  std::vector<uint8_t> accepted_;
};

// VelocityUKF (src/VelocityUKF.hpp:33-62): 4-DOF {v, z}, one filter per lane.
struct DVLMeasurement : BatchMeasurement<3> {};
struct GyroMeasurement : BatchMeasurement<3> {};
struct VelBodyEffortsMeasurement : BatchMeasurement<6> {};
struct PressureMeasurement : BatchMeasurement<1> {};

class VelocityUKF {
 public:
  VelocityUKF(int64_t batch, const std::vector<double>& state, const std::vector<double>& cov, int device = 0)
      : batch_(batch) {
    check_abi();
    check(uwvk_vel_create(batch, device, &h_), "uwvk_vel_create");
    if (state.size() != (size_t)batch * 4 || cov.size() != (size_t)batch * 16) {
      uwvk_vel_destroy(h_);
      throw std::invalid_argument("VelocityUKF: wrong size");
    }
    check(uwvk_vel_init(h_, state.data(), cov.data()), "VelocityUKF");
  }
  VelocityUKF(const VelocityUKF&) = delete;
  VelocityUKF& operator=(const VelocityUKF&) = delete;
  virtual ~VelocityUKF() { uwvk_vel_destroy(h_); }

  void setupMotionModel(const UWVParameters& p) { check(uwvk_vel_setup_motion_model(h_, &p), "setupMotionModel"); }
  // setProcessNoiseCovariance [EXT pose_estimation base]: 4x4 shared by the batch
  void setProcessNoiseCovariance(const std::array<double, 16>& Q) {
    check(uwvk_vel_set_process_noise(h_, Q.data()), "setProcessNoiseCovariance");
  }
  void predictionStep(double dt) { check(uwvk_vel_predict(h_, dt), "predictionStep"); }
  void integrateMeasurement(const GyroMeasurement& m) {
    check(uwvk_vel_set_gyro(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()), "integrateMeasurement(Gyro)");
  }
  void integrateMeasurement(const VelBodyEffortsMeasurement& m) {
    check(uwvk_vel_set_efforts(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data()),
          "integrateMeasurement(BodyEfforts)");
  }
  void integrateMeasurement(const DVLMeasurement& m) {
    check(uwvk_vel_update_dvl(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(), m.shared_cov.data(),
                              m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(DVL)");
  }
  void integrateMeasurement(const PressureMeasurement& m) {
    check(uwvk_vel_update_pressure(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(), m.shared_cov.data(),
                                   m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(Pressure)");
  }
  void getState(std::vector<double>& x, std::vector<double>* P = nullptr) {
    x.resize((size_t)batch_ * 4);
    if (P) P->resize((size_t)batch_ * 16);
    check(uwvk_vel_get_state(h_, x.data(), P ? P->data() : nullptr), "getState");
  }
  // inherited getters [EXT] (VelocityUKF.cpp:70)
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
  int64_t batch_;
  uwvk_vel* h_ = nullptr;
};

#if __has_include(<Eigen/Core>)
}  // namespace uwv_kalman_filters_amd
#include <Eigen/Core>
namespace uwv_kalman_filters_amd {
// Eigen overloads for the single-instance (batch = 1) drop-in: the reference's
// MEASUREMENT types carry Eigen .mu / .cov (PoseUKF.hpp:79-88).  Eigen is not
// installed in the build image, so this block is compiled only where it is.
template <class Meas, int M>
Meas from_eigen(const Eigen::Matrix<double, M, 1>& mu, const Eigen::Matrix<double, M, M>& cov) {
  Meas m;
  m.mu.assign(mu.data(), mu.data() + M);
  m.cov.resize((size_t)M * M);
  for (int r = 0; r < M; r++)
    for (int c = 0; c < M; c++) m.cov[(size_t)r * M + c] = cov(r, c);  // row-major in the C ABI
  return m;
}
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
