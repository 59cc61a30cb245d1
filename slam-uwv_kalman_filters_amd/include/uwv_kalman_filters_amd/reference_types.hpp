// reference_types.hpp — the reference's value types, for its single-filter call forms.
//
// A caller written against the reference's headers builds these objects and
// hands them to the facade classes (PoseUKF.hpp): the MEASUREMENT types
// (pose_estimation/Measurement.hpp [EXT], used at PoseUKF.hpp:79-88 and
// VelocityUKF.hpp:36-39), the PoseState / VelocityState manifolds
// (PoseState.hpp:29-45, VelocityUKF.hpp:24-27), PoseUKFConfig and its parts
// (PoseUKFConfig.hpp:20-194) and uwv_dynamic_model::UWVParameters [EXT] (the
// fields PoseUKF.cpp:159-171 / :303-318 and VelocityUKF.cpp:58-77 read).  Each
// converts to the C ABI's POD (include/uwvk.h) with to_c().  The vector and
// matrix types are Eigen's where Eigen is installed (linalg.hpp).
#pragma once
#include <string>
#include <vector>

#include "../../../include/uwvk.h"
#include "linalg.hpp"

namespace uwv_kalman_filters_amd {

// MEASUREMENT(Name, M) [EXT pose_estimation]: one measurement of one filter.
template <int M>
struct Measurement {
  enum { DOF = M };
  typedef Matrix<M, 1> Mu;
  typedef Matrix<M, M> Cov;
  Mu mu;
  Cov cov;
};

// ---- PoseUKFConfig.hpp:20-194 ----------------------------------------------
struct WaterVelocityParameters {  // :20-48
  double tau = 0;
  double limits = 0;
  Vector3d measurement_std = Vector3d::Zero();
  double scale = 0;
  double cell_size = 0;
  double first_cell_blank = 0;
  double minimum_correlation = 0;
  double adcp_bias_tau = 0;
  double adcp_bias_limits = 0;
};

struct InertialNoiseParameters {  // :50-63
  Vector3d randomwalk = Vector3d::Zero();
  Vector3d bias_offset = Vector3d::Zero();
  Vector3d bias_instability = Vector3d::Zero();
  double bias_tau = 0;
};

struct DynamicModelNoiseParameters {  // :65-97
  Vector6d body_efforts_std = Vector6d::Zero();
  VectorXd inertia_instability = VectorXd::Zero(9);
  VectorXd lin_damping_instability = VectorXd::Zero(9);
  VectorXd quad_damping_instability = VectorXd::Zero(9);
  double inertia_tau = 0;
  double lin_damping_tau = 0;
  double quad_damping_tau = 0;
};

using LocationConfiguration = uwvk_location;  // :99-109 (latitude, longitude, altitude)

struct VisualLandmark {  // :111-123
  std::string marker_id;
  double marker_size = 0;
  Vector3d marker_position = Vector3d::Zero();
  Vector3d marker_euler_orientation = Vector3d::Zero();
  Vector6d marker_pose_std = Vector6d::Zero();
};

struct CameraConfiguration {  // :125-131
  double fx = 0, fy = 0, cx = 0, cy = 0;
};

struct VisualLandmarkConfiguration {  // :133-143
  CameraConfiguration camera_config;
  Vector2d feature_std = Vector2d::Zero();
  std::vector<Vector3d> unit_feature_positions;
  std::vector<VisualLandmark> landmarks;
};

struct HydrostaticConfiguration {  // :145-157
  double water_density = 0;
  double water_density_limits = 0;
  double water_density_tau = 0;
  double atmospheric_pressure = 0;
  double pressure_std = 0;
};

namespace detail {
template <class V>
void put_vec(const V& v, double* out, int n, const char* what) {
  if ((int)v.size() != n) throw std::invalid_argument(std::string(what) + ": expected " + std::to_string(n) + " values");
  for (int i = 0; i < n; i++) out[i] = v(i);
}
}  // namespace detail

struct PoseUKFConfig {  // :159-194
  InertialNoiseParameters acceleration;
  InertialNoiseParameters rotation_rate;
  DynamicModelNoiseParameters model_noise_parameters;
  WaterVelocityParameters water_velocity;
  LocationConfiguration location{0, 0, 0};
  VisualLandmarkConfiguration visual_landmarks;  // used per call (the visual update's arguments)
  HydrostaticConfiguration hydrostatics;
  Vector3d max_jerk = Vector3d::Zero();
  Vector6d max_effort = Vector6d::Zero();
  double dynamic_model_min_depth = 0;

  uwvk_pose_config to_c() const {
    uwvk_pose_config c{};
    auto inertial = [](const InertialNoiseParameters& p, uwvk_inertial_noise& o) {
      detail::put_vec(p.randomwalk, o.randomwalk, 3, "randomwalk");
      detail::put_vec(p.bias_offset, o.bias_offset, 3, "bias_offset");
      detail::put_vec(p.bias_instability, o.bias_instability, 3, "bias_instability");
      o.bias_tau = p.bias_tau;
    };
    inertial(acceleration, c.acceleration);
    inertial(rotation_rate, c.rotation_rate);
    const DynamicModelNoiseParameters& m = model_noise_parameters;
    detail::put_vec(m.body_efforts_std, c.model_noise_parameters.body_efforts_std, 6, "body_efforts_std");
    detail::put_vec(m.inertia_instability, c.model_noise_parameters.inertia_instability, 9, "inertia_instability");
    detail::put_vec(m.lin_damping_instability, c.model_noise_parameters.lin_damping_instability, 9,
                    "lin_damping_instability");
    detail::put_vec(m.quad_damping_instability, c.model_noise_parameters.quad_damping_instability, 9,
                    "quad_damping_instability");
    c.model_noise_parameters.inertia_tau = m.inertia_tau;
    c.model_noise_parameters.lin_damping_tau = m.lin_damping_tau;
    c.model_noise_parameters.quad_damping_tau = m.quad_damping_tau;
    const WaterVelocityParameters& w = water_velocity;
    c.water_velocity.tau = w.tau;
    c.water_velocity.limits = w.limits;
    detail::put_vec(w.measurement_std, c.water_velocity.measurement_std, 3, "measurement_std");
    c.water_velocity.scale = w.scale;
    c.water_velocity.cell_size = w.cell_size;
    c.water_velocity.first_cell_blank = w.first_cell_blank;
    c.water_velocity.minimum_correlation = w.minimum_correlation;
    c.water_velocity.adcp_bias_tau = w.adcp_bias_tau;
    c.water_velocity.adcp_bias_limits = w.adcp_bias_limits;
    c.location = location;
    c.hydrostatics = {hydrostatics.water_density, hydrostatics.water_density_limits, hydrostatics.water_density_tau,
                      hydrostatics.atmospheric_pressure, hydrostatics.pressure_std};
    detail::put_vec(max_jerk, c.max_jerk, 3, "max_jerk");
    detail::put_vec(max_effort, c.max_effort, 6, "max_effort");
    c.dynamic_model_min_depth = dynamic_model_min_depth;
    return c;
  }
};

// [EXT] uwv_dynamic_model::UWVParameters: the fields the filters read.
struct UWVParameters {
  Matrix6d inertia_matrix = Matrix6d::Zero();
  std::vector<Matrix6d> damping_matrices = std::vector<Matrix6d>(2, Matrix6d::Zero());  // [0] linear, [1] quadratic
  double weight = 0;
  double buoyancy = 0;
  Vector3d distance_body2centerofgravity = Vector3d::Zero();
  Vector3d distance_body2centerofbuoyancy = Vector3d::Zero();

  uwvk_uwv_params to_c() const {
    if (damping_matrices.size() < 2)
      throw std::invalid_argument("UWVParameters: damping_matrices needs the linear and quadratic matrices");
    uwvk_uwv_params p{};
    detail::put_rowmajor(inertia_matrix, p.inertia_matrix);
    detail::put_rowmajor(damping_matrices[0], p.damping_matrices[0]);
    detail::put_rowmajor(damping_matrices[1], p.damping_matrices[1]);
    p.weight = weight;
    p.buoyancy = buoyancy;
    for (int k = 0; k < 3; k++) {
      p.distance_body2centerofgravity[k] = distance_body2centerofgravity(k);
      p.distance_body2centerofbuoyancy[k] = distance_body2centerofbuoyancy(k);
    }
    return p;
  }
};

// ---- PoseState.hpp:29-45: the 14 sub-manifolds, 53 DOF ---------------------
struct PoseState {
  enum { DOF = 53 };
  Vector3d position = Vector3d::Zero();
  Quaterniond orientation = Quaterniond::Identity();
  Vector3d velocity = Vector3d::Zero();
  Vector3d acceleration = Vector3d::Zero();
  Vector3d bias_gyro = Vector3d::Zero();
  Vector3d bias_acc = Vector3d::Zero();
  Matrix<1, 1> gravity = Matrix<1, 1>::Zero();
  Matrix3d inertia = Matrix3d::Zero();       // column-major in the vectorized state (PoseState.hpp:37)
  Matrix3d lin_damping = Matrix3d::Zero();
  Matrix3d quad_damping = Matrix3d::Zero();
  Vector2d water_velocity = Vector2d::Zero();
  Vector2d water_velocity_below = Vector2d::Zero();
  Vector2d bias_adcp = Vector2d::Zero();
  Matrix<1, 1> water_density = Matrix<1, 1>::Zero();

  // the C ABI's 54 stored scalars (include/uwvk.h UWVK_S_*)
  void to_store(double* x) const {
    for (int k = 0; k < 3; k++) {
      x[UWVK_S_POS + k] = position(k);
      x[UWVK_S_VEL + k] = velocity(k);
      x[UWVK_S_ACC + k] = acceleration(k);
      x[UWVK_S_BIAS_GYRO + k] = bias_gyro(k);
      x[UWVK_S_BIAS_ACC + k] = bias_acc(k);
    }
    x[UWVK_S_QUAT] = orientation.w(); x[UWVK_S_QUAT + 1] = orientation.x();
    x[UWVK_S_QUAT + 2] = orientation.y(); x[UWVK_S_QUAT + 3] = orientation.z();
    x[UWVK_S_GRAVITY] = gravity(0);
    for (int c = 0; c < 3; c++)
      for (int r = 0; r < 3; r++) {
        x[UWVK_S_INERTIA + 3 * c + r] = inertia(r, c);
        x[UWVK_S_LIN_DAMPING + 3 * c + r] = lin_damping(r, c);
        x[UWVK_S_QUAD_DAMPING + 3 * c + r] = quad_damping(r, c);
      }
    for (int k = 0; k < 2; k++) {
      x[UWVK_S_WATER_VEL + k] = water_velocity(k);
      x[UWVK_S_WATER_VEL_BELOW + k] = water_velocity_below(k);
      x[UWVK_S_BIAS_ADCP + k] = bias_adcp(k);
    }
    x[UWVK_S_WATER_DENSITY] = water_density(0);
  }
  void from_store(const double* x) {
    for (int k = 0; k < 3; k++) {
      position(k) = x[UWVK_S_POS + k];
      velocity(k) = x[UWVK_S_VEL + k];
      acceleration(k) = x[UWVK_S_ACC + k];
      bias_gyro(k) = x[UWVK_S_BIAS_GYRO + k];
      bias_acc(k) = x[UWVK_S_BIAS_ACC + k];
    }
    orientation = Quaterniond(x[UWVK_S_QUAT], x[UWVK_S_QUAT + 1], x[UWVK_S_QUAT + 2], x[UWVK_S_QUAT + 3]);
    gravity(0) = x[UWVK_S_GRAVITY];
    for (int c = 0; c < 3; c++)
      for (int r = 0; r < 3; r++) {
        inertia(r, c) = x[UWVK_S_INERTIA + 3 * c + r];
        lin_damping(r, c) = x[UWVK_S_LIN_DAMPING + 3 * c + r];
        quad_damping(r, c) = x[UWVK_S_QUAD_DAMPING + 3 * c + r];
      }
    for (int k = 0; k < 2; k++) {
      water_velocity(k) = x[UWVK_S_WATER_VEL + k];
      water_velocity_below(k) = x[UWVK_S_WATER_VEL_BELOW + k];
      bias_adcp(k) = x[UWVK_S_BIAS_ADCP + k];
    }
    water_density(0) = x[UWVK_S_WATER_DENSITY];
  }
};

// ---- VelocityUKF.hpp:24-27: {velocity, z_position}, 4 DOF -------------------
struct VelocityState {
  enum { DOF = 4 };
  Vector3d velocity = Vector3d::Zero();
  Matrix<1, 1> z_position = Matrix<1, 1>::Zero();
  void to_store(double* x) const {
    for (int k = 0; k < 3; k++) x[k] = velocity(k);
    x[3] = z_position(0);
  }
  void from_store(const double* x) {
    for (int k = 0; k < 3; k++) velocity(k) = x[k];
    z_position(0) = x[3];
  }
};

}  // namespace uwv_kalman_filters_amd
