// reference_calls.cpp — a caller written against the REFERENCE's headers and call
// forms only (src/PoseUKF.hpp:46-190, src/VelocityUKF.hpp:33-58,
// src/PoseUKFConfig.hpp:20-194): #include <uwv_kalman_filters/PoseUKF.hpp>,
// namespace uwv_kalman_filters, the batch-1 constructors in the reference's
// parameter order, the nested MEASUREMENT types with .mu / .cov,
// integrateMeasurement(adcp, cell_weighting), resetFilterWithExternalPose(Affine3d),
// getRotationRate(), getCurrentState(State&, Covariance&), VelocityUKF's
// setupMotionModel / BodyEffortsMeasurement.  The value types are the facade's
// Eigen stand-ins (Eigen is not in this image; with Eigen installed the same
// code binds Eigen's types).
//
// Beside it, the CPU oracle (oracle/uwvk_oracle.h, test infrastructure) runs
// the same calls; the GPU results must match it (tests/test_facade.py).
// Exit 0 = parity.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include <uwv_kalman_filters/PoseUKF.hpp>
#include <uwv_kalman_filters/VelocityUKF.hpp>
extern "C" {
#include "../../oracle/uwvk_oracle.h"
}

using namespace uwv_kalman_filters;

static double worst = 0;
static int gate_mismatch = 0;

// the reference-form state against the oracle's, in the oracle's std-devs
static void compare(PoseUKF& f, or_pose* o, const char* where) {
  PoseUKF::State s;
  PoseUKF::Covariance P;
  if (!f.getCurrentState(s, P)) std::exit(3);
  double x[54], xo[54];
  std::vector<double> Po(53 * 53);
  s.to_store(x);
  or_pose_get_state(o, xo, Po.data());
  double w = 0;
  for (int i = 0; i < 53; i++)
    for (int j = 0; j < 53; j++)
      w = std::fmax(w, std::fabs(P(i, j) - Po[i * 53 + j]) / std::sqrt(Po[i * 53 + i] * Po[j * 53 + j]));
  for (int i = 0; i < 54; i++) {
    if (i >= 3 && i < 7) continue;
    const int d = i < 3 ? i : i - 1;
    w = std::fmax(w, std::fabs(x[i] - xo[i]) / std::sqrt(Po[d * 53 + d]));
  }
  // orientation: the angle between the quaternions, 2 |vec(conj(q_o) q)|
  // (well conditioned near 0, unlike acos of the dot product), in the
  // orientation std-dev
  const double* q = x + 3;
  const double* r = xo + 3;
  const double vx = r[0] * q[1] - r[1] * q[0] - r[2] * q[3] + r[3] * q[2];
  const double vy = r[0] * q[2] + r[1] * q[3] - r[2] * q[0] - r[3] * q[1];
  const double vz = r[0] * q[3] - r[1] * q[2] + r[2] * q[1] - r[3] * q[0];
  const double ang = 2 * std::sqrt(vx * vx + vy * vy + vz * vz);
  w = std::fmax(w, ang / std::sqrt(std::fmin(Po[3 * 53 + 3], std::fmin(Po[4 * 53 + 4], Po[5 * 53 + 5]))));
  std::printf("%-28s worst %.3e\n", where, w);
  worst = std::fmax(worst, w);
}

template <class M>
static void gate(PoseUKF& f, int acc) {
  (void)sizeof(M);
  gate_mismatch += (acc != 0) != (f.lastAccepted().at(0) != 0);
}

int main() {
  const double dt = 1e-3;
  // ---- PoseUKFConfig, written as the reference's configuration code would ----
  PoseUKFConfig config;
  config.acceleration.randomwalk = Vector3d(1e-3, 1e-3, 1e-3);
  config.acceleration.bias_instability = Vector3d(1e-4, 1e-4, 1e-4);
  config.acceleration.bias_tau = 600;
  config.rotation_rate.randomwalk = Vector3d(1e-4, 1e-4, 1e-4);
  config.rotation_rate.bias_instability = Vector3d(1e-5, 1e-5, 1e-5);
  config.rotation_rate.bias_offset = Vector3d(1e-6, -2e-6, 0.5e-6);
  config.rotation_rate.bias_tau = 600;
  config.model_noise_parameters.body_efforts_std << 5, 5, 5, 1, 1, 1;
  config.model_noise_parameters.inertia_instability = VectorXd::Constant(9, 10);
  config.model_noise_parameters.lin_damping_instability = VectorXd::Constant(9, 5);
  config.model_noise_parameters.quad_damping_instability = VectorXd::Constant(9, 5);
  config.model_noise_parameters.inertia_tau = 3600;
  config.model_noise_parameters.lin_damping_tau = 3600;
  config.model_noise_parameters.quad_damping_tau = 3600;
  config.water_velocity.tau = 900;
  config.water_velocity.limits = 0.1;
  config.water_velocity.scale = 1e-3;
  config.water_velocity.measurement_std = Vector3d(0.05, 0.05, 0.05);
  config.water_velocity.adcp_bias_tau = 900;
  config.water_velocity.adcp_bias_limits = 0.05;
  config.location.latitude = 0.9;
  config.location.longitude = 0.15;
  config.location.altitude = 0.0;
  config.hydrostatics.water_density = 1025;
  config.hydrostatics.water_density_limits = 2;
  config.hydrostatics.water_density_tau = 3600;
  config.hydrostatics.atmospheric_pressure = 101325;
  config.hydrostatics.pressure_std = 100;
  config.max_jerk = Vector3d(0.5, 0.5, 0.5);
  config.max_effort << 100, 100, 100, 20, 20, 20;

  // ---- uwv_dynamic_model::UWVParameters ----
  uwv_dynamic_model::UWVParameters model;
  Vector6d Md, Dl, Dq;
  Md << 200, 250, 300, 20, 30, 30;
  Dl << 20, 30, 40, 5, 5, 5;
  Dq << 50, 80, 100, 10, 10, 10;
  model.inertia_matrix = Md.asDiagonal();
  model.damping_matrices[0] = Dl.asDiagonal();
  model.damping_matrices[1] = Dq.asDiagonal();
  model.weight = 2000;
  model.buoyancy = 2000;
  model.distance_body2centerofbuoyancy = Vector3d(0, 0, 0.05);

  // ---- PoseUKF(imu_in_nwu_pos, pos_cov, rot, rot_cov, config, model, imu_in_body) ----
  const Vector3d pos(1.5, -2.0, -3.0);
  const Matrix3d pos_cov = Matrix3d::Identity() * 0.1;
  const Quaterniond rot = Quaterniond(AngleAxisd(0.3, Vector3d::UnitZ())) * Quaterniond(AngleAxisd(0.02, Vector3d::UnitX()));
  const Matrix3d rot_cov = Matrix3d::Identity() * 1e-3;
  Affine3d imu_in_body = Affine3d::Identity();
  imu_in_body.translation() = Vector3d(0.1, 0.0, -0.2);
  PoseUKF filter(pos, pos_cov, rot, rot_cov, config, model, imu_in_body);
  filter.setProcessNoiseFromConfig(config, dt);

  const uwvk_pose_config cfg = config.to_c();
  const uwvk_uwv_params uwv = model.to_c();
  or_pose* o = (or_pose*)calloc(1, or_pose_sizeof());
  {
    const double p3[3] = {pos.x(), pos.y(), pos.z()}, q4[4] = {rot.w(), rot.x(), rot.y(), rot.z()};
    double pc[9], rc[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) pc[i * 3 + j] = pos_cov(i, j), rc[i * 3 + j] = rot_cov(i, j);
    const double ib[7] = {0.1, 0.0, -0.2, 1, 0, 0, 0};
    or_pose_init_from_config(o, 53, p3, pc, q4, rc, &cfg, &uwv, ib);
    or_pose_set_process_noise_from_config(o, &cfg, dt, nullptr);
  }
  compare(filter, o, "constructor");

  std::mt19937_64 rng(11);
  std::normal_distribution<double> n01;
  PoseUKF::RotationRate rotation_rate;
  PoseUKF::Acceleration acceleration;
  PoseUKF::Velocity velocity;
  PoseUKF::Pressure pressure;
  PoseUKF::WaterVelocityMeasurement adcp;
  PoseUKF::BodyEffortsMeasurement efforts;
  PoseUKF::XY_Position xy;
  PoseUKF::Z_Position z;
  PoseUKF::GeographicPosition geo;
  rotation_rate.cov = Matrix3d::Identity() * 1e-8;
  acceleration.cov = Matrix3d::Identity() * 1e-4;
  velocity.cov = Matrix3d::Identity() * 1e-4;
  pressure.cov << 1e4;
  adcp.cov = Matrix2d::Identity() * 4e-3;
  efforts.cov = Matrix6d::Identity() * 25.0;
  xy.cov = Matrix2d::Identity() * 0.25;
  z.cov << 0.04;
  geo.cov = Matrix2d::Identity() * 4.0;
  const Vector3d pressure_sensor_in_imu(0.0, 0.05, 0.1);

  auto epoch = [&](int e) {
    int acc = 0;
    rotation_rate.mu = Vector3d(0.01 * n01(rng), 0.01 * n01(rng), 0.02 + 0.01 * n01(rng));
    acceleration.mu = Vector3d(0.02 * n01(rng), 0.02 * n01(rng), 9.81 + 0.02 * n01(rng));
    filter.integrateMeasurement(rotation_rate);
    filter.predictionStep(dt);
    filter.integrateMeasurement(acceleration);
    double m9[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) m9[i * 3 + j] = rotation_rate.cov(i, j);
    or_pose_set_rotation_rate(o, rotation_rate.mu.data(), m9);
    or_pose_predict(o, dt);
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) m9[i * 3 + j] = acceleration.cov(i, j);
    or_pose_update_acceleration(o, acceleration.mu.data(), m9, &acc);
    if (e % 50 == 49) {
      velocity.mu = Vector3d(0.5 + 0.05 * n01(rng), 0.05 * n01(rng), 0.05 * n01(rng));
      filter.integrateMeasurement(velocity);
      for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) m9[i * 3 + j] = velocity.cov(i, j);
      or_pose_update_velocity(o, velocity.mu.data(), m9, &acc);
      gate<PoseUKF::Velocity>(filter, acc);
    }
    if (e % 100 == 99) {
      pressure.mu << 101325 + 1025 * 9.81 * 3.0 + 50 * n01(rng);
      filter.integrateMeasurement(pressure, pressure_sensor_in_imu);
      const double c1[1] = {pressure.cov(0, 0)};
      or_pose_update_pressure(o, pressure.mu.data(), c1, pressure_sensor_in_imu.data(), &acc);
      gate<PoseUKF::Pressure>(filter, acc);
    }
    if (e % 120 == 119) {  // ADCP, the reference's (measurement, cell_weighting) form
      adcp.mu = Vector2d(0.05 * n01(rng), 0.05 * n01(rng));
      filter.integrateMeasurement(adcp, 0.5);
      const double c4[4] = {adcp.cov(0, 0), adcp.cov(0, 1), adcp.cov(1, 0), adcp.cov(1, 1)};
      or_pose_update_water_velocity(o, adcp.mu.data(), c4, 0.5, &acc);
      gate<PoseUKF::WaterVelocityMeasurement>(filter, acc);
    }
    if (e == 150 || e == 250) {  // BodyEfforts: constrainVelocity, then the full model
      efforts.mu << 5 * n01(rng), 5 * n01(rng), 5 * n01(rng), n01(rng), n01(rng), n01(rng);
      const bool only_affect_velocity = e == 150;
      filter.integrateMeasurement(efforts, only_affect_velocity);
      double c36[36];
      for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) c36[i * 6 + j] = efforts.cov(i, j);
      or_pose_update_efforts(o, efforts.mu.data(), c36, only_affect_velocity ? 1 : 0, &acc);
    }
    if (e == 300) {
      xy.mu = Vector2d(1.5 + 0.3 * n01(rng), -2.0 + 0.3 * n01(rng));
      filter.integrateMeasurement(xy);
      const double c4[4] = {xy.cov(0, 0), 0, 0, xy.cov(1, 1)};
      or_pose_update_xy(o, xy.mu.data(), c4, &acc);
      gate<PoseUKF::XY_Position>(filter, acc);
    }
    if (e == 330) {
      z.mu << -3.0 + 0.1 * n01(rng);
      filter.integrateMeasurement(z);
      const double c1[1] = {z.cov(0, 0)};
      or_pose_update_z(o, z.mu.data(), c1, &acc);
      gate<PoseUKF::Z_Position>(filter, acc);
    }
    if (e == 360) {  // WGS-84 latitude / longitude of the filter's position, perturbed
      geo.mu = Vector2d(0.9 + 1.5 / 6.37e6 + 2e-7 * n01(rng), 0.15 + 2e-7 * n01(rng));
      const Vector3d gps_in_body(0.0, 0.0, 0.5);
      filter.integrateMeasurement(geo, gps_in_body);
      const double c4[4] = {geo.cov(0, 0), 0, 0, geo.cov(1, 1)};
      or_pose_update_geographic(o, geo.mu.data(), c4, gps_in_body.data(), &acc);
      gate<PoseUKF::GeographicPosition>(filter, acc);
    }
    if (e == 390) {
      xy.mu = Vector2d(1.5 + 0.3 * n01(rng), -2.0 + 0.3 * n01(rng));
      const Vector2d delayed_position(1.45, -2.02);
      filter.integrateDelayedPositionMeasurement(xy, delayed_position);
      const double c4[4] = {xy.cov(0, 0), 0, 0, xy.cov(1, 1)};
      or_pose_update_delayed_xy(o, xy.mu.data(), c4, delayed_position.data(), &acc);
      gate<PoseUKF::XY_Position>(filter, acc);
    }
  };
  for (int e = 0; e < 400; e++) epoch(e);
  compare(filter, o, "400 epochs");

  // getRotationRate (PoseUKF.hpp:190)
  {
    const PoseUKF::RotationRate::Mu w = filter.getRotationRate();
    double wo[3];
    or_pose_get_rotation_rate(o, wo);
    double d = 0;
    for (int k = 0; k < 3; k++) d = std::fmax(d, std::fabs(w(k) - wo[k]));
    std::printf("%-28s |dw| %.3e\n", "getRotationRate", d);
    if (!(d < 1e-12)) worst = 1;
  }

  // the visual-marker update: four corners of a marker 3 m ahead, projected
  {
    PoseUKF::State s;
    filter.getCurrentState(s);
    CameraConfiguration camera_config;
    camera_config.fx = 600; camera_config.fy = 620; camera_config.cx = 320; camera_config.cy = 240;
    Affine3d camera_in_IMU(Quaterniond(0.5, -0.5, 0.5, -0.5));  // z_cam = x_imu
    camera_in_IMU.translation() = Vector3d(0.1, 0.0, 0.05);
    Affine3d marker_pose(s.orientation);
    marker_pose.translation() = s.position + s.orientation * Vector3d(3.0, 0.0, 0.0);
    const std::vector<Vector3d> feature_positions = {Vector3d(0.2, 0.2, 0), Vector3d(-0.2, 0.2, 0),
                                                     Vector3d(-0.2, -0.2, 0), Vector3d(0.2, -0.2, 0)};
    std::vector<PoseUKF::VisualFeatureMeasurement> features(4);
    const Affine3d cam_in_nav = Affine3d(s.orientation).pretranslate(s.position) * camera_in_IMU;
    for (int i = 0; i < 4; i++) {
      const Vector3d pc = cam_in_nav.inverse() * (marker_pose * feature_positions[i]);
      features[i].mu = Vector2d(camera_config.fx * pc.x() / pc.z() + camera_config.cx + 0.3 * n01(rng),
                                camera_config.fy * pc.y() / pc.z() + camera_config.cy + 0.3 * n01(rng));
      features[i].cov = Matrix2d::Identity() * 0.09;
    }
    Matrix<6, 6> cov_marker_pose = Matrix<6, 6>::Identity() * 1e-4;
    filter.integrateMeasurement(features, feature_positions, marker_pose, cov_marker_pose, camera_config,
                                camera_in_IMU);
    double ft[8], fc[16], fp[12], mp[7], cm[36], cin[7];
    for (int i = 0; i < 4; i++) {
      ft[i * 2] = features[i].mu(0); ft[i * 2 + 1] = features[i].mu(1);
      fc[i * 4] = 0.09; fc[i * 4 + 1] = 0; fc[i * 4 + 2] = 0; fc[i * 4 + 3] = 0.09;
      for (int k = 0; k < 3; k++) fp[i * 3 + k] = feature_positions[i](k);
    }
    detail::pose7_of(marker_pose, mp);
    detail::pose7_of(camera_in_IMU, cin);
    for (int i = 0; i < 36; i++) cm[i] = (i % 7 == 0) ? 1e-4 : 0.0;
    const double cam4[4] = {600, 620, 320, 240};
    or_pose_update_visual(o, 4, ft, fc, fp, mp, cm, cam4, cin);
    compare(filter, o, "visual landmark");
  }

  // resetFilterWithExternalPose(Affine3d) (PoseUKF.hpp:187)
  {
    Affine3d imu_in_nav(Quaterniond(AngleAxisd(-0.4, Vector3d::UnitZ())));
    imu_in_nav.translation() = Vector3d(10.0, 5.0, -4.0);
    filter.resetFilterWithExternalPose(imu_in_nav);
    double p7[7];
    detail::pose7_of(imu_in_nav, p7);
    or_pose_reset_with_external_pose(o, p7);
    for (int e = 400; e < 450; e++) epoch(e);
    compare(filter, o, "reset + 50 epochs");
  }

  // PoseUKF(State, Covariance, location, model, PoseUKFParameter) (PoseUKF.hpp:113-115)
  {
    PoseUKF::State state;
    PoseUKF::Covariance cov;
    filter.getCurrentState(state, cov);
    PoseUKF::PoseUKFParameter filter_parameter;
    filter_parameter.imu_in_body = Vector3d(0.1, 0.0, -0.2);
    filter_parameter.gyro_bias_offset = Vector3d(1e-6, -2e-6, 0.5e-6);
    filter_parameter.gyro_bias_tau = 600;
    filter_parameter.acc_bias_tau = 600;
    filter_parameter.inertia_tau = filter_parameter.lin_damping_tau = filter_parameter.quad_damping_tau = 3600;
    filter_parameter.water_velocity_tau = 900;
    filter_parameter.water_velocity_limits = 0.1;
    filter_parameter.water_velocity_scale = 1e-3;
    filter_parameter.adcp_bias_tau = 900;
    filter_parameter.atmospheric_pressure = 101325;
    filter_parameter.water_density_tau = 3600;
    LocationConfiguration location;
    location.latitude = 0.9; location.longitude = 0.15; location.altitude = 0.0;
    PoseUKF second(state, cov, location, model, filter_parameter);
    second.setProcessNoiseFromConfig(config, dt);
    or_pose* o2 = (or_pose*)calloc(1, or_pose_sizeof());
    double x[54];
    state.to_store(x);
    std::vector<double> Pr(53 * 53);
    detail::put_rowmajor(cov, Pr.data());
    const uwvk_pose_parameter par = filter_parameter.to_c();
    or_pose_init_from_state(o2, 53, x, Pr.data(), &location, &uwv, &par);
    or_pose_set_process_noise_from_config(o2, &cfg, dt, nullptr);
    for (int e = 0; e < 100; e++) {
      int acc;
      rotation_rate.mu = Vector3d(0.01 * n01(rng), 0.01 * n01(rng), 0.01 * n01(rng));
      acceleration.mu = Vector3d(0.02 * n01(rng), 0.02 * n01(rng), 9.81 + 0.02 * n01(rng));
      second.integrateMeasurement(rotation_rate);
      second.predictionStep(dt);
      second.integrateMeasurement(acceleration);
      double m9[9], a9[9];
      detail::put_rowmajor(rotation_rate.cov, m9);
      detail::put_rowmajor(acceleration.cov, a9);
      or_pose_set_rotation_rate(o2, rotation_rate.mu.data(), m9);
      or_pose_predict(o2, dt);
      or_pose_update_acceleration(o2, acceleration.mu.data(), a9, &acc);
    }
    compare(second, o2, "state constructor + 100");
    free(o2);
  }

  // error behaviour: a NaN measurement throws like checkMeasurment [EXT]
  bool threw = false;
  try {
    acceleration.mu(1) = NAN;
    filter.integrateMeasurement(acceleration);
  } catch (const std::runtime_error&) {
    threw = true;
  }
  free(o);

  // ---- VelocityUKF (VelocityUKF.hpp:33-58) ----
  double vworst = 0;
  {
    VelocityUKF::State initial_state;
    initial_state.velocity = Vector3d(0.5, 0.0, 0.0);
    initial_state.z_position << -2.0;
    VelocityUKF::Covariance state_cov = VelocityUKF::Covariance::Identity() * 0.01;
    VelocityUKF vf(initial_state, state_cov);
    const bool model_ok = vf.setupMotionModel(model);
    VelocityUKF::Covariance Q = VelocityUKF::Covariance::Zero();
    Q(0, 0) = Q(1, 1) = Q(2, 2) = 1e-4;
    Q(3, 3) = 1e-3;
    vf.setProcessNoiseCovariance(Q);
    or_vel ov;
    double x4[4], P16[16], q16[16];
    initial_state.to_store(x4);
    detail::put_rowmajor(state_cov, P16);
    detail::put_rowmajor(Q, q16);
    or_vel_init(&ov, x4, P16);
    or_vel_setup_motion_model(&ov, &uwv);
    or_vel_set_process_noise(&ov, q16);
    VelocityUKF::GyroMeasurement gyro;
    VelocityUKF::BodyEffortsMeasurement body_efforts;
    VelocityUKF::DVLMeasurement dvl;
    VelocityUKF::PressureMeasurement depth;
    gyro.cov = Matrix3d::Identity() * 1e-6;
    body_efforts.cov = Matrix6d::Identity() * 1.0;
    dvl.cov = Matrix3d::Identity() * 1e-4;
    depth.cov << 0.01;
    for (int e = 0; e < 200; e++) {
      gyro.mu = Vector3d(0.01 * n01(rng), 0.01 * n01(rng), 0.01 * n01(rng));
      body_efforts.mu << 20 + n01(rng), n01(rng), n01(rng), 0.1 * n01(rng), 0.1 * n01(rng), 0.1 * n01(rng);
      vf.integrateMeasurement(gyro);
      vf.integrateMeasurement(body_efforts);
      vf.predictionStep(0.01);
      double g9[9], e36[36];
      detail::put_rowmajor(gyro.cov, g9);
      detail::put_rowmajor(body_efforts.cov, e36);
      or_vel_set_gyro(&ov, gyro.mu.data(), g9);
      or_vel_set_efforts(&ov, body_efforts.mu.data(), e36);
      or_vel_predict(&ov, 0.01);
      if (e % 10 == 9) {
        dvl.mu = Vector3d(0.5 + 0.02 * n01(rng), 0.02 * n01(rng), 0.02 * n01(rng));
        vf.integrateMeasurement(dvl);
        double d9[9];
        detail::put_rowmajor(dvl.cov, d9);
        or_vel_update_dvl(&ov, dvl.mu.data(), d9);
      }
      if (e % 20 == 19) {
        depth.mu << -2.0 + 0.05 * n01(rng);
        vf.integrateMeasurement(depth);
        const double c1[1] = {depth.cov(0, 0)};
        or_vel_update_pressure(&ov, depth.mu.data(), c1);
      }
    }
    VelocityUKF::State vs;
    VelocityUKF::Covariance vc;
    if (!vf.getCurrentState(vs, vc) || !model_ok) vworst = 1;
    double xv[4];
    vs.to_store(xv);
    for (int i = 0; i < 4; i++) {
      vworst = std::fmax(vworst, std::fabs(xv[i] - ov.mu[i]) / std::sqrt(ov.sigma[i * 5]));
      for (int j = 0; j < 4; j++)
        vworst = std::fmax(vworst, std::fabs(vc(i, j) - ov.sigma[i * 4 + j]) / std::sqrt(ov.sigma[i * 5] * ov.sigma[j * 5]));
    }
    std::printf("%-28s worst %.3e\n", "VelocityUKF 200 epochs", vworst);
  }

  std::printf("reference call forms: worst %.3e (std units), velocity %.3e, gate mismatches %d, nan throws %d\n",
              worst, vworst, gate_mismatch, (int)threw);
  return (worst < 1e-7 && vworst < 1e-7 && gate_mismatch == 0 && threw) ? 0 : 1;
}
