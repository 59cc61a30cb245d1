// linalg_test.cpp — CPU checks of the facade's value types (linalg.hpp,
// reference_types.hpp) that carry the reference call forms: Eigen's
// conventions (column-major storage, row-major comma fill, Quaterniond
// (w, x, y, z), AngleAxisd, rotation-matrix round trips, Affine3d algebra) and
// the conversions to the C ABI (PoseState store layout, PoseUKFConfig / UWVParameters
// to_c).  Quaternion algebra is checked against the oracle's (or_quat_*,
// or_so3_exp).  Exit 0 = pass.
#include <cmath>
#include <cstdio>
#include <random>

#include <uwv_kalman_filters/PoseUKF.hpp>
extern "C" {
#include "../../oracle/uwvk_oracle.h"
}

using namespace uwv_kalman_filters;

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      fails++;                                                    \
    }                                                             \
  } while (0)
static bool near(double a, double b, double t = 1e-13) { return std::fabs(a - b) <= t; }

int main() {
  // storage and comma initializer
  Matrix3d A;
  A << 1, 2, 3, 4, 5, 6, 7, 8, 9;
  CHECK(A(0, 1) == 2 && A(1, 0) == 4 && A(2, 2) == 9);
  CHECK(A.data()[1] == 4);  // column-major
  CHECK(A.transpose()(0, 1) == 4);
  const Matrix3d I = Matrix3d::Identity();
  CHECK((A * I) == A);
  CHECK((A * Vector3d::UnitY())(2) == 8);
  Vector3d v(1, 2, 3);
  CHECK(v.cross(Vector3d(0, 0, 1)) == Vector3d(2, -1, 0));
  CHECK(near(v.norm(), std::sqrt(14.0)));
  CHECK(Vector6d::Ones().asDiagonal()(5, 5) == 1.0);
  bool threw = false;
  try {
    Vector3d w;
    w << 1, 2;  // too few coefficients
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);

  // quaternions against the oracle
  std::mt19937_64 rng(3);
  std::normal_distribution<double> n01;
  for (int t = 0; t < 200; t++) {
    const double rv[3] = {n01(rng), n01(rng), n01(rng)};
    double qo[4], Ro[9];
    or_so3_exp(rv, qo);
    const double ang = std::sqrt(rv[0] * rv[0] + rv[1] * rv[1] + rv[2] * rv[2]);
    const Quaterniond q(AngleAxisd(ang, Vector3d(rv[0] / ang, rv[1] / ang, rv[2] / ang)));
    const double qc[4] = {q.w(), q.x(), q.y(), q.z()};
    for (int k = 0; k < 4; k++) CHECK(near(qc[k], qo[k], 1e-14));
    or_quat_to_matrix(qo, Ro);
    const Matrix3d R = q.toRotationMatrix();
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) CHECK(near(R(i, j), Ro[i * 3 + j], 1e-14));
    const Quaterniond qr(R);
    const double s = qr.w() * q.w() + qr.x() * q.x() + qr.y() * q.y() + qr.z() * q.z();
    CHECK(near(std::fabs(s), 1.0, 1e-14));
    const double v3[3] = {n01(rng), n01(rng), n01(rng)};
    double ro[3];
    or_quat_rotate(qo, v3, ro);
    const Vector3d rr = q * Vector3d(v3[0], v3[1], v3[2]);
    for (int k = 0; k < 3; k++) CHECK(near(rr(k), ro[k], 1e-13));
    double qq[4];
    or_quat_mul(qo, qo, qq);
    const Quaterniond q2 = q * q;
    CHECK(near(q2.w(), qq[0], 1e-14) && near(q2.x(), qq[1], 1e-14) && near(q2.z(), qq[3], 1e-14));
  }

  // Affine3d
  Affine3d T(Quaterniond(AngleAxisd(0.7, Vector3d::UnitZ())));
  T.translation() = Vector3d(1, 2, 3);
  const Vector3d p(0.3, -0.2, 0.5);
  const Vector3d back = T.inverse() * (T * p);
  for (int k = 0; k < 3; k++) CHECK(near(back(k), p(k)));
  double p7[7];
  detail::pose7_of(T, p7);
  CHECK(near(p7[0], 1) && near(p7[3], std::cos(0.35)) && near(p7[6], std::sin(0.35)));

  // PoseState store round trip (include/uwvk.h UWVK_S_*)
  PoseState st;
  st.position = Vector3d(1, 2, 3);
  st.orientation = Quaterniond(0.5, 0.5, -0.5, 0.5);
  st.inertia(1, 0) = 7;  // column-major: slot INERTIA + 1
  st.water_density << 1025;
  double x[54];
  st.to_store(x);
  CHECK(x[UWVK_S_POS + 2] == 3 && x[UWVK_S_QUAT + 2] == -0.5 && x[UWVK_S_INERTIA + 1] == 7 &&
        x[UWVK_S_WATER_DENSITY] == 1025);
  PoseState st2;
  st2.from_store(x);
  double x2[54];
  st2.to_store(x2);
  for (int k = 0; k < 54; k++) CHECK(x[k] == x2[k]);

  // configuration conversions
  PoseUKFConfig cfg;
  cfg.acceleration.randomwalk = Vector3d(1, 2, 3);
  cfg.model_noise_parameters.inertia_instability = VectorXd::Constant(9, 4.0);
  cfg.hydrostatics.pressure_std = 5;
  cfg.max_effort << 1, 2, 3, 4, 5, 6;
  const uwvk_pose_config c = cfg.to_c();
  CHECK(c.acceleration.randomwalk[2] == 3 && c.model_noise_parameters.inertia_instability[8] == 4.0 &&
        c.hydrostatics.pressure_std == 5 && c.max_effort[5] == 6);
  threw = false;
  try {
    cfg.model_noise_parameters.lin_damping_instability = VectorXd::Zero(3);  // the reference maps 9 components
    (void)cfg.to_c();
  } catch (const std::invalid_argument&) {
    threw = true;
  }
  CHECK(threw);
  uwv_dynamic_model::UWVParameters m;
  m.inertia_matrix(0, 5) = 3;
  m.damping_matrices[1](5, 0) = 4;
  const uwvk_uwv_params mc = m.to_c();
  CHECK(mc.inertia_matrix[5] == 3 && mc.damping_matrices[1][30] == 4);  // row-major in the C ABI

  std::printf("linalg / reference types: %d failures\n", fails);
  return fails ? 1 : 0;
}
