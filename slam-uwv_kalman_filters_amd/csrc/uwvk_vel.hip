// uwvk_vel.hip — VelocityUKF (src/VelocityUKF.hpp:231-266, VelocityUKF.cpp) on
// gfx950: one filter instance per LANE.  The state is 4 DOF (body velocity +
// z position) with 9 sigma points, so Sigma, the sigma points and the RK4
// integration of the [EXT] uwv_dynamic_model ModelSimulation all live in
// VGPRs; the kernel is bound by the fp64 model evaluation (9 x RK4 per predict).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "uwvk_dev.hpp"
#include "uwvk_host.hpp"

using namespace uwvk;

namespace {

struct VelShared {  // batch-shared model parameters (by value)
  double M[36], Dl[36], Dq[36], Minv[36];
  double weight, buoyancy, cog[3], cob[3];
  double Q0[16];  // process_noise_cov (VelocityUKF.cpp:54-55)
  double gk, gm[3];  // weight - buoyancy, weight cog - buoyancy cob (restoring forces, v_deriv)
};

struct VelBufs {
  int64_t batch;
  const VelShared* shared;  // device copy of the handle's VelShared (k_vel_epoch_g stages it in LDS)
  double* mu;       // [batch][4]
  double* sigma;    // [batch][16]
  double* gyro;     // [batch][3]  stored GyroMeasurement
  double* efforts;  // [batch][6]  stored BodyEffortsMeasurement
  double* model;    // [batch][13] motion_model pose p(3) q(4) v(3) w(3)
  uint32_t* status;
};

struct VelEpochArgs {
  const uint32_t* flags;
  const double* gyro;     // [epochs][batch][3]
  const double* efforts;  // [epochs][batch][6]
  const int32_t* dvl_index;
  const double* dvl;
  double dvl_cov[9];
  const int32_t* p_index;
  const double* pressure;
  double p_cov;
  double dt;
  int64_t first, count;
};

// The model parameters reach the RK4 code through a pointer laundered before
// every derivative, so that each derivative loads the rows it uses next to
// their use instead of the whole set being hoisted out of the epoch loop (the
// by-value matrices were 370 spilled SGPR slots and ~1,250 v_readlane per
// epoch).
UWVK_DEV const VelShared& vlaunder(const VelShared& p) { return p; }
// (r04) the device copy in the constant address space, its pointer
// re-laundered (an SGPR pair) before every derivative, so that the matrices
// arrive by scalar loads (s_load, the scalar data cache) next to their use
using GVS = __attribute__((address_space(4))) const VelShared;
UWVK_DEV GVS& vlaunder(GVS& p) {
  GVS* q = &p;
  asm volatile("" : "+s"(q));
  return *q;
}

// ---- [EXT] ModelSimulation: M nu_dot + C(nu) nu + D(nu) nu + g(q) = tau, RK4 --
// (r04) fp64 sqrt and division are ~10-15 VALU sequences each on
// gfx950; the Cholesky, the quaternion normalisation and the means' 1/N use
// 1/sqrt (hardware seed + one Halley step, < 1 ulp) and products instead, the
// means' x / N as x (1/N) with one FMA correction (correctly rounded quotient).
// Rounding-level differences from the literal forms, inside the tolerances.
UWVK_DEV double v_rsqrt(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  const double e = fma(-(x * r), r, 1.0);
  return fma(r * e, fma(0.375, e, 0.5), r);
}
template <int N>
UWVK_DEV double v_divn(double x) {
  constexpr double y = 1.0 / N;
  const double q = x * y;
  return fma(fma(-q, (double)N, x), y, q);
}
template <class PS>
UWVK_DEV void v_coriolis(const PS& P, const double nu[6], double c[6]) {
  double a[3], b[3], t0[3], t1[3], t2[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    double sa = 0, sb = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      sa += P.M[i * 6 + j] * nu[j];
      sb += P.M[(3 + i) * 6 + j] * nu[j];
    }
    a[i] = sa; b[i] = sb;
  }
  cross3(nu + 3, a, t0);
  cross3(nu, a, t1);
  cross3(nu + 3, b, t2);
#pragma unroll
  for (int i = 0; i < 3; i++) { c[i] = t0[i]; c[3 + i] = t1[i] + t2[i]; }
}

template <class PS>
UWVK_DEV void v_deriv(const PS& P, const double tau[6], const double s[13], double ds[13]) {
  const double q[4] = {s[3], s[4], s[5], s[6]};
  const double nu[6] = {s[7], s[8], s[9], s[10], s[11], s[12]};
  const double v[3] = {s[7], s[8], s[9]};
  qrot(q, v, ds);
  const double wq[4] = {0, s[10], s[11], s[12]};
  double qd[4];
  qmul(q, wq, qd);
#pragma unroll
  for (int i = 0; i < 4; i++) ds[3 + i] = 0.5 * qd[i];
  double c[6], d[6], g[6], r[6];
  v_coriolis(P, nu, c);
  const auto& PD = P;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double sl = 0, sq = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      sl += PD.Dl[i * 6 + j] * nu[j];
      sq += PD.Dq[i * 6 + j] * (fabs(nu[j]) * nu[j]);
    }
    d[i] = sl + sq;
  }
  // (r04) the restoring forces through one rotation: qrot_inv is linear in its
  // vector and both forces lie along the nav z axis, so with r = R^T e_z
  //   -(fg + fb) = (W - B) r,   -(cog x fg + cob x fb) = (W cog - B cob) x r
  // (the same quantities, one rotation and one cross product instead of two)
  {
    const double ez[3] = {0, 0, 1};
    double r[3], m3[3];
    qrot_inv(q, ez, r);
    const double gm[3] = {P.gm[0], P.gm[1], P.gm[2]};
    cross3(gm, r, m3);
#pragma unroll
    for (int i = 0; i < 3; i++) { g[i] = P.gk * r[i]; g[3 + i] = m3[i]; }
  }
#pragma unroll
  for (int i = 0; i < 6; i++) r[i] = tau[i] - c[i] - d[i] - g[i];
  const auto& PI = P;
#pragma unroll
  for (int i = 0; i < 6; i++) {
    double a = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) a += PI.Minv[i * 6 + j] * r[j];
    ds[7 + i] = a;
  }
}

// the stage sum k1 + 2 k2 + 2 k3 + k4 is accumulated as the stages finish, in
// the same left-to-right order (one 13-vector live instead of four)
template <class PS>
UWVK_DEV void v_rk4(const PS& P, const double tau[6], double dt, const double s[13], double o[13]) {
  double k[13], acc[13], t[13];
  v_deriv(vlaunder(P), tau, s, k);
#pragma unroll
  for (int i = 0; i < 13; i++) {
    acc[i] = k[i];
    t[i] = s[i] + 0.5 * dt * k[i];
  }
  v_deriv(vlaunder(P), tau, t, k);
#pragma unroll
  for (int i = 0; i < 13; i++) {
    acc[i] = acc[i] + 2.0 * k[i];
    t[i] = s[i] + 0.5 * dt * k[i];
  }
  v_deriv(vlaunder(P), tau, t, k);
#pragma unroll
  for (int i = 0; i < 13; i++) {
    acc[i] = acc[i] + 2.0 * k[i];
    t[i] = s[i] + dt * k[i];
  }
  v_deriv(vlaunder(P), tau, t, k);
#pragma unroll
  for (int i = 0; i < 13; i++) o[i] = s[i] + (dt / 6.0) * (acc[i] + k[i]);
  const double in = v_rsqrt(o[3] * o[3] + o[4] * o[4] + o[5] * o[5] + o[6] * o[6]);
#pragma unroll
  for (int i = 3; i < 7; i++) o[i] *= in;
}

// ---- 4-DOF vector-manifold UKF core in registers [EXT ukfom] -----------------
UWVK_DEV bool v_chol(const double A[16], double L[16]) {
  bool ok = true;
  double inv[4];
#pragma unroll
  for (int i = 0; i < 16; i++) L[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
#pragma unroll
    for (int j = 0; j <= i; j++) {
      double s = A[i * 4 + j];
#pragma unroll
      for (int k = 0; k < j; k++) s -= L[i * 4 + k] * L[j * 4 + k];
      if (i == j) {
        ok = ok && (s > 0.0);
        inv[i] = v_rsqrt(s);
        L[i * 4 + i] = s * inv[i];
      } else {
        L[i * 4 + j] = s * inv[j];
      }
    }
  }
  return ok;
}

UWVK_DEV void v_points(const double mu[4], const double L[16], double X[9][4]) {
#pragma unroll
  for (int k = 0; k < 4; k++) X[0][k] = mu[k];
#pragma unroll
  for (int j = 0; j < 4; j++)
#pragma unroll
    for (int k = 0; k < 4; k++) {
      X[2 * j + 1][k] = mu[k] + 1.0 * L[k * 4 + j];
      X[2 * j + 2][k] = mu[k] + -1.0 * L[k * 4 + j];
    }
}

// manifold mean (all-vector here): ref = X0, delta = mean(X - ref), |delta| <= 1e-6
template <int M, int N>
UWVK_DEV void v_mean(const double (&X)[N][M], double ref[M]) {
#pragma unroll
  for (int k = 0; k < M; k++) ref[k] = X[0][k];
  int it = 0;
  double nrm;
  do {
    double d[M];
#pragma unroll
    for (int k = 0; k < M; k++) d[k] = 0.0;
#pragma unroll
    for (int p = 0; p < N; p++)
#pragma unroll
      for (int k = 0; k < M; k++) d[k] += X[p][k] - ref[k];
    nrm = 0.0;
#pragma unroll
    for (int k = 0; k < M; k++) {
      d[k] = v_divn<N>(d[k]);
      nrm += d[k] * d[k];
    }
#pragma unroll
    for (int k = 0; k < M; k++) ref[k] = ref[k] + 1.0 * d[k];
  } while (nrm > 1e-12 && ++it < 10000);  // |delta|^2 against (1e-6)^2: no sqrt
}

UWVK_DEV void v_cov(const double (&X)[9][4], const double mean[4], double S[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) S[i] = 0.0;
#pragma unroll
  for (int p = 0; p < 9; p++) {
    double d[4];
#pragma unroll
    for (int k = 0; k < 4; k++) d[k] = X[p][k] - mean[k];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) S[i * 4 + j] += d[i] * d[j];
  }
#pragma unroll
  for (int i = 0; i < 16; i++) S[i] = 0.5 * S[i];
}

// processMotionModel, VelocityUKF.cpp:6-33
template <class PS>
UWVK_DEV void v_process(const PS& P, const double q[4], const double w[3], const double tau[6], double dt,
                        double x[4]) {
  double s[13], n[13], r[3], t[3];
  s[0] = s[1] = s[2] = 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) s[3 + k] = q[k];
#pragma unroll
  for (int k = 0; k < 3; k++) { s[7 + k] = x[k]; s[10 + k] = w[k]; }
  v_rk4(P, tau, dt, s, n);
#pragma unroll
  for (int i = 0; i < 3; i++) t[i] = x[i] + (n[7 + i] - x[i]);
  qrot(q, t, r);
  x[3] = x[3] + dt * r[2];
  x[0] = t[0]; x[1] = t[1]; x[2] = t[2];
}

template <class PS>
UWVK_DEV bool v_predict(const PS& P, double mu[4], double S[16], const double model[13], const double w[3],
                        const double tau[6], double dt) {
  double L[16], X[9][4];
  const bool ok = v_chol(S, L);
  v_points(mu, L, X);
  const double q[4] = {model[3], model[4], model[5], model[6]};
#pragma unroll
  for (int p = 0; p < 9; p++) v_process(P, q, w, tau, dt, X[p]);
  v_mean<4, 9>(X, mu);
  v_cov(X, mu, S);
#pragma unroll
  for (int i = 0; i < 16; i++) S[i] += dt * P.Q0[i];
  return ok;
}

// update with h = a sub-vector of the state (DVL: v, m = 3; pressure: z, m = 1),
// vect-manifold measurement (iterative mean), accept any
template <int M, int OFF>
UWVK_DEV bool v_update(double mu[4], double S[16], const double z[M], const double R[M * M]) {
  double L[16], X[9][4], Z[9][M];
  bool ok = v_chol(S, L);
  v_points(mu, L, X);
#pragma unroll
  for (int p = 0; p < 9; p++)
#pragma unroll
    for (int a = 0; a < M; a++) Z[p][a] = X[p][OFF + a];
  double zm[M];
  v_mean<M, 9>(Z, zm);
  double Sz[M * M], C[4 * M], Si[M * M], K[4 * M], nu[M];
#pragma unroll
  for (int i = 0; i < M * M; i++) Sz[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 4 * M; i++) C[i] = 0.0;
#pragma unroll
  for (int p = 0; p < 9; p++) {
    double dz[M], dx[4];
#pragma unroll
    for (int a = 0; a < M; a++) dz[a] = Z[p][a] - zm[a];
#pragma unroll
    for (int k = 0; k < 4; k++) dx[k] = X[p][k] - mu[k];
#pragma unroll
    for (int a = 0; a < M; a++)
#pragma unroll
      for (int b = 0; b < M; b++) Sz[a * M + b] += dz[a] * dz[b];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int a = 0; a < M; a++) C[i * M + a] += dx[i] * dz[a];
  }
#pragma unroll
  for (int i = 0; i < M * M; i++) Sz[i] = 0.5 * Sz[i] + R[i];
#pragma unroll
  for (int i = 0; i < 4 * M; i++) C[i] = 0.5 * C[i];
  if constexpr (M == 1) {
    Si[0] = 1.0 / Sz[0];
  } else {
    const double* A = Sz;
    const double c00 = A[4] * A[8] - A[5] * A[7];
    const double c01 = A[5] * A[6] - A[3] * A[8];
    const double c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    const double id = 1.0 / det;
    Si[0] = c00 * id;
    Si[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    Si[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    Si[3] = c01 * id;
    Si[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    Si[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    Si[6] = c02 * id;
    Si[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    Si[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int a = 0; a < M; a++) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < M; b++) s += C[i * M + b] * Si[b * M + a];
      K[i * M + a] = s;
    }
#pragma unroll
  for (int a = 0; a < M; a++) nu[a] = z[a] - zm[a];
  // accept_any_mahalanobis_distance: Sigma -= C K^T, apply_delta(K nu)
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double s = 0.0;
#pragma unroll
      for (int a = 0; a < M; a++) s += C[i * M + a] * K[j * M + a];
      S[i * 4 + j] -= s;
    }
  double delta[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < M; a++) s += K[i * M + a] * nu[a];
    delta[i] = s;
  }
  ok = v_chol(S, L) && ok;
  v_points(mu, L, X);
#pragma unroll
  for (int k = 0; k < 4; k++) mu[k] = mu[k] + 1.0 * delta[k];
#pragma unroll
  for (int p = 0; p < 9; p++)
#pragma unroll
    for (int k = 0; k < 4; k++) X[p][k] = X[p][k] + 1.0 * delta[k];
  v_cov(X, mu, S);
  return ok;
}

UWVK_DEV void v_load(const VelBufs& b, int64_t i, double mu[4], double S[16]) {
#pragma unroll
  for (int k = 0; k < 4; k++) mu[k] = b.mu[i * 4 + k];
#pragma unroll
  for (int k = 0; k < 16; k++) S[k] = b.sigma[i * 16 + k];
}
UWVK_DEV void v_store(const VelBufs& b, int64_t i, const double mu[4], const double S[16]) {
#pragma unroll
  for (int k = 0; k < 4; k++) b.mu[i * 4 + k] = mu[k];
#pragma unroll
  for (int k = 0; k < 16; k++) b.sigma[i * 16 + k] = S[k];
}

// (r04) the model parameters by scalar loads from the handle's device copy
// (vlaunder above): the by-value kernel argument (144 doubles of
// matrices) did not fit the SGPRs, was spilled to VGPR lanes and read back by
// ~1,000 v_readlane per epoch; C2 534.6-542.1 -> 620.3-620.9 M steps/s
// (profiles/r04/c2smem/)
#define VEL_PARAMS(b, P0) GVS& P = *(GVS*)(b).shared; (void)(P0)

__global__ __launch_bounds__(64) void k_vel_predict(VelBufs b, VelShared P0, double dt) {
  VEL_PARAMS(b, P0);
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= b.batch) return;
  double mu[4], S[16], m[13], w[3], tau[6];
  v_load(b, i, mu, S);
#pragma unroll
  for (int k = 0; k < 13; k++) m[k] = b.model[i * 13 + k];
#pragma unroll
  for (int k = 0; k < 3; k++) w[k] = b.gyro[i * 3 + k];
#pragma unroll
  for (int k = 0; k < 6; k++) tau[k] = b.efforts[i * 6 + k];
  const bool ok = v_predict(P, mu, S, m, w, tau, dt);
  double n[13];
  v_rk4(P, tau, dt, m, n);  // motion_model->sendEffort(tau) (VelocityUKF.cpp:126-127)
#pragma unroll
  for (int k = 0; k < 13; k++) b.model[i * 13 + k] = n[k];
  if (!ok) b.status[i] |= UWVK_ST_NOTPD;
  v_store(b, i, mu, S);
}

template <int M, int OFF>
__global__ __launch_bounds__(64) void k_vel_update(VelBufs b, const double* z, const double* cov, VelShared P,
                                                   double shared_cov0, const double* shared_cov, const uint8_t* mask) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= b.batch || (mask && !mask[i])) return;
  double mu[4], S[16], zz[M], R[M * M];
  v_load(b, i, mu, S);
#pragma unroll
  for (int a = 0; a < M; a++) zz[a] = z[i * M + a];
#pragma unroll
  for (int a = 0; a < M * M; a++) R[a] = cov ? cov[i * M * M + a] : shared_cov[a];
  const bool ok = v_update<M, OFF>(mu, S, zz, R);
  if (!ok) b.status[i] |= UWVK_ST_NOTPD;
  v_store(b, i, mu, S);
  (void)P;
  (void)shared_cov0;
}

__global__ __launch_bounds__(64) void k_vel_epoch(VelBufs b, VelShared P0, VelEpochArgs ea) {
  VEL_PARAMS(b, P0);
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= b.batch) return;
  const int64_t B = b.batch;
  double mu[4], S[16], m[13], w[3], tau[6];
  v_load(b, i, mu, S);
#pragma unroll
  for (int k = 0; k < 13; k++) m[k] = b.model[i * 13 + k];
  bool ok = true;
  for (int64_t e = ea.first; e < ea.first + ea.count; e++) {
    // GyroMeasurement: stored + copied into the motion model (VelocityUKF.cpp:87-98)
#pragma unroll
    for (int k = 0; k < 3; k++) { w[k] = ea.gyro[(e * B + i) * 3 + k]; m[10 + k] = w[k]; }
#pragma unroll
    for (int k = 0; k < 6; k++) tau[k] = ea.efforts[(e * B + i) * 6 + k];
    ok = v_predict(P, mu, S, m, w, tau, ea.dt) && ok;
    double n[13];
    v_rk4(P, tau, ea.dt, m, n);
#pragma unroll
    for (int k = 0; k < 13; k++) m[k] = n[k];
    const uint32_t fl = ea.flags[e];
    if (fl & UWVK_EV_DVL) {
      const double* z = ea.dvl + ((int64_t)ea.dvl_index[e] * B + i) * 3;
      const double zz[3] = {z[0], z[1], z[2]};
      ok = v_update<3, 0>(mu, S, zz, ea.dvl_cov) && ok;
    }
    if (fl & UWVK_EV_PRESSURE) {
      const double zz[1] = {ea.pressure[(int64_t)ea.p_index[e] * B + i]};
      const double R[1] = {ea.p_cov};
      ok = v_update<1, 3>(mu, S, zz, R) && ok;
    }
  }
  if (ea.count > 0) {
#pragma unroll
    for (int k = 0; k < 3; k++) b.gyro[i * 3 + k] = w[k];
#pragma unroll
    for (int k = 0; k < 6; k++) b.efforts[i * 6 + k] = tau[k];
  }
#pragma unroll
  for (int k = 0; k < 13; k++) b.model[i * 13 + k] = m[k];
  if (!ok) b.status[i] |= UWVK_ST_NOTPD;
  v_store(b, i, mu, S);
}

// ---------------------------------------------------------------------------
// Lane-group epoch kernel: 16 lanes (one DPP row) per filter, ONE SIGMA POINT
// PER LANE (lanes 0..8), lane 9 advances the side motion model
// (motion_model->sendEffort, VelocityUKF.cpp:126-127) in the same RK4 pass.
// mu / Sigma are replicated in every lane of the row and kept bitwise
// identical: the cross-point sums are butterfly reductions inside the row
// (quad_perm / half-mirror / mirror DPP), whose result is the same in every
// lane.  4 filters per wave: batch 4096 fills 1024 waves, one per SIMD,
// where the lane-per-filter kernel occupies 64.
// ---------------------------------------------------------------------------
// (r04) every lane has a source lane under the controls used here
// (quad_perm, row_half_mirror, row_mirror, all rows and banks), so the old value
// is never read: mov_dpp leaves it undefined, where update_dpp's explicit 0 cost
// a v_mov_b32 before every DPP move (~490 per wave-epoch pass of the C2 kernel)
template <int CTRL>
UWVK_DEV double vdpp(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
// sum over the 16 lanes of this lane's DPP row, identical in every lane
UWVK_DEV double row_sum16(double v) {
  v = v + vdpp<0xb1>(v);   // quad_perm [1,0,3,2]
  v = v + vdpp<0x4e>(v);   // quad_perm [2,3,0,1]
  v = v + vdpp<0x141>(v);  // row_half_mirror
  v = v + vdpp<0x140>(v);  // row_mirror
  return v;
}
// lane SRC of each 16-lane row to the whole row (two ds_bpermute; the DPP
// row_newbcast form was not kept, profiles/EXPERIMENTS.md)
template <int SRC>
UWVK_DEV double row_bcast_c(double v) {
  static_assert(SRC >= 0 && SRC < 16, "row lane");
  const int ba = (((int)threadIdx.x & ~15) + SRC) * 4;
  const int lo = __builtin_amdgcn_ds_bpermute(ba, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(ba, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
// value of row lane src (0..15) in every lane of the row
UWVK_DEV double row_bcast(double v, int src) {
  const int ba = (((int)threadIdx.x & ~15) + src) * 4;
  const int lo = __builtin_amdgcn_ds_bpermute(ba, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(ba, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

// sigma point g of (mu, L) [EXT ukfom]: 0 = mu, 2j+1 = mu + L_j, 2j+2 = mu - L_j
UWVK_DEV void vg_point(const double mu[4], const double L[16], int g, double x[4]) {
  const int j = g >= 1 && g < 9 ? (g - 1) >> 1 : 0;
  const double sg = (g >= 1 && g < 9) ? ((g & 1) ? 1.0 : -1.0) : 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double c = L[k * 4];
#pragma unroll
    for (int jj = 1; jj < 4; jj++) {
      c = (j == jj) ? L[k * 4 + jj] : c;
      asm volatile("" : "+v"(c));  // keep the selects: as one lane-indexed L[k][j] the compiler put L in scratch
    }
    x[k] = sg == 0.0 ? mu[k] : mu[k] + sg * c;
  }
}

// iterative vect mean over the 9 point lanes (ref = X_0, |delta| <= 1e-6)
template <int M>
UWVK_DEV void vg_mean(const double x[M], bool pt, double ref[M]) {
#pragma unroll
  for (int k = 0; k < M; k++) ref[k] = row_bcast_c<0>(x[k]);
  int it = 0;
  double nrm;
  do {
    double d[M];
    nrm = 0.0;
#pragma unroll
    for (int k = 0; k < M; k++) {
      d[k] = v_divn<9>(row_sum16(pt ? x[k] - ref[k] : 0.0));
      nrm += d[k] * d[k];
    }
#pragma unroll
    for (int k = 0; k < M; k++) ref[k] = ref[k] + 1.0 * d[k];
  } while (nrm > 1e-12 && ++it < 10000);
}

// Sigma = 1/2 sum_p d_p d_p^T over the point lanes (+ add)
UWVK_DEV void vg_cov(const double x[4], const double mean[4], bool pt, double S[16]) {
  double d[4];
#pragma unroll
  for (int k = 0; k < 4; k++) d[k] = pt ? x[k] - mean[k] : 0.0;
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      const double s = 0.5 * row_sum16(d[i] * d[j]);
      S[i * 4 + j] = s;
      S[j * 4 + i] = s;
    }
}

// update with h = x[OFF..OFF+M) (VelocityUKF.cpp:100-124), accept any
template <int M, int OFF>
UWVK_DEV bool vg_update(double mu[4], double S[16], const double z[M], const double R[M * M], int g) {
  const bool pt = g < 9;
  double L[16], x[4];
  bool ok = v_chol(S, L);
  vg_point(mu, L, g, x);
  double zp[M], zm[M];
#pragma unroll
  for (int a = 0; a < M; a++) zp[a] = x[OFF + a];
  vg_mean<M>(zp, pt, zm);
  double dz[M], dx[4];
#pragma unroll
  for (int a = 0; a < M; a++) dz[a] = pt ? zp[a] - zm[a] : 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) dx[k] = pt ? x[k] - mu[k] : 0.0;
  double Sz[M * M], C[4 * M], Si[M * M], K[4 * M], nu[M];
#pragma unroll
  for (int a = 0; a < M; a++)
#pragma unroll
    for (int b = 0; b <= a; b++) {
      const double s = row_sum16(dz[a] * dz[b]);
      Sz[a * M + b] = 0.5 * s + R[a * M + b];
      Sz[b * M + a] = 0.5 * s + R[b * M + a];
    }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int a = 0; a < M; a++) C[i * M + a] = 0.5 * row_sum16(dx[i] * dz[a]);
  if constexpr (M == 1) {
    Si[0] = 1.0 / Sz[0];
  } else {
    const double* A = Sz;
    const double c00 = A[4] * A[8] - A[5] * A[7];
    const double c01 = A[5] * A[6] - A[3] * A[8];
    const double c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    const double id = 1.0 / det;
    Si[0] = c00 * id;
    Si[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    Si[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    Si[3] = c01 * id;
    Si[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    Si[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    Si[6] = c02 * id;
    Si[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    Si[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int a = 0; a < M; a++) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < M; b++) s += C[i * M + b] * Si[b * M + a];
      K[i * M + a] = s;
    }
#pragma unroll
  for (int a = 0; a < M; a++) nu[a] = z[a] - zm[a];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double s = 0.0;
#pragma unroll
      for (int a = 0; a < M; a++) s += C[i * M + a] * K[j * M + a];
      S[i * 4 + j] -= s;
    }
  double delta[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    double s = 0.0;
#pragma unroll
    for (int a = 0; a < M; a++) s += K[i * M + a] * nu[a];
    delta[i] = s;
  }
  // apply_delta: re-spread about mu, shift every point and mu by delta
  ok = v_chol(S, L) && ok;
  vg_point(mu, L, g, x);
#pragma unroll
  for (int k = 0; k < 4; k++) {
    mu[k] = mu[k] + 1.0 * delta[k];
    x[k] = x[k] + 1.0 * delta[k];
  }
  vg_cov(x, mu, pt, S);
  return ok;
}

// lanes per filter: 16 (one DPP row).  VG = 32 is a diagnostic (UWVK_VEL_OPT_LANE_GROUPS
// 2, r05): every filter runs twice, in the two rows of its 32-lane group, and
// only the first row stores; the wave's instruction stream is the VG = 16
// kernel's, with half the filters per wave and twice the waves (2 per SIMD at
// C2's batch 4,096, which needs <= 256 VGPR + AGPR: amdgpu_waves_per_eu(2)).
// It prices the latency hiding a 32-lane split would get before any of the
// split's own savings.

// (r04) loop-invariant scalar data (Q0, the DVL covariance) loaded where it is
// used: hoisted out of the epoch loop it held 50 SGPRs, which the register
// allocator spilled to VGPR lanes and restored with v_readlane every epoch

template <int VG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(VG / 16, VG / 16))) void k_vel_epoch_g(VelBufs b, VelShared P0, VelEpochArgs ea) {
  VEL_PARAMS(b, P0);
  const int g = (int)threadIdx.x & 15;
  const int64_t B = b.batch, inst = (int64_t)blockIdx.x * (64 / VG) + (int)threadIdx.x / VG;
  const bool live = inst < B;
  const int64_t i = live ? inst : B - 1;  // dead groups compute on a copy and store nothing
  const bool pt = g < 9, side = g == 9;
  double mu[4], S[16], m[13], w[3], tau[6];
  v_load(b, i, mu, S);
#pragma unroll
  for (int k = 0; k < 13; k++) m[k] = b.model[i * 13 + k];
  double q[4] = {m[3], m[4], m[5], m[6]};
  bool ok = true;
  // (r04) the next epoch's gyro / efforts / flag word issued one epoch ahead:
  // at one wave per SIMD the loads' latency was exposed at the top of every epoch
  double w_n[3] = {0, 0, 0}, tau_n[6] = {0, 0, 0, 0, 0, 0};
  uint32_t fl_n = 0;
  auto fetch = [&](int64_t e) {
#pragma unroll
    for (int k = 0; k < 3; k++) w_n[k] = ea.gyro[(e * B + i) * 3 + k];
#pragma unroll
    for (int k = 0; k < 6; k++) tau_n[k] = ea.efforts[(e * B + i) * 6 + k];
    fl_n = ea.flags[e + (g >> 4)];  // a lane-dependent (zero) offset: a VGPR until used
  };
  if (ea.count > 0) fetch(ea.first);
  for (int64_t e = ea.first; e < ea.first + ea.count; e++) {
    const uint32_t fl = __builtin_amdgcn_readfirstlane(fl_n);
#pragma unroll
    for (int k = 0; k < 3; k++) { w[k] = w_n[k]; m[10 + k] = w[k]; }
#pragma unroll
    for (int k = 0; k < 6; k++) tau[k] = tau_n[k];
    if (e + 1 < ea.first + ea.count) fetch(e + 1);
    // predict (VelocityUKF.cpp:115-128): point lanes integrate their sigma
    // point, lane 9 the side model, in one RK4 pass
    double L[16], x[4];
    ok = v_chol(S, L) && ok;
    vg_point(mu, L, g, x);
    double s13[13], n13[13];
#pragma unroll
    for (int k = 0; k < 13; k++) s13[k] = m[k];
    if (!side) {
      s13[0] = s13[1] = s13[2] = 0.0;
#pragma unroll
      for (int k = 0; k < 4; k++) s13[3 + k] = q[k];
#pragma unroll
      for (int k = 0; k < 3; k++) s13[7 + k] = x[k];
    }
    v_rk4(P, tau, ea.dt, s13, n13);
    {  // processMotionModel tail (VelocityUKF.cpp:22-32)
      double t[3], r[3];
#pragma unroll
      for (int k = 0; k < 3; k++) t[k] = x[k] + (n13[7 + k] - x[k]);
      qrot(q, t, r);
      x[3] = x[3] + ea.dt * r[2];
      x[0] = t[0]; x[1] = t[1]; x[2] = t[2];
    }
    vg_mean<4>(x, pt, mu);
    vg_cov(x, mu, pt, S);
    {  // Q0 by scalar loads here, not hoisted out of the loop into 32 SGPRs held across it
      const auto& PQ = vlaunder(P);
#pragma unroll
      for (int k = 0; k < 16; k++) S[k] += ea.dt * PQ.Q0[k];
    }
    if (side) {
#pragma unroll
      for (int k = 0; k < 13; k++) m[k] = n13[k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) q[k] = row_bcast_c<9>(side ? m[3 + k] : 0.0);
    if (fl & UWVK_EV_DVL) {
      const double* z = ea.dvl + ((int64_t)ea.dvl_index[e] * B + i) * 3;
      const double zz[3] = {z[0], z[1], z[2]};
      const double* Rd = ea.dvl_cov;
      asm volatile("" : "+s"(Rd));  // R loaded in the branch, not held in SGPRs across the loop
      ok = vg_update<3, 0>(mu, S, zz, Rd, g) && ok;
    }
    if (fl & UWVK_EV_PRESSURE) {
      const double zz[1] = {ea.pressure[(int64_t)ea.p_index[e] * B + i]};
      const double R[1] = {ea.p_cov};
      ok = vg_update<1, 3>(mu, S, zz, R, g) && ok;
    }
  }
  if (!live) return;
  if (VG == 32 && (threadIdx.x & 16)) return;  // the shadow row
  if (side) {
    if (ea.count > 0) {
#pragma unroll
      for (int k = 0; k < 3; k++) b.gyro[i * 3 + k] = w[k];
#pragma unroll
      for (int k = 0; k < 6; k++) b.efforts[i * 6 + k] = tau[k];
    }
#pragma unroll
    for (int k = 0; k < 13; k++) b.model[i * 13 + k] = m[k];
    if (!ok) b.status[i] |= UWVK_ST_NOTPD;
    v_store(b, i, mu, S);
  }
}

__global__ void k_vel_setup(VelBufs b) {  // setupMotionModel pose (VelocityUKF.cpp:65-74)
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= b.batch) return;
  double* m = b.model + i * 13;
  m[0] = m[1] = m[2] = 0.0;
  m[3] = 1.0; m[4] = m[5] = m[6] = 0.0;
  for (int k = 0; k < 3; k++) { m[7 + k] = b.mu[i * 4 + k]; m[10 + k] = b.gyro[i * 3 + k]; }
}

__global__ void k_vel_gyro_to_model(VelBufs b) {
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= b.batch) return;
  for (int k = 0; k < 3; k++) b.model[i * 13 + 10 + k] = b.gyro[i * 3 + k];
}

}  // namespace

struct uwvk_vel {
  int64_t batch = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  double *d_mu = nullptr, *d_sigma = nullptr, *d_gyro = nullptr, *d_eff = nullptr, *d_model = nullptr,
         *d_meas = nullptr;
  uint8_t* d_mask = nullptr;
  uint32_t* d_status = nullptr;
  VelShared* d_shared = nullptr;  // device copy of P (uploaded by every call that changes P)
  VelShared P{};
  bool has_state = false, has_model = false;
  int groups = -1;  // UWVK_VEL_OPT_LANE_GROUPS: -1 auto, 0 lane per filter, 1 16 lanes per filter
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
};
// auto: lane groups below the measured crossover (MI355X, r04 kernels,
// profiles/r04/velx/: the lane-per-filter kernel's epoch takes ~32-34 us at any
// batch up to 65536, one wave per SIMD; the lane-group kernel 4.6 us at 4096
// and ~1.04 ns per instance once the chip is full: equal near 31k; r03: 24576)
static constexpr int64_t kVelGroupsMaxBatch = 30720;

static VelBufs vbufs(const uwvk_vel* h) {
  VelBufs b;
  b.batch = h->batch; b.mu = h->d_mu; b.sigma = h->d_sigma; b.gyro = h->d_gyro; b.efforts = h->d_eff;
  b.model = h->d_model; b.status = h->d_status;
  b.shared = h->d_shared;
  return b;
}

#define HIPCHK(x)                                  \
  do {                                             \
    const hipError_t e_ = (x);                     \
    if (e_ != hipSuccess) {                        \
      ::uwvk::note_hip_error((int)e_, __func__);   \
      return UWVK_EDEVICE;                         \
    }                                              \
  } while (0)

static unsigned vgrid(int64_t B) { return (unsigned)((B + 63) / 64); }

static bool vfinite(const double* a, size_t n) {
  for (size_t k = 0; k < n; k++)
    if (!std::isfinite(a[k])) return false;
  return true;
}

extern "C" {

uwvk_status uwvk_vel_create(int64_t batch, int device, uwvk_vel** out) {
  ::uwvk::DeviceGuard uwvk_device_guard_(device);
  if (!out || batch <= 0) return UWVK_EINVAL;
  *out = nullptr;
  if (!uwvk_device_available(device)) return UWVK_EDEVICE;
  uwvk_vel* h = new uwvk_vel();
  h->batch = batch;
  h->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return UWVK_EDEVICE;
  }
  const size_t B = (size_t)batch;
  const bool ok = hipMalloc(&h->d_mu, B * 4 * 8) == hipSuccess && hipMalloc(&h->d_sigma, B * 16 * 8) == hipSuccess &&
                  hipMalloc(&h->d_gyro, B * 3 * 8) == hipSuccess && hipMalloc(&h->d_eff, B * 6 * 8) == hipSuccess &&
                  hipMalloc(&h->d_model, B * 13 * 8) == hipSuccess && hipMalloc(&h->d_meas, B * 12 * 8) == hipSuccess &&
                  hipMalloc(&h->d_mask, B) == hipSuccess && hipMalloc(&h->d_status, B * 4) == hipSuccess &&
                  hipMalloc(&h->d_shared, sizeof(VelShared)) == hipSuccess;
  if (!ok) {
    uwvk_vel_destroy(h);
    return UWVK_ENOMEM;
  }
  (void)hipMemsetAsync(h->d_gyro, 0, B * 3 * 8, h->stream);
  (void)hipMemsetAsync(h->d_eff, 0, B * 6 * 8, h->stream);
  (void)hipMemsetAsync(h->d_model, 0, B * 13 * 8, h->stream);
  (void)hipMemsetAsync(h->d_status, 0, B * 4, h->stream);
  // process_noise_cov = 0 except velocity diag 1e-4 (VelocityUKF.cpp:54-55)
  for (int k = 0; k < 3; k++) h->P.Q0[k * 4 + k] = 0.0001;
  if (hipMemcpyAsync(h->d_shared, &h->P, sizeof(VelShared), hipMemcpyHostToDevice, h->stream) != hipSuccess ||
      hipStreamSynchronize(h->stream) != hipSuccess) {
    uwvk_vel_destroy(h);
    return UWVK_EDEVICE;
  }
  *out = h;
  return UWVK_OK;
}

void uwvk_vel_destroy(uwvk_vel* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : {(void*)h->d_mu, (void*)h->d_sigma, (void*)h->d_gyro, (void*)h->d_eff, (void*)h->d_model,
                  (void*)h->d_meas, (void*)h->d_mask, (void*)h->d_status, (void*)h->d_shared})
    if (p) (void)hipFree(p);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

uwvk_status uwvk_vel_set_option(uwvk_vel* h, int option, int value) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (option != UWVK_VEL_OPT_LANE_GROUPS || value < -1 || value > 2) return UWVK_EINVAL;
  h->groups = value;
  return UWVK_OK;
}

uwvk_status uwvk_vel_set_process_noise(uwvk_vel* h, const double Q[16]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !Q) return UWVK_EINVAL;
  if (!vfinite(Q, 16)) return UWVK_ENAN;
  std::memcpy(h->P.Q0, Q, sizeof(h->P.Q0));
  // after all queued work (a running kernel may read the previous copy)
  HIPCHK(hipStreamSynchronize(h->stream));
  HIPCHK(hipMemcpyAsync(h->d_shared, &h->P, sizeof(VelShared), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_synchronize(uwvk_vel* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  return hipStreamSynchronize(h->stream) == hipSuccess ? UWVK_OK : UWVK_EDEVICE;
}

uwvk_status uwvk_vel_timer_start(uwvk_vel* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->ev0 && hipEventCreate(&h->ev0) != hipSuccess) return UWVK_EDEVICE;
  if (!h->ev1 && hipEventCreate(&h->ev1) != hipSuccess) return UWVK_EDEVICE;
  HIPCHK(hipEventRecord(h->ev0, h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_timer_stop(uwvk_vel* h, float* ms) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !ms || !h->ev0 || !h->ev1) return UWVK_EINVAL;
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  HIPCHK(hipEventSynchronize(h->ev1));
  HIPCHK(hipEventElapsedTime(ms, h->ev0, h->ev1));
  return UWVK_OK;
}

void* uwvk_vel_stream(const uwvk_vel* h) { return h ? (void*)h->stream : nullptr; }

uwvk_status uwvk_vel_init(uwvk_vel* h, const double* x, const double* P) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !x || !P) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(h->d_mu, x, (size_t)h->batch * 4 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_sigma, P, (size_t)h->batch * 16 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return UWVK_OK;
}

uwvk_status uwvk_vel_setup_motion_model(uwvk_vel* h, const uwvk_uwv_params* u) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !u) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  std::memcpy(h->P.M, u->inertia_matrix, 36 * 8);
  std::memcpy(h->P.Dl, u->damping_matrices[0], 36 * 8);
  std::memcpy(h->P.Dq, u->damping_matrices[1], 36 * 8);
  if (!host::invert6(u->inertia_matrix, h->P.Minv)) return UWVK_EINVAL;
  h->P.weight = u->weight;
  h->P.buoyancy = u->buoyancy;
  for (int k = 0; k < 3; k++) {
    h->P.cog[k] = u->distance_body2centerofgravity[k];
    h->P.cob[k] = u->distance_body2centerofbuoyancy[k];
  }
  h->P.gk = u->weight - u->buoyancy;
  for (int k = 0; k < 3; k++)
    h->P.gm[k] = u->weight * u->distance_body2centerofgravity[k] - u->buoyancy * u->distance_body2centerofbuoyancy[k];
  HIPCHK(hipStreamSynchronize(h->stream));  // a running kernel may read the previous copy
  HIPCHK(hipMemcpyAsync(h->d_shared, &h->P, sizeof(VelShared), hipMemcpyHostToDevice, h->stream));
  hipLaunchKernelGGL(k_vel_setup, dim3(vgrid(h->batch)), dim3(64), 0, h->stream, vbufs(h));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_model = true;
  return UWVK_OK;
}

uwvk_status uwvk_vel_set_gyro(uwvk_vel* h, const double* w, const double* cov) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !w) return UWVK_EINVAL;
  if (!vfinite(w, (size_t)h->batch * 3) || (cov && !vfinite(cov, (size_t)h->batch * 9))) return UWVK_ENAN;
  HIPCHK(hipMemcpyAsync(h->d_gyro, w, (size_t)h->batch * 3 * 8, hipMemcpyHostToDevice, h->stream));
  if (h->has_model) {
    hipLaunchKernelGGL(k_vel_gyro_to_model, dim3(vgrid(h->batch)), dim3(64), 0, h->stream, vbufs(h));
    HIPCHK(hipGetLastError());
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_set_efforts(uwvk_vel* h, const double* tau, const double* cov) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !tau) return UWVK_EINVAL;
  if (!vfinite(tau, (size_t)h->batch * 6) || (cov && !vfinite(cov, (size_t)h->batch * 36))) return UWVK_ENAN;
  HIPCHK(hipMemcpyAsync(h->d_eff, tau, (size_t)h->batch * 6 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_predict(uwvk_vel* h, double dt) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->has_model) return UWVK_ENOMODEL;  // VelocityUKF.cpp:117-118
  hipLaunchKernelGGL(k_vel_predict, dim3(vgrid(h->batch)), dim3(64), 0, h->stream, vbufs(h), h->P, dt);
  HIPCHK(hipGetLastError());
  return UWVK_OK;
}

static uwvk_status vel_update(uwvk_vel* h, int m, const double* mu, const double* cov, const double* shared_cov,
                              const uint8_t* mask) {
  if (!h || !mu || (!cov && !shared_cov)) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  const int64_t B = h->batch;
  for (int64_t i = 0; i < B; i++) {
    if (mask && !mask[i]) continue;
    if (!vfinite(mu + i * m, m) || (cov && !vfinite(cov + i * m * m, (size_t)m * m))) return UWVK_ENAN;
  }
  if (!cov && !vfinite(shared_cov, (size_t)m * m)) return UWVK_ENAN;
  double* dz = h->d_meas;
  double* dc = h->d_meas + B * 3;
  HIPCHK(hipMemcpyAsync(dz, mu, (size_t)B * m * 8, hipMemcpyHostToDevice, h->stream));
  const double* dcov = nullptr;
  if (cov) {
    HIPCHK(hipMemcpyAsync(dc, cov, (size_t)B * m * m * 8, hipMemcpyHostToDevice, h->stream));
    dcov = dc;
  }
  double* dshared = h->d_meas + B * 12 - 9;
  if (!cov) HIPCHK(hipMemcpyAsync(dshared, shared_cov, (size_t)m * m * 8, hipMemcpyHostToDevice, h->stream));
  const uint8_t* dmask = nullptr;
  if (mask) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)B, hipMemcpyHostToDevice, h->stream));
    dmask = h->d_mask;
  }
  if (m == 3)
    hipLaunchKernelGGL((k_vel_update<3, 0>), dim3(vgrid(B)), dim3(64), 0, h->stream, vbufs(h), dz, dcov, h->P, 0.0,
                       dshared, dmask);
  else
    hipLaunchKernelGGL((k_vel_update<1, 3>), dim3(vgrid(B)), dim3(64), 0, h->stream, vbufs(h), dz, dcov, h->P, 0.0,
                       dshared, dmask);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_update_dvl(uwvk_vel* h, const double* mu, const double* cov, const double* sc,
                                const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  return vel_update(h, 3, mu, cov, sc, mask);
}
uwvk_status uwvk_vel_update_pressure(uwvk_vel* h, const double* mu, const double* cov, const double* sc,
                                     const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  return vel_update(h, 1, mu, cov, sc, mask);
}

uwvk_status uwvk_vel_get_state(uwvk_vel* h, double* x, double* P) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !x) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(x, h->d_mu, (size_t)h->batch * 4 * 8, hipMemcpyDeviceToHost, h->stream));
  if (P) HIPCHK(hipMemcpyAsync(P, h->d_sigma, (size_t)h->batch * 16 * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_get_model_state(uwvk_vel* h, double* out) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !out) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(out, h->d_model, (size_t)h->batch * 13 * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_vel_run_log(uwvk_vel* h, const uwvk_vel_log* log, int64_t first, int64_t count) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !log || first < 0 || count < 0 || first + count > log->epochs) return UWVK_EINVAL;
  if (!h->has_model) return UWVK_ENOMODEL;
  VelEpochArgs ea{};
  ea.flags = log->flags; ea.gyro = log->gyro; ea.efforts = log->efforts;
  ea.dvl_index = log->dvl_index; ea.dvl = log->dvl;
  std::memcpy(ea.dvl_cov, log->dvl_cov, sizeof(ea.dvl_cov));
  ea.p_index = log->pressure_index; ea.pressure = log->pressure; ea.p_cov = log->pressure_cov;
  ea.dt = log->dt;
  // one launch per chunk of epochs (state stays in registers across the chunk)
  const bool groups = h->groups > 0 || (h->groups < 0 && h->batch <= kVelGroupsMaxBatch);
  constexpr int64_t kChunk = 4096;
  for (int64_t e = first; e < first + count; e += kChunk) {
    ea.first = e;
    ea.count = std::min<int64_t>(kChunk, first + count - e);
    if (groups && h->groups == 2)
      hipLaunchKernelGGL(k_vel_epoch_g<32>, dim3((unsigned)((h->batch + 1) / 2)), dim3(64), 0, h->stream, vbufs(h),
                         h->P, ea);
    else if (groups)
      hipLaunchKernelGGL(k_vel_epoch_g<16>, dim3((unsigned)((h->batch + 3) / 4)), dim3(64), 0, h->stream, vbufs(h),
                         h->P, ea);
    else
      hipLaunchKernelGGL(k_vel_epoch, dim3(vgrid(h->batch)), dim3(64), 0, h->stream, vbufs(h), h->P, ea);
    HIPCHK(hipGetLastError());
  }
  return UWVK_OK;
}

}  // extern "C"
