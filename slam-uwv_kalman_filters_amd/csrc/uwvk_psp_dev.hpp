// uwvk_psp_dev.hpp — partitioned sigma-point (PSP) PoseUKF: the same unscented
// transform as ukfom's (frozen spec), evaluated in O(n^2) per step.
//
// Why this is exact.  ukfom spreads X_0 = mu, X_{2j+1,2j+2} = mu [+] +-L_j with
// L the lower Cholesky factor of Sigma.  Let a model g (process model or
// measurement function) depend NON-affinely only on tangent DOFs < k (for fixed
// values of those, g is affine in the rest).  Column j >= k of a lower
// triangular L is zero in rows < k, so X_{j,+-} agrees with mu bitwise on every
// DOF g is non-affine in, and g(X_{j,+-}) = g(mu) +- J L_j with J the constant
// Jacobian of the affine part.  Substituting into ukfom's mean (weights 1/N) and
// covariances (weight 1/2, all 2n+1 points) gives, in exact arithmetic:
//   predict (k = 15: orientation depends on pos.x, q, gyro bias):
//     lin x lin = A Sigma A^T          (A: I + dt couplings + decays)
//     ori x lin = 1/2 A L_a Delta       (Delta_j = d_{j+} - d_{j-}, j < k)
//     ori x ori = 1/2 [sum_{2k pts} d d^T + (1 + 2(n-k)) c c^T]
//   update (k per model, H = Jacobian of the affine part at mu):
//     zbar = z_0 + (1/N) sum_{2k pts} (z_p - z_0)
//     S = 1/2 [sum_{2k} dz dz^T + (1 + 2(n-k)) e e^T] + H (Sigma - L_a L_a^T) H^T + R
//     C = 1/2 sum_{j<k} L_j (z_{j+} - z_{j-})^T + (Sigma - L_a L_a^T) H^T
// with L_a the first k columns of L (a k-step partial Cholesky).  Only 2k+1
// model evaluations and O(n^2) covariance algebra remain; results equal the
// literal spread to rounding (parity tests run both paths against the oracle).
// The literal path (uwvk_pose_dev.hpp) stays selectable: UWVK_OPT_DENSE_SIGMA.
//
// Execution: one wavefront (64 lanes) per filter instance, Sigma packed
// (lower triangle, row i at i(i+1)/2) in LDS for the whole multi-epoch run.
#pragma once
#include "uwvk_pose_dev.hpp"

namespace uwvk {
namespace psp {

template <int DOF>
struct PG {
  static constexpr int NP = DOF * (DOF + 1) / 2;     // packed entries
  static constexpr int NSLOT = (NP + 63) / 64;       // flat slots per lane
  static constexpr int N = 2 * DOF + 1;              // ukfom sigma points
  static constexpr int KP = 15;                      // predict: nonlinear prefix (pos.x .. gyro bias)
  static constexpr int STG = 128;                    // staged rows of L_a for the point lanes
  static constexpr int WS = 64 + 6 * DOF;            // work area (Delta/X or dz/C/K)
};

template <int DOF>
struct alignas(16) PspSmem {
  double S[PG<DOF>::NP];  // Sigma, packed lower triangle
  double mu[56];          // mean (store layout)
  double stg[PG<DOF>::STG];
  double W[PG<DOF>::WS];
  double vec[64];         // delta / small broadcasts
  double ad[64];          // predict: diagonal of the process Jacobian A per DOF
  double off[32];         // per-instance model-parameter / density offsets (loaded once)
  double H[32];           // update: affine Jacobian H[i][t] (M x NC)
  double P[64];           // update: P = H L_a (M x K), then Dz/2 - P (K x M)
};

UWVK_DEV constexpr int pidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// flat packed index e -> (i, j), i >= j
UWVK_DEV void unpack(int e, int& i, int& j) {
  int r = (int)((__builtin_sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if ((r + 1) * (r + 2) / 2 <= e) r++;
  if (r * (r + 1) / 2 > e) r--;
  i = r;
  j = e - r * (r + 1) / 2;
}

// lane id that the optimiser cannot treat as loop-invariant: phases inside the
// multi-epoch loop recompute their lane-derived addresses instead of having
// LICM hoist hundreds of them out of the epoch loop (register blow-up)
UWVK_DEV int olane() {
  int l = (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;
}

UWVK_DEV void psync() {  // LDS ordering point for the single wave of the block
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------------
// k-column partial Cholesky, lane r owns row r: a[c] = L[r][c] (0 above the
// diagonal).  Right-looking; L[c][J] is broadcast from lane c's registers.
// ---------------------------------------------------------------------------
template <int K, int J>
UWVK_DEV void pchol_step(double (&a)[K], int r, bool& ok) {
  if constexpr (J < K) {
    const double piv = readlane_d(a[J], J);
    ok = ok && (piv > 0.0);
    const double inv = rsqrt_f64(piv);
    a[J] = (r == J) ? piv * inv : (r > J ? a[J] * inv : 0.0);
#pragma unroll
    for (int c = J + 1; c < K; c++) a[c] -= a[J] * readlane_d(a[J], c);
#pragma unroll
    for (int c = J + 1; c < K; c++) asm volatile("" : "+v"(a[c]));
    pchol_step<K, J + 1>(a, r, ok);
  }
}

template <int DOF, int K>
UWVK_DEV bool pchol(const double* S, int r, double (&a)[K]) {
  const int rr = r < DOF ? r : DOF - 1;
#pragma unroll
  for (int c = 0; c < K; c++) a[c] = S[pidx(rr, c)];
  bool ok = true;
  pchol_step<K, 0>(a, r, ok);
  return ok;
}

// row list helpers (compile-time lists of tangent DOFs)
template <int NR>
UWVK_DEV constexpr int row_pos(const int (&rows)[NR], int d) {
  for (int q = 0; q < NR; q++)
    if (rows[q] == d) return q;
  return -1;
}

// lanes owning rows in ROWS write L[r][0..K) into stg[q*K + j]
template <class RL, int K>
UWVK_DEV void stage_rows(double* stg, int r, const double (&a)[K]) {
#pragma unroll
  for (int q = 0; q < RL::NR; q++) {
    if (r == RL::rows[q]) {
#pragma unroll
      for (int j = 0; j < K; j++) stg[q * K + j] = a[j];
    }
  }
}

// point p (< 2K: column p>>1, sign + for even p; p == 2K: centre) restricted to
// the DOFs in RL::rows (template recursion: every register index is constant);
// the other entries of x keep mu.
template <class RL, int DOF, int K, int Q>
UWVK_DEV void gen_rows_q(const double* mu, const double* stg, int j, double sg, double (&v)[3], double* x) {
  if constexpr (Q < RL::NR) {
    constexpr int d = RL::rows[Q];
    const double l = stg[Q * K + j];
    if constexpr (d >= 3 && d < 6) {
      v[d - 3] = sg * l;
    } else {
      x[d2s(d)] = mu[d2s(d)] + sg * l;
    }
    gen_rows_q<RL, DOF, K, Q + 1>(mu, stg, j, sg, v, x);
  }
}
template <class RL>
UWVK_DEV constexpr bool has_rot() {
  for (int q = 0; q < RL::NR; q++)
    if (RL::rows[q] >= 3 && RL::rows[q] < 6) return true;
  return false;
}
template <class RL, int DOF, int K>
UWVK_DEV void gen_rows(const double* mu, const double* stg, int p, double x[Lay<DOF>::store]) {
  using L = Lay<DOF>;
#pragma unroll
  for (int s = 0; s < L::store; s++) x[s] = mu[s];
  if constexpr (K > 0) {
    const bool in = p < 2 * K;
    const int j = in ? (p >> 1) : 0;
    const double sg = in ? ((p & 1) ? -1.0 : 1.0) : 0.0;  // the centre: mu + 0 (bitwise mu)
    double v[3] = {0.0, 0.0, 0.0};
    gen_rows_q<RL, DOF, K, 0>(mu, stg, j, sg, v, x);
    if constexpr (has_rot<RL>()) {
      double e[4];
      so3_exp(v, e);
      qmul(e, mu + L::s_quat, x + L::s_quat);
    }
  }
}

// ---------------------------------------------------------------------------
// Process model pieces (PoseUKF.cpp:12-84), bitwise the same expressions as
// process_point() in uwvk_pose_dev.hpp.
// ---------------------------------------------------------------------------
template <int DOF>
UWVK_DEV void proc_orientation(const double x[Lay<DOF>::store], const PoseShared& sh, const ProcCtx& c, double o[4]) {
  using L = Lay<DOF>;
  const double lat = sh.lat0 + x[L::s_pos] * sh.inv_rm;
  double sl, cl;
  sincos(lat, &sl, &cl);
  const double er[3] = {kEarthW * cl, 0.0, kEarthW * sl};
  double wb[3], wn[3];
#pragma unroll
  for (int i = 0; i < 3; i++) wb[i] = c.w[i] - x[L::s_bg + i];
  qrot(x + L::s_quat, wb, wn);
#pragma unroll
  for (int i = 0; i < 3; i++) wn[i] = (wn[i] - er[i]) * c.dt;
  double e[4];
  so3_exp(wn, e);
  qmul(e, x + L::s_quat, o);
}

// storage component s (not orientation) of f(mu)
template <int DOF>
UWVK_DEV double proc_vect(int s, const double* mu, const PoseShared& sh, const ProcCtx& c) {
  using L = Lay<DOF>;
  const uwvk_pose_parameter& P = sh.p;
  const double dt = c.dt, x = mu[s];
  if (s < 3) return x + dt * mu[L::s_vel + s];
  if (s >= L::s_vel && s < L::s_vel + 3) return x + dt * mu[L::s_acc + s - L::s_vel];
  if (s >= L::s_bg && s < L::s_bg + 3) {
    const double d = sh.ntau[0] * (x - P.gyro_bias_offset[s - L::s_bg]);
    return x + dt * d;
  }
  if (s >= L::s_ba && s < L::s_ba + 3) {
    const double d = sh.ntau[1] * (x - P.acc_bias_offset[s - L::s_ba]);
    return x + dt * d;
  }
  if constexpr (L::has_params) {
    if (s >= L::s_inertia && s < L::s_inertia + 9) {
      const double d = sh.ntau[2] * (x - c.off[s - L::s_inertia]);
      return x + dt * d;
    }
    if (s >= L::s_lin && s < L::s_lin + 9) {
      const double d = sh.ntau[3] * (x - c.off[9 + s - L::s_lin]);
      return x + dt * d;
    }
    if (s >= L::s_quad && s < L::s_quad + 9) {
      const double d = sh.ntau[4] * (x - c.off[18 + s - L::s_quad]);
      return x + dt * d;
    }
  }
  if (s >= L::s_wv && s < L::s_wv + 4) {
    const double d = sh.ntau[5] * x;
    return x + dt * d;
  }
  if (s >= L::s_badcp && s < L::s_badcp + 2) {
    const double d = sh.ntau[6] * x;
    return x + dt * d;
  }
  if (s == L::s_rho) {
    const double d = sh.ntau[7] * (x - c.off[27]);
    return x + dt * d;
  }
  return x;  // acceleration, gravity
}

// Jacobian of the affine rows of f: A = diag(ad) + dt * (pos <- vel, vel <- acc)
template <int DOF>
UWVK_DEV double proc_diag(int d, const PoseShared& sh, double dt) {
  using L = Lay<DOF>;
  if (d >= L::d_bg && d < L::d_bg + 3) return 1.0 + dt * sh.ntau[0];
  if (d >= L::d_ba && d < L::d_ba + 3) return 1.0 + dt * sh.ntau[1];
  if constexpr (L::has_params) {
    if (d >= L::d_inertia && d < L::d_inertia + 9) return 1.0 + dt * sh.ntau[2];
    if (d >= L::d_lin && d < L::d_lin + 9) return 1.0 + dt * sh.ntau[3];
    if (d >= L::d_quad && d < L::d_quad + 9) return 1.0 + dt * sh.ntau[4];
  }
  if (d >= L::d_wv && d < L::d_wv + 4) return 1.0 + dt * sh.ntau[5];
  if (d >= L::d_badcp && d < L::d_badcp + 2) return 1.0 + dt * sh.ntau[6];
  if (d == L::d_rho) return 1.0 + dt * sh.ntau[7];
  return 1.0;
}
// coupled column of row d (pos -> vel, vel -> acc) or -1
UWVK_DEV constexpr int proc_couple(int d) { return d < 3 ? d + 6 : (d >= 6 && d < 9 ? d + 3 : -1); }

// DOFs the orientation row of the process model reads (lat from pos.x, q, b_g)
struct PredRows {
  static constexpr int NR = 7;
  static constexpr int rows[NR] = {0, 3, 4, 5, 12, 13, 14};
};

// ---------------------------------------------------------------------------
// predictionStepImpl (PoseUKF.cpp:446-474) + ukf::predict, PSP form
// ---------------------------------------------------------------------------
// Q: process_noise_cov (DOF x DOF); Qp: dt^2 Q in packed order (host-made per dt)
template <int DOF>
UWVK_DEV bool psp_predict(PspSmem<DOF>& sm, const PoseShared& sh, const ProcCtx& pc, const double* Q,
                          const double* Qp, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int K = G::KP;
  const int l = olane();
  const double dt = pc.dt, dt2 = dt * dt;
  // process-noise shaping from the pre-predict mean (PoseUKF.cpp:448-460)
  if (l < 9) {
    double R[9];
    qmatrix(sm.mu + L::s_quat, R);
    const int r = l / 3, c = l % 3;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      double u = 0.0;
#pragma unroll
      for (int m = 0; m < 3; m++) u += R[r * 3 + m] * sh.q_ori[m * 3 + k];
      s += u * R[c * 3 + k];
    }
    sm.vec[48 + l] = s;
  }
  if (l < DOF) sm.ad[l] = proc_diag<DOF>(l, sh, dt);
  const double vs0 = sm.mu[L::s_vel], vs1 = sm.mu[L::s_vel + 1], vs2 = 10 * sm.mu[L::s_vel + 2];
  const double wv_add = sh.p.water_velocity_scale * (vs0 * vs0 + vs1 * vs1 + vs2 * vs2) * dt;
  // partial Cholesky and row staging
  double a[K];
  const bool ok = pchol<DOF, K>(sm.S, l, a);
  stage_rows<PredRows, K>(sm.stg, l, a);
  psync();
  UWVK_STAMP(20);
  // sigma points: lanes < 2K plus the centre lane 2K; orientation output only
  const bool pt = l < 2 * K, ctr = l == 2 * K;
  double o[4];
  {
    double x[L::store];
    gen_rows<PredRows, DOF, K>(sm.mu, sm.stg, l, x);
    proc_orientation<DOF>(x, sh, pc, o);
  }
  UWVK_STAMP(21);
  // manifold mean of the orientations (ukfom: ref = X_0, Gauss-Newton, |d| <= 1e-6)
  constexpr double wc = 1.0 + 2.0 * (DOF - K);
  double mq[4];
#pragma unroll
  for (int i = 0; i < 4; i++) mq[i] = readlane_d(o[i], 2 * K);
  {
    int it = 0;
    double nrm;
    do {
      double d[3];
      qboxminus(o, mq, d);
      const double w = pt ? 1.0 : (ctr ? wc : 0.0);
      nrm = 0.0;
#pragma unroll
      for (int i = 0; i < 3; i++) {
        d[i] = wave_sum(w * d[i]) / (double)G::N;
        nrm += d[i] * d[i];
      }
      double e[4], q[4];
      so3_exp(d, e);
      qmul(e, mq, q);
#pragma unroll
      for (int i = 0; i < 4; i++) mq[i] = q[i];
      nrm = sqrt(nrm);
    } while (nrm > 1e-6 && ++it < 10000);
  }
  UWVK_STAMP(22);
  // deviations; ori x ori block; Delta_j = d_{j+} - d_{j-}
  double d[3];
  qboxminus(o, mq, d);
  double oo[6];
  {
    const double w = pt ? 1.0 : (ctr ? wc : 0.0);
    int k = 0;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) oo[k++] = 0.5 * wave_sum(w * d[i] * d[j]);
  }
  {
    double dn[3];
#pragma unroll
    for (int i = 0; i < 3; i++) dn[i] = shfl_xor_d(d[i], 1);
    if (pt && !(l & 1)) {
#pragma unroll
      for (int i = 0; i < 3; i++) sm.W[(l >> 1) * 3 + i] = d[i] - dn[i];
    }
  }
  psync();
  // ori x lin: X_r = 1/2 (A (L_a Delta))_r, lane r
  double X[3];
  {
    double Y[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int j = 0; j < K; j++)
#pragma unroll
      for (int i = 0; i < 3; i++) Y[i] += a[j] * sm.W[j * 3 + i];
    const int cp = proc_couple(l);
    const int src = cp >= 0 ? cp : l;
    const double ar = proc_diag<DOF>(l, sh, dt);
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const double yc = shfl_d(Y[i], src);
      X[i] = 0.5 * (cp >= 0 ? (ar * Y[i] + dt * yc) : ar * Y[i]);
    }
  }
  UWVK_STAMP(23);
  // rows/cols coupled by A (pos, vel): new values into registers first
  constexpr int pv[6] = {0, 1, 2, 6, 7, 8};
  double nv[6];
  const int jl = l < DOF ? l : DOF - 1;
  const int jc = proc_couple(jl);
  const double aj = proc_diag<DOF>(jl, sh, dt);
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const int r = pv[q], rc = proc_couple(r);
    const double t0 = aj * sm.S[pidx(r, jl)] + (jc >= 0 ? dt * sm.S[pidx(r, jc)] : 0.0);
    const double t1 = aj * sm.S[pidx(rc, jl)] + (jc >= 0 ? dt * sm.S[pidx(rc, jc)] : 0.0);
    nv[q] = t0 + dt * t1;  // A_rr = 1 for pos/vel rows
  }
  psync();
  if (l < DOF && !(l >= 3 && l < 6)) {
    const bool jpv = jc >= 0;
#pragma unroll
    for (int q = 0; q < 6; q++)
      if (!jpv || l <= pv[q]) sm.S[pidx(pv[q], l)] = nv[q];
  }
  if (l < DOF) {
#pragma unroll
    for (int i = 0; i < 3; i++) sm.W[64 + l * 3 + i] = X[i];
  }
  psync();
  UWVK_STAMP(24);
  // flat pass: ori rows/cols, decays, + Q' (packed dt^2 Q loads issued up front)
  {
    double qv[G::NSLOT];
#pragma unroll
    for (int t = 0; t < G::NSLOT; t++) {
      const int e = l + 64 * t;
      qv[t] = e < G::NP ? Qp[e] : 0.0;
    }
#pragma unroll
    for (int t = 0; t < G::NSLOT; t++) {
      const int e = l + 64 * t;
      if (e < G::NP) {
        int i, j;
        unpack(e, i, j);
        const bool io = i >= 3 && i < 6, jo = j >= 3 && j < 6;
        double v, q = qv[t];
        if (io && jo) {
          const int a2 = i - 3, b2 = j - 3;
          v = oo[a2 * (a2 + 1) / 2 + b2];
          q = dt2 * sm.vec[48 + a2 * 3 + b2];
        } else if (io) {
          v = sm.W[64 + j * 3 + (i - 3)];
        } else if (jo) {
          v = sm.W[64 + i * 3 + (j - 3)];
        } else if (proc_couple(i) >= 0 || proc_couple(j) >= 0) {
          v = sm.S[e];
        } else {
          v = sm.ad[i] * sm.ad[j] * sm.S[e];
        }
        if (i == j && i >= L::d_wv && i < L::d_wv + 4) q = dt2 * (sh.q_wv[i - L::d_wv] + wv_add);
        sm.S[e] = v + q;
      }
    }
  }
  UWVK_STAMP(25);
  // new mean: vect parts f(mu), orientation the manifold mean
  double mv = 0.0;
  if (l < L::store && !(l >= 3 && l < 7)) mv = proc_vect<DOF>(l, sm.mu, sh, pc);
  psync();
  if (l < L::store && !(l >= 3 && l < 7)) sm.mu[l] = mv;
  if (l < 4) sm.mu[3 + l] = mq[l];
  psync();
  UWVK_STAMP(26);
  return ok;
}

// ---------------------------------------------------------------------------
// measurement models in PSP form: K = nonlinear prefix, ROWS = DOFs eval reads
// (beyond mu), COLS = columns of the affine Jacobian H (COLS within ROWS)
// ---------------------------------------------------------------------------
template <int DOF>
struct PAcc {  // measurementAcceleration, PoseUKF.cpp:125-131
  using L = Lay<DOF>;
  static constexpr int M = 3, K = 6, NR = 10, NC = 7, ZMODE = 1, GATE = 0;
  static constexpr int rows[NR] = {3, 4, 5, 9, 10, 11, 15, 16, 17, 18};
  static constexpr int cols[NC] = {9, 10, 11, 15, 16, 17, 18};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { HAcc<DOF>{}(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);  // z = R^T (a + g e_z) + ba
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
      for (int i = 0; i < 3; i++) {
        H[r][i] = R[i * 3 + r];
        H[r][3 + i] = r == i ? 1.0 : 0.0;
      }
      H[r][6] = R[2 * 3 + r];
    }
  }
};
template <int DOF>
struct PVel {  // measurementVelocity, PoseUKF.cpp:117-123
  using L = Lay<DOF>;
  static constexpr int M = 3, K = 6, NR = 6, NC = 3, ZMODE = 1, GATE = 0;
  static constexpr int rows[NR] = {3, 4, 5, 6, 7, 8};
  static constexpr int cols[NC] = {6, 7, 8};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { HVel<DOF>{}(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int i = 0; i < 3; i++) H[r][i] = R[i * 3 + r];
  }
};
template <int DOF>
struct PPressure {  // measurementPressureSensor, PoseUKF.cpp:107-115 (p_z * g * rho: k = 19)
  using L = Lay<DOF>;
  static constexpr int M = 1, K = 19, NR = 6, NC = 1, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {2, 3, 4, 5, 18, L::d_rho};
  static constexpr int cols[NC] = {L::d_rho};
  HPressure<DOF> h;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { h(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double r[3];
    qrot(mu + L::s_quat, h.s, r);
    const double pz = mu[L::s_pos + 2] + r[2];
    H[0][0] = -(pz * mu[L::s_grav]);
  }
};
template <int DOF>
struct PWater {  // measurementWaterCurrents, PoseUKF.cpp:133-151
  using L = Lay<DOF>;
  static constexpr int M = 2, K = 6, NR = 12, NC = 9, ZMODE = 1, GATE = 1;
  static constexpr int rows[NR] = {3, 4, 5, 6, 7, 8, L::d_wv, L::d_wv + 1, L::d_wvb, L::d_wvb + 1,
                                   L::d_badcp, L::d_badcp + 1};
  static constexpr int cols[NC] = {6, 7, 8, L::d_wv, L::d_wv + 1, L::d_wvb, L::d_wvb + 1, L::d_badcp, L::d_badcp + 1};
  double cw;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const {
    HWater<DOF> h;
    h.cw = cw;
    h(x, z);
  }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);
#pragma unroll
    for (int r = 0; r < 2; r++) {
#pragma unroll
      for (int i = 0; i < 3; i++) H[r][i] = cw * R[i * 3 + r] + (1 - cw) * R[i * 3 + r];
#pragma unroll
      for (int i = 0; i < 2; i++) {
        H[r][3 + i] = -((1 - cw) * R[i * 3 + r]);
        H[r][5 + i] = -(cw * R[i * 3 + r]);
        H[r][7 + i] = r == i ? 1.0 : 0.0;
      }
    }
  }
};
template <int DOF>
struct PXY {  // measurementXYPosition, PoseUKF.cpp:87-92: linear (k = 0)
  static constexpr int M = 2, K = 0, NR = 2, NC = 2, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {0, 1};
  static constexpr int cols[NC] = {0, 1};
  int gate = 0;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { z[0] = x[0]; z[1] = x[1]; }
  UWVK_DEV void jac(const double*, double (&H)[M][NC]) const { H[0][0] = 1; H[0][1] = 0; H[1][0] = 0; H[1][1] = 1; }
};
template <int DOF>
struct PZ {  // measurementZPosition, PoseUKF.cpp:100-105: linear (k = 0)
  static constexpr int M = 1, K = 0, NR = 1, NC = 1, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {2};
  static constexpr int cols[NC] = {2};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { z[0] = x[2]; }
  UWVK_DEV void jac(const double*, double (&H)[M][NC]) const { H[0][0] = 1; }
};

// ---------------------------------------------------------------------------
// ukf::update [EXT], PSP form.  gate: 0 accept any, 1 d2p95.  Returns the gate
// decision; *ok = false on a non-positive pivot of the partial Cholesky.
// ---------------------------------------------------------------------------
template <int DOF, class HM>
UWVK_DEV bool psp_update(PspSmem<DOF>& sm, const double (&z)[HM::M], const double (&Rm)[HM::M * HM::M], int gate,
                         const HM& hm, bool* ok, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int M = HM::M, K = HM::K, NC = HM::NC, KA = K > 0 ? K : 1;
  const int l = olane();
  double a[KA];
  bool cok = true;
  if constexpr (K > 0) {
    cok = pchol<DOF, K>(sm.S, l, a);
    stage_rows<HM, K>(sm.stg, l, a);
    psync();
  }
  UWVK_STAMP(30);
  const bool pt = l < 2 * K;
  double zp[M];
  {
    double x[L::store];
    gen_rows<HM, DOF, K>(sm.mu, sm.stg, l, x);
    hm.eval(x, zp);
  }
  double zc[M], zb[M], e[M];
#pragma unroll
  for (int i = 0; i < M; i++) zc[i] = readlane_d(zp[i], 2 * K);
  // zbar = z_0 + (1/N) sum_{2K} (z_p - z_0)  (the linear pairs cancel)
#pragma unroll
  for (int i = 0; i < M; i++) {
    const double s = K > 0 ? wave_sum(pt ? zp[i] - zc[i] : 0.0) : 0.0;
    zb[i] = zc[i] + s / (double)G::N;
    e[i] = zc[i] - zb[i];
  }
  double dz[M];
#pragma unroll
  for (int i = 0; i < M; i++) dz[i] = zp[i] - zb[i];
  constexpr double wc = 1.0 + 2.0 * (DOF - K);
  double S[M * M];
#pragma unroll
  for (int i = 0; i < M; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      const double s = K > 0 ? wave_sum(pt ? dz[i] * dz[j] : 0.0) : 0.0;
      S[i * M + j] = 0.5 * (s + wc * e[i] * e[j]);
    }
  // Delta z_j = z_{j+} - z_{j-}, staged as W[j*M + i]
  if constexpr (K > 0) {
    double zn[M];
#pragma unroll
    for (int i = 0; i < M; i++) zn[i] = shfl_xor_d(zp[i], 1);
    if (pt && !(l & 1)) {
#pragma unroll
      for (int i = 0; i < M; i++) sm.W[(l >> 1) * M + i] = zp[i] - zn[i];
    }
  }
  UWVK_STAMP(31);
  // affine part: H at mu (staged), P = H L_a and Qp = Dz/2 - P lane-parallel,
  // G = Sigma H^T (lane r).  Uniform matrices live in LDS, not in VGPRs.
  if (l == 0) {
    double H[M][NC];
    hm.jac(sm.mu, H);
#pragma unroll
    for (int i = 0; i < M; i++)
#pragma unroll
      for (int t = 0; t < NC; t++) sm.H[i * NC + t] = H[i][t];
  }
  psync();
  if constexpr (K > 0) {
    if (l < M * K) {
      const int i = l / K, j = l - (l / K) * K;
      double s = 0.0;
#pragma unroll
      for (int t = 0; t < NC; t++) s += sm.H[i * NC + t] * sm.stg[row_pos(HM::rows, HM::cols[t]) * K + j];
      sm.P[i * K + j] = s;
    }
  }
  const int rl = l < DOF ? l : DOF - 1;
  double Gr[M];
#pragma unroll
  for (int i = 0; i < M; i++) Gr[i] = 0.0;
#pragma unroll
  for (int t = 0; t < NC; t++) {
    const double s = sm.S[pidx(rl, HM::cols[t])];
#pragma unroll
    for (int i = 0; i < M; i++) Gr[i] += s * sm.H[i * NC + t];
  }
  psync();
  UWVK_STAMP(32);
  // C_r = G_r + sum_j L[r][j] (Dz_j / 2 - P[:, j])
  double C[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    double s = Gr[i];
    if constexpr (K > 0) {
#pragma unroll
      for (int j = 0; j < K; j++) s += a[j] * (0.5 * sm.W[j * M + i] - sm.P[i * K + j]);
    }
    C[i] = s;
  }
  // S += H G - P P^T + R
#pragma unroll
  for (int i = 0; i < M; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      double hg = 0.0;
#pragma unroll
      for (int t = 0; t < NC; t++) hg += sm.H[i * NC + t] * readlane_d(Gr[j], HM::cols[t]);
      double pp = 0.0;
      if constexpr (K > 0) {
#pragma unroll
        for (int k = 0; k < K; k++) pp += sm.P[i * K + k] * sm.P[j * K + k];
      }
      const double s = S[i * M + j] + (hg - pp);
      S[i * M + j] = s + Rm[i * M + j];
      if (j != i) S[j * M + i] = s + Rm[j * M + i];
    }
  double Si[M * M];
  small_inv<M>(S, Si);
  double Kg[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < M; j++) s += C[j] * Si[j * M + i];
    Kg[i] = s;
  }
  double nu[M];
#pragma unroll
  for (int i = 0; i < M; i++) nu[i] = z[i] - zb[i];
  double d2 = 0.0;
#pragma unroll
  for (int j = 0; j < M; j++) {
    double u = 0.0;
#pragma unroll
    for (int i = 0; i < M; i++) u += nu[i] * Si[i * M + j];
    d2 += u * nu[j];
  }
  *ok = cok;
  const bool accept = gate == 0 ? true : !(d2 > kD2P95);
  if (!accept) return false;
  UWVK_STAMP(33);
  // Sigma -= C K^T (flat), delta = K nu
  psync();
  if (l < DOF) {
#pragma unroll
    for (int i = 0; i < M; i++) {
      sm.W[l * 2 * M + i] = C[i];
      sm.W[l * 2 * M + M + i] = Kg[i];
    }
    double dl = 0.0;
#pragma unroll
    for (int i = 0; i < M; i++) dl += Kg[i] * nu[i];
    sm.vec[l] = dl;
  }
  psync();
#pragma unroll 1
  for (int t = 0; t < G::NSLOT; t++) {
    const int ee = l + 64 * t;
    if (ee < G::NP) {
      int i, j;
      unpack(ee, i, j);
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < M; k++) s += sm.W[i * 2 * M + k] * sm.W[j * 2 * M + M + k];
      sm.S[ee] -= s;
    }
  }
  psync();
  UWVK_STAMP(34);
  // apply_delta, exact nav-frame form: mu <- mu [+] delta, Sigma <- T Sigma T^T
  {
    double R[9];
    {
      const double dv[3] = {sm.vec[3], sm.vec[4], sm.vec[5]};
      double eq[4];
      so3_exp(dv, eq);
      qmatrix(eq, R);
    }
    // rows 3..5 of every column j outside the block
    if (l < DOF && !(l >= 3 && l < 6)) {
      const double s0 = sm.S[pidx(3, l)], s1 = sm.S[pidx(4, l)], s2 = sm.S[pidx(5, l)];
#pragma unroll
      for (int i = 0; i < 3; i++) sm.S[pidx(3 + i, l)] = R[i * 3] * s0 + R[i * 3 + 1] * s1 + R[i * 3 + 2] * s2;
    }
    // ori x ori: R B R^T
    double nb = 0.0;
    if (l < 9) {
      const int r = l / 3, c = l % 3;
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < 3; u++) {
        double t = 0.0;
#pragma unroll
        for (int v = 0; v < 3; v++) t += sm.S[pidx(3 + u, 3 + v)] * R[c * 3 + v];
        s += R[r * 3 + u] * t;
      }
      nb = s;
    }
    double mnew = 0.0;
    if (l < L::store && !(l >= 3 && l < 7)) {
      const int d = l < 3 ? l : l - 1;
      mnew = sm.mu[l] + 1.0 * sm.vec[d];
    }
    double qn[4];
    {
      double eq[4];
      const double dv[3] = {sm.vec[3], sm.vec[4], sm.vec[5]};
      so3_exp(dv, eq);
      qmul(eq, sm.mu + L::s_quat, qn);
    }
    psync();
    if (l < 9 && (l / 3) >= (l % 3)) sm.S[pidx(3 + l / 3, 3 + l % 3)] = nb;
    if (l < L::store && !(l >= 3 && l < 7)) sm.mu[l] = mnew;
    if (l < 4) sm.mu[3 + l] = qn[l];
    psync();
  }
  UWVK_STAMP(35);
  return true;
}

}  // namespace psp
}  // namespace uwvk
