// uwvk_aug_dev.hpp — generic lane-group UKF for the small and the
// marker-augmented filters on gfx950:
//   BottomUKF                  n = 3  (distance + S2 normal)      N = 7   -> 8 lanes
//   IndirectPoseUKF            n = 6  (position + SO3 error)      N = 13  -> 16 lanes
//   IndirectPoseUKF + marker   n = 12 (visual update)             N = 25  -> 32 lanes
//   PoseUKF + marker           n = 59 / 32 (visual update)        N = 119 / 65 -> 128 lanes
//
// Layout: G lanes (a power of two >= N) own one filter instance, ONE SIGMA
// POINT PER LANE; IPB = 64 / G instances share a 64-lane block (G <= 64), or
// one instance spans a G-lane block (G = 128).  Sigma, the Cholesky factor and
// the deviation matrix live in LDS; sigma points, process and measurement
// models live in VGPRs.  Cross-lane sums go through LDS (lane r < n owns row r
// of every n x n / n x m result), fp64 throughout.
//
// Semantics follow ukfom::ukf [EXT] as frozen in DESIGN.md §3 (items 1-4) and
// the CPU oracle oracle/uwvk_small_oracle.c (citations there), including the
// literal apply_delta re-spread (no closed-form shortcut: the S2 segment has
// no exact rotation identity).  S2 is DESIGN.md §3 item 11.
#pragma once
#include "uwvk_dev.hpp"

namespace uwvk {
namespace aug {

// SEG_SO3R: SO3 with the body-frame (right) [+] / [-], q exp(d) and log(b^-1 a)
// (the PoseUKF visual update under UWVK_OPT_SO3_RIGHT); SEG_SO3 the nav-frame one
enum { SEG_V = 0, SEG_SO3 = 1, SEG_S2 = 2, SEG_SO3R = 3 };

template <int K, int D = 0>
struct Seg {
  static constexpr int kind = K;
  static constexpr int dof = K == SEG_V ? D : (K == SEG_S2 ? 2 : 3);
  static constexpr int store = K == SEG_V ? D : (K == SEG_S2 ? 3 : 4);
};

// ---- S2 [EXT MTK S2], DESIGN.md §3 item 11 ---------------------------------
// R_x = minimal rotation e3 -> x, columns (b1, b2, x)
UWVK_DEV void s2_basis(const double x[3], double b1[3], double b2[3]) {
  const double k = 1.0 / (1.0 + x[2]);
  b1[0] = 1.0 - x[0] * x[0] * k; b1[1] = -x[0] * x[1] * k; b1[2] = -x[0];
  b2[0] = -x[0] * x[1] * k; b2[1] = 1.0 - x[1] * x[1] * k; b2[2] = -x[1];
}
// x [+] s d = R_x (sinc|sd| sd, cos|sd|)
UWVK_DEV void s2_boxplus(const double x[3], const double d[2], double s, double o[3]) {
  const double a = s * d[0], b = s * d[1];
  const double t = sqrt(a * a + b * b);
  double sn, c;
  sincos(t, &sn, &c);
  const double sc = t == 0.0 ? 1.0 : sn / t;
  double b1[3], b2[3], r[3];
  s2_basis(x, b1, b2);
#pragma unroll
  for (int i = 0; i < 3; i++) r[i] = b1[i] * (sc * a) + b2[i] * (sc * b) + x[i] * c;
  o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
}
// y [-] x = log(R_x^T y)
UWVK_DEV void s2_boxminus(const double y[3], const double x[3], double o[2]) {
  double b1[3], b2[3];
  s2_basis(x, b1, b2);
  const double w1 = b1[0] * y[0] + b1[1] * y[1] + b1[2] * y[2];
  const double w2 = b2[0] * y[0] + b2[1] * y[1] + b2[2] * y[2];
  const double w3 = x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
  const double nn = sqrt(w1 * w1 + w2 * w2);
  if (nn == 0.0) { o[0] = 0.0; o[1] = 0.0; return; }
  const double k = atan2(nn, w3) / nn;
  o[0] = k * w1; o[1] = k * w2;
}
// MTK::S2(v): normalised
UWVK_DEV void s2_from(const double v[3], double o[3]) {
  const double nn = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  o[0] = v[0] / nn; o[1] = v[1] / nn; o[2] = v[2] / nn;
}

// ---- compound manifold over a segment list ---------------------------------
template <int DI, int SI>
UWVK_DEV void bplus(const double*, const double*, double, double*) {}
template <int DI, int SI, class S0, class... R>
UWVK_DEV void bplus(const double* x, const double* d, double s, double* o) {
  if constexpr (S0::kind == SEG_V) {
#pragma unroll
    for (int k = 0; k < S0::dof; k++) o[SI + k] = x[SI + k] + s * d[DI + k];
  } else if constexpr (S0::kind == SEG_SO3 || S0::kind == SEG_SO3R) {
    double v[3] = {s * d[DI], s * d[DI + 1], s * d[DI + 2]}, e[4], r[4];
    so3_exp(v, e);
    if constexpr (S0::kind == SEG_SO3R) qmul(x + SI, e, r);
    else qmul(e, x + SI, r);
#pragma unroll
    for (int k = 0; k < 4; k++) o[SI + k] = r[k];
  } else {
    double r[3];
    s2_boxplus(x + SI, d + DI, s, r);
#pragma unroll
    for (int k = 0; k < 3; k++) o[SI + k] = r[k];
  }
  bplus<DI + S0::dof, SI + S0::store, R...>(x, d, s, o);
}

template <int DI, int SI>
UWVK_DEV void bminus(const double*, const double*, double*) {}
template <int DI, int SI, class S0, class... R>
UWVK_DEV void bminus(const double* a, const double* b, double* o) {
  if constexpr (S0::kind == SEG_V) {
#pragma unroll
    for (int k = 0; k < S0::dof; k++) o[DI + k] = a[SI + k] - b[SI + k];
  } else if constexpr (S0::kind == SEG_SO3) {
    qboxminus(a + SI, b + SI, o + DI);
  } else if constexpr (S0::kind == SEG_SO3R) {
    double bc[4] = {b[SI], -b[SI + 1], -b[SI + 2], -b[SI + 3]}, r[4];
    qmul(bc, a + SI, r);
    so3_log(r, o + DI);
  } else {
    s2_boxminus(a + SI, b + SI, o + DI);
  }
  bminus<DI + S0::dof, SI + S0::store, R...>(a, b, o);
}

template <class... S>
struct Manifold {
  static constexpr int dof = (S::dof + ... + 0);
  static constexpr int store = (S::store + ... + 0);
  UWVK_DEV static void boxplus(const double* x, const double* d, double s, double* o) {
    bplus<0, 0, S...>(x, d, s, o);
  }
  UWVK_DEV static void boxminus(const double* a, const double* b, double* o) { bminus<0, 0, S...>(a, b, o); }
};

// measurement manifolds (oracle: Z_VEC / Z_VECT_MANIFOLD / Z_S2)
enum { Z_VEC = 0, Z_VECT = 1, Z_S2 = 2 };

constexpr int pow2_at_least(int v) { return v <= 8 ? 8 : (v <= 16 ? 16 : (v <= 32 ? 32 : (v <= 64 ? 64 : 128))); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------
// Engine<M>: per-instance LDS layout and the group-cooperative UKF steps.
// Every member is called by ALL threads of the block (they contain barriers).
// ---------------------------------------------------------------------------
template <class M>
struct Engine {
  static constexpr int n = M::dof, S = M::store, N = 2 * n + 1;
  static constexpr int G = pow2_at_least(N);
  static constexpr int IPB = G >= 64 ? 1 : 64 / G;
  static constexpr int BLOCK = G >= 64 ? G : 64;
  // per-instance LDS words (doubles)
  static constexpr int o_sig = 0;                  // n x n, full symmetric
  static constexpr int o_wd = o_sig + n * n;       // Cholesky work (n x n) | deviations D (N x n)
  static constexpr int o_z = o_wd + cmax(n * n, N * n);  // Z points (N x 3) then dZ (N x 2)
  static constexpr int o_dz = o_z + 3 * N;
  static constexpr int o_k = o_dz + 2 * N;         // gain K (n x 2)
  static constexpr int o_vec = o_k + 2 * n;        // mean step / delta (n)
  static constexpr int o_mu = o_vec + n;           // mu (S)
  static constexpr int o_ref = o_mu + S;           // mean iterate broadcast (S)
  static constexpr int o_flag = o_ref + S;         // [0] Cholesky ok, [1] mean done
  static constexpr int words = o_flag + 2;

  double* sm;  // this instance's LDS words
  int g;       // lane within the group (sigma point index)
  bool live;   // instance < batch

  UWVK_DEV double& sig(int r, int c) { return sm[o_sig + r * n + c]; }
  UWVK_DEV double& W(int r, int c) { return sm[o_wd + r * n + c]; }
  UWVK_DEV double& D(int p, int r) { return sm[o_wd + p * n + r]; }

  // lower Cholesky of Sigma into W (right-looking, lane r owns row r).
  // Returns the group's success flag (non-positive pivot -> false).
  UWVK_DEV bool cholesky() {
    for (int i = g; i < n * n; i += G) sm[o_wd + i] = sm[o_sig + i];
    if (g == 0) sm[o_flag] = live ? 1.0 : 0.0;
    __syncthreads();
    for (int k = 0; k < n; k++) {
      if (g == k) {
        const double d = W(k, k);
        if (!(d > 0.0)) sm[o_flag] = 0.0;
        W(k, k) = sqrt(d > 0.0 ? d : 1.0);
      }
      __syncthreads();
      if (g > k && g < n) W(g, k) = W(g, k) / W(k, k);
      __syncthreads();
      if (g > k && g < n) {
        const double lg = W(g, k);
        for (int c = k + 1; c <= g; c++) W(g, c) -= lg * W(c, k);
      }
    }
    __syncthreads();
    return sm[o_flag] != 0.0;
  }

  // sigma point g of (mu, W): X0 = mu, X_{2j+1} = mu [+] L_j, X_{2j+2} = mu [+] -L_j
  UWVK_DEV void sigma_point(double x[S]) {
    double mu[S], col[n];
#pragma unroll
    for (int k = 0; k < S; k++) mu[k] = sm[o_mu + k];
    const int j = g >= 1 ? (g - 1) >> 1 : 0;
    const double sgn = (g & 1) ? 1.0 : -1.0;
#pragma unroll
    for (int r = 0; r < n; r++) col[r] = (g >= 1 && g < N && r >= j) ? W(r, j) : 0.0;
    M::boxplus(mu, col, sgn, x);
  }

  // Sigma = 1/2 sum_p D_p D_p^T (+ Qp(r, c)) from this lane's deviation d;
  // written only when `write` (same barrier sequence either way)
  template <class QF>
  UWVK_DEV void covariance(const double d[n], QF qf, bool write) {
    __syncthreads();  // W (aliased by D) no longer read
    if (g < N) {
#pragma unroll
      for (int r = 0; r < n; r++) D(g, r) = d[r];
    }
    __syncthreads();
    if (write && g < n) {
      for (int c = 0; c < n; c++) {
        double s = 0.0;
        for (int p = 0; p < N; p++) s += D(p, g) * D(p, c);
        sig(g, c) = 0.5 * s + qf(g, c);
      }
    }
    __syncthreads();
  }

  // manifold mean of the groups' points x (Gauss-Newton, |delta| <= 1e-6,
  // at most 1e4 iterations) into ref (registers, identical in every lane)
  UWVK_DEV void mean(const double x[S], double ref[S], bool active) {
    if (g == 0) {
#pragma unroll
      for (int k = 0; k < S; k++) sm[o_ref + k] = x[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < S; k++) ref[k] = sm[o_ref + k];
    bool done = !active;
    int it = 0;
    while (__syncthreads_or(!done)) {
      if (!done && g < N) {
        double d[n];
        M::boxminus(x, ref, d);
#pragma unroll
        for (int r = 0; r < n; r++) D(g, r) = d[r];
      }
      __syncthreads();
      if (!done && g < n) {
        double s = 0.0;
        for (int p = 0; p < N; p++) s += D(p, g);
        sm[o_vec + g] = s / (double)N;
      }
      __syncthreads();
      if (!done) {
        double dl[n], nrm = 0.0;
#pragma unroll
        for (int r = 0; r < n; r++) {
          dl[r] = sm[o_vec + r];
          nrm += dl[r] * dl[r];
        }
        M::boxplus(ref, dl, 1.0, ref);
        done = !(sqrt(nrm) > 1e-6 && ++it < 10000);
      }
      __syncthreads();
    }
  }

  // ukf::predict [EXT]: sigma spread, process g, manifold mean, covariance + Qp
  template <class PF, class QF>
  UWVK_DEV bool predict(PF pf, QF qf) {
    const bool ok = cholesky();
    double x[S];
    sigma_point(x);
    pf(x);
    double ref[S];
    mean(x, ref, ok);
    double d[n];
    M::boxminus(x, ref, d);
    covariance(d, qf, ok);
    if (ok && g == 0) {
#pragma unroll
      for (int k = 0; k < S; k++) sm[o_mu + k] = ref[k];
    }
    __syncthreads();
    return ok;
  }

  // ukf::update [EXT] with measurement functor h (zmode ZK, dimension MZ),
  // accept_any_mahalanobis_distance, then the literal apply_delta.
  template <int ZK, int MZ, class H>
  UWVK_DEV bool update(const double z[3], const double* Rm, H h) {
    constexpr int ZS = ZK == Z_S2 ? 3 : MZ;
    bool ok = cholesky();
    double x[S];
    sigma_point(x);
    double zp[3] = {0.0, 0.0, 0.0};
    h(x, zp);
    if (g < N) {
#pragma unroll
      for (int a = 0; a < 3; a++) sm[o_z + g * 3 + a] = zp[a];
    }
    __syncthreads();
    // mean of Z, redundantly in every lane (m <= 2)
    double zm[3] = {0.0, 0.0, 0.0};
    if (ZK == Z_VEC) {
      for (int p = 0; p < N; p++)
#pragma unroll
        for (int a = 0; a < MZ; a++) zm[a] += sm[o_z + p * 3 + a];
#pragma unroll
      for (int a = 0; a < MZ; a++) zm[a] = zm[a] / (double)N;
    } else {
#pragma unroll
      for (int a = 0; a < ZS; a++) zm[a] = sm[o_z + a];
      int it = 0;
      double nrm;
      do {
        double d[2] = {0.0, 0.0}, dd[2];
        for (int p = 0; p < N; p++) {
          zminus<ZK, MZ>(&sm[o_z + p * 3], zm, dd);
#pragma unroll
          for (int a = 0; a < MZ; a++) d[a] += dd[a];
        }
        nrm = 0.0;
#pragma unroll
        for (int a = 0; a < MZ; a++) {
          d[a] /= (double)N;
          nrm += d[a] * d[a];
        }
        if constexpr (ZK == Z_S2) {
          s2_boxplus(zm, d, 1.0, zm);
        } else {
#pragma unroll
          for (int a = 0; a < MZ; a++) zm[a] = zm[a] + d[a];
        }
        nrm = sqrt(nrm);
      } while (nrm > 1e-6 && ++it < 10000);
    }
    // deviations
    double mu[S], dx[n];
#pragma unroll
    for (int k = 0; k < S; k++) mu[k] = sm[o_mu + k];
    M::boxminus(x, mu, dx);
    double dz[2] = {0.0, 0.0};
    zminus<ZK, MZ>(zp, zm, dz);
    __syncthreads();  // W (aliased by D) no longer read
    if (g < N) {
#pragma unroll
      for (int r = 0; r < n; r++) D(g, r) = dx[r];
#pragma unroll
      for (int a = 0; a < MZ; a++) sm[o_dz + g * 2 + a] = dz[a];
    }
    __syncthreads();
    // S = 1/2 sum dz dz^T + R (every lane), S^-1 (oracle's closed forms)
    double Sm[4] = {0, 0, 0, 0}, Si[4];
    for (int p = 0; p < N; p++)
#pragma unroll
      for (int a = 0; a < MZ; a++)
#pragma unroll
        for (int b = 0; b < MZ; b++) Sm[a * MZ + b] += sm[o_dz + p * 2 + a] * sm[o_dz + p * 2 + b];
#pragma unroll
    for (int i = 0; i < MZ * MZ; i++) Sm[i] = 0.5 * Sm[i] + Rm[i];
    if constexpr (MZ == 1) {
      Si[0] = 1.0 / Sm[0];
    } else {
      const double id = 1.0 / (Sm[0] * Sm[3] - Sm[1] * Sm[2]);
      Si[0] = Sm[3] * id; Si[1] = -Sm[1] * id; Si[2] = -Sm[2] * id; Si[3] = Sm[0] * id;
    }
    double nu[2] = {0.0, 0.0};
    zminus<ZK, MZ>(z, zm, nu);  // innovation z [-] meanZ
    // lane r: C_r = 1/2 sum_p D(p, r) dz_p ; K_r = C_r S^-1 ; delta_r = K_r nu
    double Cr[2] = {0.0, 0.0}, Kr[2] = {0.0, 0.0};
    if (g < n) {
      for (int p = 0; p < N; p++)
#pragma unroll
        for (int a = 0; a < MZ; a++) Cr[a] += D(p, g) * sm[o_dz + p * 2 + a];
#pragma unroll
      for (int a = 0; a < MZ; a++) Cr[a] = 0.5 * Cr[a];
#pragma unroll
      for (int a = 0; a < MZ; a++) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < MZ; b++) s += Cr[b] * Si[b * MZ + a];
        Kr[a] = s;
      }
      double dl = 0.0;
#pragma unroll
      for (int a = 0; a < MZ; a++) {
        sm[o_k + g * 2 + a] = Kr[a];
        dl += Kr[a] * nu[a];
      }
      sm[o_vec + g] = dl;
    }
    __syncthreads();
    // Sigma -= C K^T (row g), only where the spread succeeded
    if (ok && g < n) {
      for (int c = 0; c < n; c++) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < MZ; a++) s += Cr[a] * sm[o_k + c * 2 + a];
        sig(g, c) -= s;
      }
    }
    __syncthreads();
    // apply_delta (literal re-spread about mu [+] delta)
    double delta[n];
#pragma unroll
    for (int r = 0; r < n; r++) delta[r] = sm[o_vec + r];
    const bool ok2 = cholesky() && ok;
    double y[S];
    sigma_point(y);
    M::boxplus(y, delta, 1.0, y);
    double mu2[S];
    M::boxplus(mu, delta, 1.0, mu2);
    double d2[n];
    M::boxminus(y, mu2, d2);
    covariance(d2, [](int, int) { return 0.0; }, ok2);
    if (ok2 && g == 0) {
#pragma unroll
      for (int k = 0; k < S; k++) sm[o_mu + k] = mu2[k];
    }
    __syncthreads();
    return ok2;
  }

  template <int ZK, int MZ>
  UWVK_DEV static void zminus(const double* a, const double* b, double* o) {
    if constexpr (ZK == Z_S2) {
      s2_boxminus(a, b, o);
    } else {
#pragma unroll
      for (int k = 0; k < MZ; k++) o[k] = a[k] - b[k];
    }
  }
};

// ---------------------------------------------------------------------------
// visual-landmark update shared by PoseUKF (PoseUKF.cpp:613-654) and
// IndirectPoseUKF (IndirectPoseUKF.cpp:94-135)
// ---------------------------------------------------------------------------
struct VisArgs {             // device pointers
  int nf;                    // features per instance (the same for the batch)
  const double* features;    // [batch][nf][2] undistorted image coordinates
  const double* fcov;        // [batch][nf][4] or shared [nf][4]
  int64_t fcov_stride;       // doubles per instance (0 = shared)
  const double* fpos;        // [nf][3] feature positions in the marker frame
  const double* marker;      // [batch][7] or shared [7]: marker pose in nav, t(3) q(4)
  int64_t marker_stride;     // 7 or 0
  const double* ref;         // IndirectPoseUKF: [batch][7] pose_ref (body in nav); PoseUKF: unused
  const uint8_t* mask;       // nullable
  double cov_marker[36];
  double cam[4];             // fx, fy, cx, cy (CameraConfiguration, PoseUKFConfig.hpp:125-131)
  double cam_in[7];          // camera in body / IMU, t(3) q(4)
};

// measurementVisualLandmark: ((body_in_nav [* pose_error]) * cam_in_body)^-1 *
// (q_m f + t_m) as S2 (IndirectPoseUKF.cpp:38-50, PoseUKF.cpp:231-244).
// SM: storage offset of marker_position; INDIRECT: state is the pose error.
template <int SM, bool INDIRECT>
struct VisualH {
  double f[3], cam[7], ref[7];
  UWVK_DEV void operator()(const double* x, double* z) const {
    double fn[3], t[3], u[3], w[3], fc[3];
    qrot(x + SM + 3, f, fn);
#pragma unroll
    for (int k = 0; k < 3; k++) fn[k] += x[SM + k];
    if constexpr (INDIRECT) {
#pragma unroll
      for (int k = 0; k < 3; k++) t[k] = fn[k] - ref[k];
      qrot_inv(ref + 3, t, u);
#pragma unroll
      for (int k = 0; k < 3; k++) u[k] -= x[k];
      qrot_inv(x + 3, u, w);
    } else {
#pragma unroll
      for (int k = 0; k < 3; k++) t[k] = fn[k] - x[k];
      qrot_inv(x + 3, t, w);
    }
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] -= cam[k];
    qrot_inv(cam + 3, w, fc);
    s2_from(fc, z);
  }
};

// The feature loop on an augmented state already in LDS (mu, Sigma loaded):
// one ukf::update per feature, S2-valued, accept_any_mahalanobis_distance.
template <class E, int SM, bool INDIRECT>
UWVK_DEV bool visual_loop(E& e, const VisArgs& va, int64_t inst) {
  VisualH<SM, INDIRECT> h;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    h.cam[k] = va.cam_in[k];
    h.ref[k] = (INDIRECT && e.live) ? va.ref[inst * 7 + k] : 0.0;
  }
  const double fx2 = va.cam[0] * va.cam[0], fy2 = va.cam[1] * va.cam[1], fxy = va.cam[0] * va.cam[1];
  bool ok = true;
  for (int i = 0; i < va.nf; i++) {
    double z[3] = {0.0, 0.0, 1.0}, R[4] = {1.0, 0.0, 0.0, 1.0};
    if (e.live) {
      const double* mu = va.features + (inst * va.nf + i) * 2;
      const double* cv = va.fcov + inst * va.fcov_stride + i * 4;
      const double pv[3] = {(mu[0] - va.cam[2]) / va.cam[0], (mu[1] - va.cam[3]) / va.cam[1], 1.0};
      s2_from(pv, z);
      R[0] = cv[0] / fx2; R[1] = cv[1] / fxy; R[2] = cv[2] / fxy; R[3] = cv[3] / fy2;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) h.f[k] = va.fpos[i * 3 + k];
    ok = e.template update<Z_S2, 2>(z, R, h) && ok;
  }
  return ok;
}

// Per-handle device staging buffer for the visual inputs: grown on demand,
// reused across calls, freed with the handle (no per-call allocation).
struct VisStage {
  double* d = nullptr;
  size_t cap = 0;  // doubles
  bool reserve(size_t words, hipStream_t st) {
    if (words <= cap) return true;
    if (d) {
      if (hipStreamSynchronize(st) != hipSuccess) return false;
      (void)hipFree(d);
      d = nullptr;
      cap = 0;
    }
    if (hipMalloc((void**)&d, words * 8) != hipSuccess) {
      d = nullptr;
      return false;
    }
    cap = words;
    return true;
  }
  void release() {
    if (d) (void)hipFree(d);
    d = nullptr;
    cap = 0;
  }
};

// host: validate (checkMeasurment on every feature) and stage one visual
// update's inputs on the device.  Returns 0 ok, 1 EINVAL, 2 ENAN, 5 EDEVICE.
// nf == 0 returns 0 with va->nf == 0 (nothing to launch).
inline int stage_visual(hipStream_t st, int64_t B, int32_t nf_, const double* features, const double* feature_cov,
                        int fcov_pi, const double* fpos, const double* marker, int marker_pi,
                        const double* cov_marker, const double* cam, const double* cam_in, const uint8_t* mask,
                        VisArgs* va, VisStage* stage) {
  if (nf_ < 0 || (nf_ > 0 && (!features || !feature_cov || !fpos)) || !marker || !cov_marker || !cam || !cam_in)
    return 1;
  const size_t nf = (size_t)nf_;
  auto fin = [](const double* a, size_t n) {
    for (size_t k = 0; k < n; k++)
      if (!(a[k] - a[k] == 0.0)) return false;  // NaN / Inf
    return true;
  };
  for (int64_t i = 0; i < B; i++) {
    if (mask && !mask[i]) continue;
    if (!fin(features + i * nf * 2, nf * 2)) return 2;
    if (fcov_pi && !fin(feature_cov + i * nf * 4, nf * 4)) return 2;
  }
  if (!fcov_pi && nf && !fin(feature_cov, nf * 4)) return 2;
  if (!fin(cov_marker, 36) || !fin(cam, 4) || !fin(cam_in, 7) || !fin(marker, marker_pi ? (size_t)B * 7 : 7)) return 2;
  if (nf == 0) return 0;
  const size_t wf = (size_t)B * nf * 2, wc = fcov_pi ? (size_t)B * nf * 4 : nf * 4, wp = nf * 3,
               wm = marker_pi ? (size_t)B * 7 : 7, wk = mask ? ((size_t)B + 7) / 8 : 0;
  if (!stage->reserve(wf + wc + wp + wm + wk, st)) return 5;
  double* d = stage->d;
  va->nf = nf_;
  va->features = d;
  va->fcov = d + wf;
  va->fcov_stride = fcov_pi ? (int64_t)nf * 4 : 0;
  va->fpos = d + wf + wc;
  va->marker = d + wf + wc + wp;
  va->marker_stride = marker_pi ? 7 : 0;
  va->mask = mask ? (const uint8_t*)(d + wf + wc + wp + wm) : nullptr;
  for (int k = 0; k < 36; k++) va->cov_marker[k] = cov_marker[k];
  for (int k = 0; k < 4; k++) va->cam[k] = cam[k];
  for (int k = 0; k < 7; k++) va->cam_in[k] = cam_in[k];
  hipError_t e = hipMemcpyAsync(d, features, wf * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + wf, feature_cov, wc * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + wf + wc, fpos, wp * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = hipMemcpyAsync(d + wf + wc + wp, marker, wm * 8, hipMemcpyHostToDevice, st);
  if (e == hipSuccess && mask) e = hipMemcpyAsync((void*)va->mask, mask, (size_t)B, hipMemcpyHostToDevice, st);
  return e == hipSuccess ? 0 : 5;
}

}  // namespace aug
}  // namespace uwvk
