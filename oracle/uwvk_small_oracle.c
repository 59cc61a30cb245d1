/*
 * uwvk_small_oracle.c — CPU fp64 restatement of BottomUKF, IndirectPoseUKF and
 * the marker-augmented visual-landmark updates (PoseUKF and IndirectPoseUKF).
 *
 * TEST INFRASTRUCTURE ONLY (see uwvk_oracle.h): only tests/ and smoke() load it.
 * PARITY STATUS: UNPINNED (the reference cannot be built and ships no tests,
 * SURVEY.md §8c).  Follows the reference files line by line:
 *   BottomUKF.cpp:1-71, BottomUKF.hpp:15-53
 *   IndirectPoseUKF.cpp:1-147, IndirectPoseUKF.hpp:16-86
 *   PoseUKF.cpp:221-244 (PoseStateWithMarker, measurementVisualLandmark),
 *   PoseUKF.cpp:613-654 (integrateMeasurement(vector<VisualFeatureMeasurement>))
 * plus the frozen [EXT] spec of DESIGN.md §3, extended by item 11 (S2):
 *   x [+] d = R_x exp(d), y [-] x = log(R_x^T y), with R_x the minimal
 *   rotation taking e3 to x, exp(d) = (sinc|d| d1, sinc|d| d2, cos|d|) and
 *   log(w) = atan2(|w12|, w3) w12 / |w12|.
 */
#include <math.h>
#include <string.h>

#include "uwvk_oracle.h"

#define SM_MAXN 59
#define SM_MAXS 61
#define SM_NPTS (2 * SM_MAXN + 1)
#define SM_MAXSEG 8

/* SEG_SO3R: an SO3 segment with the body-frame (right) [+]/[-], q exp(d) and
 * log(b^-1 a): the PoseUKF visual update's segments under or_set_so3_right(1) */
enum { SEG_V = 0, SEG_SO3 = 1, SEG_S2 = 2, SEG_SO3R = 3 };

typedef struct sm_manifold {
  int nseg, dof, store;
  int kind[SM_MAXSEG], dim[SM_MAXSEG]; /* dim: DOF of the segment (vect only) */
} sm_manifold;

static void sm_add(sm_manifold* M, int kind, int dim) {
  M->kind[M->nseg] = kind;
  M->dim[M->nseg] = kind == SEG_V ? dim : (kind == SEG_S2 ? 2 : 3);
  M->dof += M->dim[M->nseg];
  M->store += kind == SEG_V ? dim : (kind == SEG_S2 ? 3 : 4);
  M->nseg++;
}

/* ---- S2 [EXT MTK S2], frozen spec item 11 ------------------------------ */
/* columns of R_x (minimal rotation e3 -> x): b1, b2, x */
static void s2_basis(const double x[3], double b1[3], double b2[3]) {
  double k = 1.0 / (1.0 + x[2]);
  b1[0] = 1.0 - x[0] * x[0] * k; b1[1] = -x[0] * x[1] * k; b1[2] = -x[0];
  b2[0] = -x[0] * x[1] * k; b2[1] = 1.0 - x[1] * x[1] * k; b2[2] = -x[1];
}

void or_s2_boxplus(const double x[3], const double d[2], double s, double o[3]) {
  double a = s * d[0], b = s * d[1];
  double t = sqrt(a * a + b * b);
  double sc = t == 0.0 ? 1.0 : sin(t) / t;
  double c = cos(t), b1[3], b2[3], r[3];
  s2_basis(x, b1, b2);
  for (int i = 0; i < 3; i++) r[i] = b1[i] * (sc * a) + b2[i] * (sc * b) + x[i] * c;
  o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
}

void or_s2_boxminus(const double y[3], const double x[3], double o[2]) {
  double b1[3], b2[3];
  s2_basis(x, b1, b2);
  double w1 = b1[0] * y[0] + b1[1] * y[1] + b1[2] * y[2];
  double w2 = b2[0] * y[0] + b2[1] * y[1] + b2[2] * y[2];
  double w3 = x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
  double n = sqrt(w1 * w1 + w2 * w2);
  if (n == 0.0) { o[0] = 0.0; o[1] = 0.0; return; }
  double k = atan2(n, w3) / n;
  o[0] = k * w1; o[1] = k * w2;
}

/* MTK::S2 constructor from a vector: normalised */
void or_s2_from_vector(const double v[3], double o[3]) {
  double n = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  o[0] = v[0] / n; o[1] = v[1] / n; o[2] = v[2] / n;
}

/* ---- compound manifold ---------------------------------------------------- */
static void sm_boxplus(const sm_manifold* M, const double* x, const double* d, double s, double* o) {
  int di = 0, si = 0;
  double tmp[SM_MAXS];
  for (int g = 0; g < M->nseg; g++) {
    if (M->kind[g] == SEG_V) {
      for (int k = 0; k < M->dim[g]; k++) tmp[si + k] = x[si + k] + s * d[di + k];
      si += M->dim[g];
    } else if (M->kind[g] == SEG_SO3 || M->kind[g] == SEG_SO3R) {
      double v[3] = {s * d[di], s * d[di + 1], s * d[di + 2]}, e[4];
      or_so3_exp(v, e);
      if (M->kind[g] == SEG_SO3R) or_quat_mul(x + si, e, tmp + si);
      else or_quat_mul(e, x + si, tmp + si);
      si += 4;
    } else {
      or_s2_boxplus(x + si, d + di, s, tmp + si);
      si += 3;
    }
    di += M->dim[g];
  }
  memcpy(o, tmp, sizeof(double) * M->store);
}

static void sm_boxminus(const sm_manifold* M, const double* a, const double* b, double* o) {
  int di = 0, si = 0;
  for (int g = 0; g < M->nseg; g++) {
    if (M->kind[g] == SEG_V) {
      for (int k = 0; k < M->dim[g]; k++) o[di + k] = a[si + k] - b[si + k];
      si += M->dim[g];
    } else if (M->kind[g] == SEG_SO3 || M->kind[g] == SEG_SO3R) {
      double bc[4] = {b[si], -b[si + 1], -b[si + 2], -b[si + 3]}, r[4];
      if (M->kind[g] == SEG_SO3R) or_quat_mul(bc, a + si, r);
      else or_quat_mul(a + si, bc, r);
      or_so3_log(r, o + di);
      si += 4;
    } else {
      or_s2_boxminus(a + si, b + si, o + di);
      si += 3;
    }
    di += M->dim[g];
  }
}

/* ---- ukfom::ukf [EXT] on a compound manifold ----- */
static int sm_sigma_points(const sm_manifold* M, const double* mu, const double* sigma, double* X) {
  int n = M->dof;
  double L[SM_MAXN * SM_MAXN], col[SM_MAXN];
  if (or_cholesky(n, sigma, L) != 0) return -1;
  memcpy(X, mu, sizeof(double) * M->store);
  for (int j = 0; j < n; j++) {
    for (int r = 0; r < n; r++) col[r] = L[r * n + j];
    sm_boxplus(M, mu, col, 1.0, X + (2 * j + 1) * SM_MAXS);
    sm_boxplus(M, mu, col, -1.0, X + (2 * j + 2) * SM_MAXS);
  }
  return 0;
}

static void sm_mean(const sm_manifold* M, const double* X, int N, int stride, double* ref) {
  int n = M->dof, it = 0;
  double d[SM_MAXN], dd[SM_MAXN], nrm;
  memcpy(ref, X, sizeof(double) * M->store);
  do {
    for (int k = 0; k < n; k++) d[k] = 0.0;
    for (int p = 0; p < N; p++) {
      sm_boxminus(M, X + p * stride, ref, dd);
      for (int k = 0; k < n; k++) d[k] += dd[k];
    }
    nrm = 0.0;
    for (int k = 0; k < n; k++) { d[k] /= (double)N; nrm += d[k] * d[k]; }
    sm_boxplus(M, ref, d, 1.0, ref);
    nrm = sqrt(nrm);
  } while (nrm > 1e-6 && ++it < 10000);
}

static void sm_cov(const sm_manifold* M, const double* mean, const double* X, int N, double* S) {
  int n = M->dof;
  double d[SM_MAXN];
  for (int i = 0; i < n * n; i++) S[i] = 0.0;
  for (int p = 0; p < N; p++) {
    sm_boxminus(M, X + p * SM_MAXS, mean, d);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) S[i * n + j] += d[i] * d[j];
  }
  for (int i = 0; i < n * n; i++) S[i] = 0.5 * S[i];
}

typedef void (*sm_fn)(void* ctx, const double* x, double* out);

static int sm_predict(const sm_manifold* M, double* mu, double* sigma, sm_fn g, void* ctx, const double* Qp) {
  static __thread double X[SM_NPTS * SM_MAXS];
  int n = M->dof, N = 2 * n + 1;
  if (sm_sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  for (int p = 0; p < N; p++) g(ctx, X + p * SM_MAXS, X + p * SM_MAXS);
  sm_mean(M, X, N, SM_MAXS, mu);
  sm_cov(M, mu, X, N, sigma);
  for (int i = 0; i < n * n; i++) sigma[i] += Qp[i];
  return UWVK_OK;
}

static int sm_apply_delta(const sm_manifold* M, double* mu, double* sigma, const double* delta) {
  static __thread double X[SM_NPTS * SM_MAXS];
  int n = M->dof, N = 2 * n + 1;
  if (sm_sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  sm_boxplus(M, mu, delta, 1.0, mu);
  for (int p = 0; p < N; p++) sm_boxplus(M, X + p * SM_MAXS, delta, 1.0, X + p * SM_MAXS);
  sm_cov(M, mu, X, N, sigma);
  return UWVK_OK;
}

/* measurement manifolds: 0 Eigen vector (plain average), 1 vect manifold
 * (iterative mean), 2 S2 (iterative mean; z and Z stored as unit 3-vectors) */
enum { Z_VEC = 0, Z_VECT_MANIFOLD = 1, Z_S2 = 2 };

static void z_boxminus(int zk, int m, const double* a, const double* b, double* o) {
  if (zk == Z_S2) { or_s2_boxminus(a, b, o); return; }
  for (int k = 0; k < m; k++) o[k] = a[k] - b[k];
}

static int sm_update(const sm_manifold* M, double* mu, double* sigma, int zk, int m, const double* z, sm_fn h,
                     void* ctx, const double* R, int* accepted) {
  static __thread double X[SM_NPTS * SM_MAXS];
  static __thread double Z[SM_NPTS * 3];
  int n = M->dof, N = 2 * n + 1, zs = zk == Z_S2 ? 3 : m;
  double zm[3], S[4], Si[4], C[SM_MAXN * 2], K[SM_MAXN * 2], nu[2], dx[SM_MAXN], dz[2];
  *accepted = 0;
  if (sm_sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  for (int p = 0; p < N; p++) h(ctx, X + p * SM_MAXS, Z + p * 3);
  if (zk == Z_VEC) {
    for (int a = 0; a < m; a++) zm[a] = 0.0;
    for (int p = 0; p < N; p++)
      for (int a = 0; a < m; a++) zm[a] += Z[p * 3 + a];
    for (int a = 0; a < m; a++) zm[a] = zm[a] / (double)N;
  } else {
    int it = 0;
    double d[2], dd[2], nrm;
    for (int a = 0; a < zs; a++) zm[a] = Z[a];
    do {
      d[0] = d[1] = 0.0;
      for (int p = 0; p < N; p++) {
        z_boxminus(zk, m, Z + p * 3, zm, dd);
        for (int a = 0; a < m; a++) d[a] += dd[a];
      }
      nrm = 0.0;
      for (int a = 0; a < m; a++) { d[a] /= (double)N; nrm += d[a] * d[a]; }
      if (zk == Z_S2) or_s2_boxplus(zm, d, 1.0, zm);
      else for (int a = 0; a < m; a++) zm[a] = zm[a] + d[a];
      nrm = sqrt(nrm);
    } while (nrm > 1e-6 && ++it < 10000);
  }
  for (int i = 0; i < m * m; i++) S[i] = 0.0;
  for (int i = 0; i < n * m; i++) C[i] = 0.0;
  for (int p = 0; p < N; p++) {
    z_boxminus(zk, m, Z + p * 3, zm, dz);
    sm_boxminus(M, X + p * SM_MAXS, mu, dx);
    for (int a = 0; a < m; a++)
      for (int b = 0; b < m; b++) S[a * m + b] += dz[a] * dz[b];
    for (int i = 0; i < n; i++)
      for (int a = 0; a < m; a++) C[i * m + a] += dx[i] * dz[a];
  }
  for (int i = 0; i < m * m; i++) S[i] = 0.5 * S[i] + R[i];
  for (int i = 0; i < n * m; i++) C[i] = 0.5 * C[i];
  if (or_invert(m, S, Si) != 0) return UWVK_ENOTPD;
  for (int i = 0; i < n; i++)
    for (int a = 0; a < m; a++) {
      double s = 0.0;
      for (int b = 0; b < m; b++) s += C[i * m + b] * Si[b * m + a];
      K[i * m + a] = s;
    }
  z_boxminus(zk, m, z, zm, nu); /* innovation z [-] meanZ */
  /* every update of these filters uses accept_any_mahalanobis_distance */
  *accepted = 1;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0.0;
      for (int a = 0; a < m; a++) s += C[i * m + a] * K[j * m + a];
      sigma[i * n + j] -= s;
    }
  double delta[SM_MAXN];
  for (int i = 0; i < n; i++) {
    double s = 0.0;
    for (int a = 0; a < m; a++) s += K[i * m + a] * nu[a];
    delta[i] = s;
  }
  return sm_apply_delta(M, mu, sigma, delta);
}

static int finite_n(const double* a, int n) {
  for (int i = 0; i < n; i++)
    if (!isfinite(a[i])) return 0;
  return 1;
}

/* ======================================================================== */
/* BottomUKF (BottomUKF.cpp / .hpp)                                          */
/* ======================================================================== */
static sm_manifold bottom_manifold(void) {
  sm_manifold M = {0};
  sm_add(&M, SEG_V, 1);  /* distance: mtkwrap<Scalar>, BottomUKF.hpp:19 */
  sm_add(&M, SEG_S2, 2); /* normal: mtkwrap<S2>, BottomUKF.hpp:20 */
  return M;
}

/* BottomUKF(initial_state, state_cov), BottomUKF.cpp:40-46: x = {d, n(3)} */
void or_bottom_init(or_bottom* f, const double x[4], const double P[9]) {
  f->mu[0] = x[0];
  or_s2_from_vector(x + 1, f->mu + 1);
  memcpy(f->sigma, P, sizeof(double) * 9);
  for (int i = 0; i < 9; i++) f->Q[i] = (i % 4 == 0) ? 1.0 : 0.0; /* Covariance::Identity(), :48 */
  f->velocity[0] = f->velocity[1] = f->velocity[2] = 0.0;
}

void or_bottom_set_process_noise(or_bottom* f, const double Q[9]) { memcpy(f->Q, Q, sizeof(double) * 9); }

/* setProcessNoiseCovariance [EXT pose_estimation base] */
void or_ipose_set_process_noise(or_ipose* f, const double Q[36]) { memcpy(f->Q, Q, sizeof(double) * 36); }

void or_bottom_set_velocity(or_bottom* f, const double v[3]) { memcpy(f->velocity, v, sizeof(double) * 3); }

/* processModel, BottomUKF.cpp:5-16 */
static void bottom_process(void* ctx, const double* x, double* o) {
  const double* vz = (const double*)ctx;
  double tmp[4];
  memcpy(tmp, x, sizeof(tmp));
  tmp[0] = x[0] + (-1.0 * vz[0]) * vz[1];
  memcpy(o, tmp, sizeof(tmp));
}

/* predictionStepImpl, BottomUKF.cpp:48-54 */
int or_bottom_predict(or_bottom* f, double dt) {
  sm_manifold M = bottom_manifold();
  double vxy2 = f->velocity[0] * f->velocity[0] + f->velocity[1] * f->velocity[1];
  double nrm = sqrt(vxy2);
  double s = pow(nrm, 2.0) * pow(dt, 2.0), Qp[9], ctx[2] = {f->velocity[2], dt};
  for (int i = 0; i < 9; i++) Qp[i] = s * f->Q[i];
  return sm_predict(&M, f->mu, f->sigma, bottom_process, ctx, Qp);
}

typedef struct range_ctx {
  double dir[3], origin[3];
} range_ctx;

/* measurementDistance, BottomUKF.cpp:18-30 */
static void h_range(void* c, const double* x, double* z) {
  const range_ctx* r = (const range_ctx*)c;
  double bottom[3] = {0.0, 0.0, -x[0]};
  const double* n = x + 1;
  double v = r->dir[0] * n[0] + r->dir[1] * n[1] + r->dir[2] * n[2];
  if (v != 0.0) {
    double w = (bottom[0] - r->origin[0]) * n[0] + (bottom[1] - r->origin[1]) * n[1] +
               (bottom[2] - r->origin[2]) * n[2];
    z[0] = w / v;
  } else {
    z[0] = 0.0;
  }
}

/* integrateMeasurement(RangeMeasurement, unit_direction, origin), BottomUKF.cpp:56-61 */
int or_bottom_update_range(or_bottom* f, double mu, double cov, const double dir[3], const double origin[3]) {
  if (!isfinite(mu) || !isfinite(cov)) return UWVK_ENAN;
  sm_manifold M = bottom_manifold();
  range_ctx c;
  memcpy(c.dir, dir, sizeof(c.dir));
  memcpy(c.origin, origin, sizeof(c.origin));
  int acc;
  return sm_update(&M, f->mu, f->sigma, Z_VECT_MANIFOLD, 1, &mu, h_range, &c, &cov, &acc);
}

/* measurementNormal, BottomUKF.cpp:32-37 */
static void h_normal(void* c, const double* x, double* z) { z[0] = x[1]; z[1] = x[2]; z[2] = x[3]; }

/* integrateMeasurement(NormalType, cov), BottomUKF.cpp:63-67 (no NaN check there) */
int or_bottom_update_normal(or_bottom* f, const double mu[3], const double cov[4]) {
  sm_manifold M = bottom_manifold();
  double z[3];
  or_s2_from_vector(mu, z);
  int acc;
  return sm_update(&M, f->mu, f->sigma, Z_S2, 2, z, h_normal, NULL, cov, &acc);
}

/* ======================================================================== */
/* IndirectPoseUKF (IndirectPoseUKF.cpp / .hpp)                              */
/* ======================================================================== */
static sm_manifold ipose_manifold(int with_marker) {
  sm_manifold M = {0};
  /* orientation_error is an MTK::SO3 like PoseUKF's orientation: the same side
   * switch (or_set_so3_right; the default right, q exp(d)) */
  const int so3 = or_get_so3_right() ? SEG_SO3R : SEG_SO3;
  sm_add(&M, SEG_V, 3);  /* position_error, IndirectPoseUKF.hpp:20 */
  sm_add(&M, so3, 3);    /* orientation_error, :21 */
  if (with_marker) {      /* FilterStateWithMarker, IndirectPoseUKF.cpp:25-29 */
    sm_add(&M, SEG_V, 3);
    sm_add(&M, so3, 3);
  }
  return M;
}

/* IndirectPoseUKF(...), IndirectPoseUKF.cpp:53-78 */
void or_ipose_init(or_ipose* f, const double pos_std[3], const double ori_std[3], double tau,
                   const double init_pos_err[3], const double init_pos_std[3]) {
  memset(f, 0, sizeof(*f));
  for (int k = 0; k < 3; k++) f->mu[k] = init_pos_err ? init_pos_err[k] : 0.0;
  f->mu[3] = 1.0;
  for (int k = 0; k < 3; k++) {
    double s0 = init_pos_std ? init_pos_std[k] : 1.0;
    f->sigma[k * 6 + k] = fabs(s0) * fabs(s0);
    f->sigma[(k + 3) * 6 + k + 3] = fabs(ori_std[k]) * fabs(ori_std[k]);
    f->Q[k * 6 + k] = fabs(pos_std[k]) * fabs(pos_std[k]);
    f->Q[(k + 3) * 6 + k + 3] = fabs(ori_std[k]) * fabs(ori_std[k]);
  }
  f->tau = tau;
  f->pose_ref[3] = 1.0; /* Affine3d::Identity() */
}

void or_ipose_set_pose_reference(or_ipose* f, const double pose[7]) { memcpy(f->pose_ref, pose, sizeof(f->pose_ref)); }

/* processModel, IndirectPoseUKF.cpp:7-20 */
static void ipose_process(void* ctx, const double* x, double* o) {
  const double* c = (const double*)ctx; /* {tau, dt} */
  double l[3], d[3], e[4], tmp[7];
  or_so3_log(x + 3, l);
  for (int k = 0; k < 3; k++) d[k] = (-1.0 / c[0]) * l[k] * c[1];
  or_so3_exp(d, e);
  memcpy(tmp, x, sizeof(tmp));
  /* orientation_error.boxplus(d, dt), :17, on the side of the switch (e is a
   * power of x's own rotation, so the two products agree) */
  if (or_get_so3_right()) or_quat_mul(x + 3, e, tmp + 3);
  else or_quat_mul(e, x + 3, tmp + 3);
  memcpy(o, tmp, sizeof(tmp));
}

/* predictionStepImpl, IndirectPoseUKF.cpp:80-92 */
int or_ipose_predict(or_ipose* f, double dt) {
  sm_manifold M = ipose_manifold(0);
  double R[9], Qp[36], A[9], B[9];
  or_quat_to_matrix(f->mu + 3, R);
  memcpy(Qp, f->Q, sizeof(Qp));
  double s = 2.0 / (f->tau * dt);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double t = 0.0;
      for (int k = 0; k < 3; k++) t += R[i * 3 + k] * (s * f->Q[(k + 3) * 6 + j + 3]);
      A[i * 3 + j] = t;
    }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double t = 0.0;
      for (int k = 0; k < 3; k++) t += A[i * 3 + k] * R[j * 3 + k];
      B[i * 3 + j] = t;
    }
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) Qp[(i + 3) * 6 + j + 3] = B[i * 3 + j];
  double dt2 = pow(dt, 2.0);
  for (int i = 0; i < 36; i++) Qp[i] = dt2 * Qp[i];
  double ctx[2] = {f->tau, dt};
  return sm_predict(&M, f->mu, f->sigma, ipose_process, ctx, Qp);
}

/* ---- visual landmark measurement (shared by both filters) --------------- */
typedef struct vis_ctx {
  int indirect;          /* 1: IndirectPoseUKF (pose_ref * pose_error), 0: PoseUKF */
  int s_marker;          /* storage offset of marker_position (quaternion follows) */
  double feature[3];     /* feature position in the marker frame */
  double cam[7];         /* camera in body / IMU: t(3), q(4) */
  double ref[7];         /* IndirectPoseUKF pose_ref (body in nav) */
} vis_ctx;

static void qinv_rotate(const double q[4], const double v[3], double o[3]) { or_quat_rotate_inv(q, v, o); }

/* measurementVisualLandmark, IndirectPoseUKF.cpp:38-50 / PoseUKF.cpp:231-244:
 * feature_in_cam = ((body_in_nav [* pose_error]) * cam_in_body)^-1 * (q_m f + t_m), as S2 */
static void h_visual(void* c, const double* x, double* z) {
  const vis_ctx* v = (const vis_ctx*)c;
  double fn[3], t[3], u[3], w[3], fc[3];
  or_quat_rotate(x + v->s_marker + 3, v->feature, fn);
  for (int k = 0; k < 3; k++) fn[k] += x[v->s_marker + k];
  if (v->indirect) { /* T_ref * T_err: x -> R_ref (R_err x + p_err) + t_ref */
    for (int k = 0; k < 3; k++) t[k] = fn[k] - v->ref[k];
    qinv_rotate(v->ref + 3, t, u);
    for (int k = 0; k < 3; k++) u[k] -= x[k];
    qinv_rotate(x + 3, u, w);
  } else { /* imu_in_nav = (q, p) */
    for (int k = 0; k < 3; k++) t[k] = fn[k] - x[k];
    qinv_rotate(x + 3, t, w);
  }
  for (int k = 0; k < 3; k++) w[k] -= v->cam[k];
  qinv_rotate(v->cam + 3, w, fc);
  or_s2_from_vector(fc, z);
}

/* the augmented update loop shared by IndirectPoseUKF.cpp:94-135 and PoseUKF.cpp:613-654 */
static int visual_loop(const sm_manifold* A, double* amu, double* asig, vis_ctx* c, int nf, const double* features,
                       const double* feature_cov, const double* feature_pos, const double cam_cfg[4]) {
  double fx2 = pow(cam_cfg[0], 2.0), fy2 = pow(cam_cfg[1], 2.0), fxy = cam_cfg[0] * cam_cfg[1];
  for (int i = 0; i < nf; i++) {
    const double* mu = features + 2 * i;
    const double* cv = feature_cov + 4 * i;
    double pv[3] = {(mu[0] - cam_cfg[2]) / cam_cfg[0], (mu[1] - cam_cfg[3]) / cam_cfg[1], 1.0}, z[3];
    or_s2_from_vector(pv, z);
    double R[4] = {cv[0] / fx2, cv[1] / fxy, cv[2] / fxy, cv[3] / fy2};
    memcpy(c->feature, feature_pos + 3 * i, sizeof(c->feature));
    int acc, st = sm_update(A, amu, asig, Z_S2, 2, z, h_visual, c, R, &acc);
    if (st != UWVK_OK) return st;
  }
  return UWVK_OK;
}

static int check_features(int nf, const double* features, const double* feature_cov) {
  for (int i = 0; i < nf; i++) /* checkMeasurment on every feature (the loop throws) */
    if (!finite_n(features + 2 * i, 2) || !finite_n(feature_cov + 4 * i, 4)) return 0;
  return 1;
}

/* IndirectPoseUKF::integrateMeasurement(features, positions, marker_pose, cov, camera, cam_in_body),
 * IndirectPoseUKF.cpp:94-135.  marker_pose, cam_in_body: t(3), q(4). */
int or_ipose_update_visual(or_ipose* f, int nf, const double* features, const double* feature_cov,
                           const double* feature_pos, const double marker_pose[7], const double cov_marker[36],
                           const double cam_cfg[4], const double cam_in_body[7]) {
  if (!check_features(nf, features, feature_cov)) return UWVK_ENAN;
  sm_manifold A = ipose_manifold(1);
  double amu[14], asig[144];
  memcpy(amu, f->mu, sizeof(double) * 7);
  memcpy(amu + 7, marker_pose, sizeof(double) * 7);
  memset(asig, 0, sizeof(asig));
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) {
      asig[i * 12 + j] = f->sigma[i * 6 + j];
      asig[(i + 6) * 12 + j + 6] = cov_marker[i * 6 + j];
    }
  vis_ctx c;
  memset(&c, 0, sizeof(c));
  c.indirect = 1;
  c.s_marker = 7;
  memcpy(c.cam, cam_in_body, sizeof(c.cam));
  memcpy(c.ref, f->pose_ref, sizeof(c.ref));
  int st = visual_loop(&A, amu, asig, &c, nf, features, feature_cov, feature_pos, cam_cfg);
  if (st != UWVK_OK) return st;
  memcpy(f->mu, amu, sizeof(double) * 7);
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) f->sigma[i * 6 + j] = asig[i * 12 + j];
  return UWVK_OK;
}

/* getCorrectedPose, IndirectPoseUKF.cpp:137-142: pose_ref * pose_error */
void or_ipose_get_corrected_pose(const or_ipose* f, double out[7]) {
  double t[3];
  or_quat_rotate(f->pose_ref + 3, f->mu, t);
  for (int k = 0; k < 3; k++) out[k] = f->pose_ref[k] + t[k];
  or_quat_mul(f->pose_ref + 3, f->mu + 3, out + 3);
}

size_t or_bottom_sizeof(void) { return sizeof(or_bottom); }
size_t or_ipose_sizeof(void) { return sizeof(or_ipose); }

/* ======================================================================== */
/* PoseUKF::integrateMeasurement(vector<VisualFeatureMeasurement>, ...)       */
/* PoseUKF.cpp:613-654 with PoseStateWithMarker (:221-229)                   */
/* ======================================================================== */
int or_pose_update_visual(or_pose* f, int nf, const double* features, const double* feature_cov,
                          const double* feature_pos, const double marker_pose[7], const double cov_marker[36],
                          const double cam_cfg[4], const double cam_in_imu[7]) {
  if (!check_features(nf, features, feature_cov)) return UWVK_ENAN;
  int n = f->L.dof, s = f->L.store, na = n + 6;
  sm_manifold A = {0};
  /* both SO3 segments take the PoseUKF side (or_set_so3_right): MTK has one
   * SO3::boxplus, so the marker orientation follows the filter's */
  const int so3 = or_get_so3_right() ? SEG_SO3R : SEG_SO3;
  sm_add(&A, SEG_V, 3);     /* position */
  sm_add(&A, so3, 3);       /* orientation */
  sm_add(&A, SEG_V, n - 6); /* velocity ... water_density */
  sm_add(&A, SEG_V, 3);     /* marker_position */
  sm_add(&A, so3, 3);       /* marker_orientation */
  static __thread double amu[SM_MAXS], asig[SM_MAXN * SM_MAXN];
  memcpy(amu, f->mu, sizeof(double) * s);
  memcpy(amu + s, marker_pose, sizeof(double) * 7);
  memset(asig, 0, sizeof(double) * na * na);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) asig[i * na + j] = f->sigma[i * n + j];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) asig[(n + i) * na + n + j] = cov_marker[i * 6 + j];
  vis_ctx c;
  memset(&c, 0, sizeof(c));
  c.indirect = 0;
  c.s_marker = s;
  memcpy(c.cam, cam_in_imu, sizeof(c.cam));
  int st = visual_loop(&A, amu, asig, &c, nf, features, feature_cov, feature_pos, cam_cfg);
  if (st != UWVK_OK) return st;
  memcpy(f->mu, amu, sizeof(double) * s);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) f->sigma[i * n + j] = asig[i * na + j];
  return UWVK_OK;
}
