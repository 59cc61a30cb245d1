/*
 * uwvk_oracle.c — CPU fp64 restatement of the PoseUKF / VelocityUKF hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see uwvk_oracle.h).  Compiled with
 * -ffp-contract=off so every product is rounded on its own, like the
 * reference's Eigen code on x86-64 without FMA.
 *
 * PARITY STATUS: UNPINNED against the reference binary.
 * [EXT] marks semantics of ukfom / MTK / pose_estimation / uwv_dynamic_model,
 * which are absent from /root/reference; they follow the frozen spec in
 * DESIGN.md §3.
 */
#include "uwvk_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define EARTHW 7.292115e-5 /* pose_estimation::EARTHW [EXT], used at PoseUKF.cpp:30,697 */
#define WGS84_A 6378137.0
#define WGS84_F (1.0 / 298.257223563)
#define D2P95 5.991 /* PoseUKF.cpp:275-286 */

/* ------------------------------------------------------------------------ */
/* layout (PoseState.hpp:29-45)                                              */
/* ------------------------------------------------------------------------ */
void or_layout_init(or_layout* L, int dof) {
  memset(L, 0, sizeof(*L));
  L->has_quat = 1;
  L->s_pos = 0; L->s_quat = 3; L->s_vel = 7; L->s_acc = 10; L->s_bg = 13; L->s_ba = 16; L->s_grav = 19;
  L->d_pos = 0; L->d_ori = 3; L->d_vel = 6; L->d_acc = 9; L->d_bg = 12; L->d_ba = 15; L->d_grav = 18;
  if (dof == UWVK_POSE_DOF_FULL) {
    L->dof = 53; L->store = 54; L->has_params = 1;
    L->s_inertia = 20; L->s_lin = 29; L->s_quad = 38; L->s_wv = 47; L->s_wvb = 49; L->s_badcp = 51; L->s_rho = 53;
    L->d_inertia = 19; L->d_lin = 28; L->d_quad = 37; L->d_wv = 46; L->d_wvb = 48; L->d_badcp = 50; L->d_rho = 52;
  } else {
    L->dof = 26; L->store = 27; L->has_params = 0;
    L->s_inertia = L->s_lin = L->s_quad = -1; L->d_inertia = L->d_lin = L->d_quad = -1;
    L->s_wv = 20; L->s_wvb = 22; L->s_badcp = 24; L->s_rho = 26;
    L->d_wv = 19; L->d_wvb = 21; L->d_badcp = 23; L->d_rho = 25;
  }
}

/* tangent index -> storage index for every non-orientation DOF */
static int dof_to_store(int d) { return d < 3 ? d : d + 1; }

/* ------------------------------------------------------------------------ */
/* quaternion / SO3 [EXT MTK SO3 + Eigen::Quaternion]                        */
/* ------------------------------------------------------------------------ */
void or_quat_mul(const double a[4], const double b[4], double o[4]) {
  double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
  double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
  o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

static void cross3(const double a[3], const double b[3], double o[3]) {
  double x = a[1] * b[2] - a[2] * b[1];
  double y = a[2] * b[0] - a[0] * b[2];
  double z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

/* Eigen QuaternionBase::_transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv */
void or_quat_rotate(const double q[4], const double v[3], double o[3]) {
  double uv[3], t[3];
  cross3(q + 1, v, uv);
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  cross3(q + 1, uv, t);
  for (int i = 0; i < 3; i++) o[i] = v[i] + q[0] * uv[i] + t[i];
}

void or_quat_rotate_inv(const double q[4], const double v[3], double o[3]) {
  double c[4] = {q[0], -q[1], -q[2], -q[3]};
  or_quat_rotate(c, v, o);
}

/* Eigen toRotationMatrix, row-major */
void or_quat_to_matrix(const double q[4], double R[9]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  double twx = tx * w, twy = ty * w, twz = tz * w;
  double txx = tx * x, txy = ty * x, txz = tz * x;
  double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

/* SO3::exp of a rotation vector (already scaled) [EXT]: (cos(t/2), sin(t/2) v/t) */
void or_so3_exp(const double v[3], double o[4]) {
  double t = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (t == 0.0) { o[0] = 1; o[1] = o[2] = o[3] = 0; return; }
  double h = 0.5 * t;
  double s = sin(h) / t;
  o[0] = cos(h); o[1] = s * v[0]; o[2] = s * v[1]; o[3] = s * v[2];
}

/* SO3::log [EXT]: shortest rotation vector, |theta| <= pi */
void or_so3_log(const double q[4], double o[3]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  if (w < 0) { w = -w; x = -x; y = -y; z = -z; }
  double nv = sqrt(x * x + y * y + z * z);
  if (nv == 0.0) { o[0] = o[1] = o[2] = 0; return; }
  double k = 2.0 * atan2(nv, w) / nv;
  o[0] = k * x; o[1] = k * y; o[2] = k * z;
}

/* SO3 boxplus side [EXT MTK], SURVEY §8(c) item 5: the largest unpinned semantic.
 * 1 (default since r05): body-frame / right, q [+] d = q * exp(d), MTK's published
 *   SO3::boxplus (Hertzberg et al. 2013).  The reference's arithmetic goes through
 *   MTK (mtkwrap<MTK::SO3<double>>, PoseState.hpp:15; orientation.boxplus,
 *   PoseUKF.cpp:32), whatever frame the caller meant when it rotated omega into
 *   nav (PoseUKF.cpp:31) -- this overrides SURVEY §8(c) item 5's left default
 *   (DESIGN.md §3).
 * 0: nav-frame / left, q [+] d = exp(d) * q, kept as an option (or_set_so3_right(0)).
 * Applies to every PoseUKF orientation [+]/[-], including processModel's
 * new_state.orientation.boxplus (PoseUKF.cpp:32).  The HIP engine has the same
 * switch (UWVK_OPT_SO3_RIGHT, default 1); tests/test_oracle_kat.py shows the two
 * conventions give materially different C3 trajectories. */
static int g_so3_right = 1;
void or_set_so3_right(int on) { g_so3_right = on ? 1 : 0; }
int or_get_so3_right(void) { return g_so3_right; }

/* q [+] v for an already scaled rotation vector v */
static void so3_plus(const double q[4], const double v[3], double o[4]) {
  double e[4];
  or_so3_exp(v, e);
  if (g_so3_right) or_quat_mul(q, e, o);
  else or_quat_mul(e, q, o);
}

/* compound-manifold boxplus: vect x + s*d; SO3 exp(s*d) * q (left) or q * exp(s*d) (right) */
void or_boxplus(const or_layout* L, const double* x, const double* d, double s, double* o) {
  double tmp[OR_MAXS];
  for (int k = 0; k < L->dof; k++) {
    if (k >= 3 && k < 6) continue;
    int si = dof_to_store(k);
    tmp[si] = x[si] + s * d[k];
  }
  double v[3] = {s * d[3], s * d[4], s * d[5]};
  so3_plus(x + 3, v, tmp + 3);
  memcpy(o, tmp, sizeof(double) * L->store);
}

/* a boxminus b: vect a - b; SO3 log(a * b^-1) (left) or log(b^-1 * a) (right) */
void or_boxminus(const or_layout* L, const double* a, const double* b, double* o) {
  for (int k = 0; k < L->dof; k++) {
    if (k >= 3 && k < 6) continue;
    int si = dof_to_store(k);
    o[k] = a[si] - b[si];
  }
  double bc[4] = {b[3], -b[4], -b[5], -b[6]}, r[4];
  if (g_so3_right) or_quat_mul(bc, a + 3, r);
  else or_quat_mul(a + 3, bc, r);
  or_so3_log(r, o + 3);
}

/* ------------------------------------------------------------------------ */
/* dense helpers                                                              */
/* ------------------------------------------------------------------------ */
int or_cholesky(int n, const double* A, double* Lo) {
  for (int i = 0; i < n * n; i++) Lo[i] = 0.0;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j <= i; j++) {
      double s = A[i * n + j];
      for (int k = 0; k < j; k++) s -= Lo[i * n + k] * Lo[j * n + k];
      if (i == j) {
        if (!(s > 0.0)) return -1;
        Lo[i * n + i] = sqrt(s);
      } else {
        Lo[i * n + j] = s / Lo[j * n + j];
      }
    }
  }
  return 0;
}

/* m x m inverse: closed forms for m <= 3 (Eigen compute_inverse), Gauss-Jordan
 * with partial pivoting otherwise (Eigen PartialPivLU) */
int or_invert(int n, const double* A, double* X) {
  if (n == 1) { X[0] = 1.0 / A[0]; return 0; }
  if (n == 2) {
    double det = A[0] * A[3] - A[1] * A[2];
    double id = 1.0 / det;
    X[0] = A[3] * id; X[1] = -A[1] * id; X[2] = -A[2] * id; X[3] = A[0] * id;
    return 0;
  }
  if (n == 3) {
    double c00 = A[4] * A[8] - A[5] * A[7];
    double c01 = A[5] * A[6] - A[3] * A[8];
    double c02 = A[3] * A[7] - A[4] * A[6];
    double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    double id = 1.0 / det;
    X[0] = c00 * id;
    X[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    X[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    X[3] = c01 * id;
    X[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    X[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    X[6] = c02 * id;
    X[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    X[8] = (A[0] * A[4] - A[1] * A[3]) * id;
    return 0;
  }
  double M[6 * 12];
  if (n > 6) return -1;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < 2 * n; j++) M[i * 2 * n + j] = j < n ? A[i * n + j] : (j - n == i ? 1.0 : 0.0);
  for (int c = 0; c < n; c++) {
    int p = c;
    for (int r = c + 1; r < n; r++)
      if (fabs(M[r * 2 * n + c]) > fabs(M[p * 2 * n + c])) p = r;
    if (M[p * 2 * n + c] == 0.0) return -1;
    if (p != c)
      for (int j = 0; j < 2 * n; j++) {
        double t = M[c * 2 * n + j]; M[c * 2 * n + j] = M[p * 2 * n + j]; M[p * 2 * n + j] = t;
      }
    double ip = 1.0 / M[c * 2 * n + c];
    for (int j = 0; j < 2 * n; j++) M[c * 2 * n + j] *= ip;
    for (int r = 0; r < n; r++) {
      if (r == c) continue;
      double f = M[r * 2 * n + c];
      if (f == 0.0) continue;
      for (int j = 0; j < 2 * n; j++) M[r * 2 * n + j] -= f * M[c * 2 * n + j];
    }
  }
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) X[i * n + j] = M[i * 2 * n + n + j];
  return 0;
}

static int finite_arr(const double* a, int n) {
  for (int i = 0; i < n; i++)
    if (!isfinite(a[i])) return 0;
  return 1;
}

/* ------------------------------------------------------------------------ */
/* geography [EXT pose_estimation::GeographicProjection / GravitationalModel] */
/* ------------------------------------------------------------------------ */
static void radii(double lat0, double* rm, double* rn) {
  double e2 = WGS84_F * (2.0 - WGS84_F);
  double s = sin(lat0);
  double den = 1.0 - e2 * s * s;
  double sq = sqrt(den);
  *rn = WGS84_A / sq;
  *rm = WGS84_A * (1.0 - e2) / (den * sq);
}

void or_nav_to_world(const uwvk_location* loc, double x, double y, double* lat, double* lon) {
  double rm, rn;
  radii(loc->latitude, &rm, &rn);
  *lat = loc->latitude + x / rm;
  *lon = loc->longitude - y / (rn * cos(loc->latitude));
}

void or_world_to_nav(const uwvk_location* loc, double lat, double lon, double* x, double* y) {
  double rm, rn;
  radii(loc->latitude, &rm, &rn);
  *x = (lat - loc->latitude) * rm;
  *y = -(lon - loc->longitude) * (rn * cos(loc->latitude));
}

double or_wgs84_gravity(double lat, double alt) {
  double s2 = sin(lat) * sin(lat);
  return 9.7803253359 * (1.0 + 0.00193185265241 * s2) / sqrt(1.0 - 0.00669437999013 * s2) - 3.086e-6 * alt;
}

static void earth_rotation(const uwvk_location* loc, double x, double y, double o[3]) {
  double lat, lon;
  or_nav_to_world(loc, x, y, &lat, &lon); /* PoseUKF.cpp:28-30 */
  o[0] = EARTHW * cos(lat);
  o[1] = 0.0;
  o[2] = EARTHW * sin(lat);
}

/* ------------------------------------------------------------------------ */
/* [EXT] uwv_dynamic_model: calcEfforts and the RK4 ModelSimulation step     */
/* ------------------------------------------------------------------------ */
static void restoring(const uwvk_uwv_params* p, const double q[4], double g[6]) {
  double fw[3] = {0, 0, -p->weight}, fb[3] = {0, 0, p->buoyancy}, fg[3], fbb[3], mg[3], mb[3];
  or_quat_rotate_inv(q, fw, fg);
  or_quat_rotate_inv(q, fb, fbb);
  cross3(p->distance_body2centerofgravity, fg, mg);
  cross3(p->distance_body2centerofbuoyancy, fbb, mb);
  for (int i = 0; i < 3; i++) {
    g[i] = -(fg[i] + fbb[i]);
    g[3 + i] = -(mg[i] + mb[i]);
  }
}

static void coriolis(const double* M, const double nu[6], double c[6]) {
  double a[3], b[3], t0[3], t1[3], t2[3];
  for (int i = 0; i < 3; i++) {
    a[i] = 0; b[i] = 0;
    for (int j = 0; j < 6; j++) {
      a[i] += M[i * 6 + j] * nu[j];
      b[i] += M[(3 + i) * 6 + j] * nu[j];
    }
  }
  cross3(nu + 3, a, t0); /* w x a */
  cross3(nu, a, t1);     /* v x a */
  cross3(nu + 3, b, t2); /* w x b */
  for (int i = 0; i < 3; i++) { c[i] = t0[i]; c[3 + i] = t1[i] + t2[i]; }
}

static void damping(const uwvk_uwv_params* p, const double nu[6], double d[6]) {
  for (int i = 0; i < 6; i++) {
    double sl = 0, sq = 0;
    for (int j = 0; j < 6; j++) {
      sl += p->damping_matrices[0][i * 6 + j] * nu[j];
      sq += p->damping_matrices[1][i * 6 + j] * (fabs(nu[j]) * nu[j]);
    }
    d[i] = sl + sq;
  }
}

void or_calc_efforts(const uwvk_uwv_params* p, const double acc6[6], const double vel6[6], const double q[4],
                     double tau[6]) {
  double c[6], d[6], g[6];
  coriolis(p->inertia_matrix, vel6, c);
  damping(p, vel6, d);
  restoring(p, q, g);
  for (int i = 0; i < 6; i++) {
    double m = 0;
    for (int j = 0; j < 6; j++) m += p->inertia_matrix[i * 6 + j] * acc6[j];
    tau[i] = m + c[i] + d[i] + g[i];
  }
}

static void model_deriv(const uwvk_uwv_params* p, const double Minv[36], const double tau[6], const double s[13],
                        double ds[13]) {
  const double* q = s + 3;
  double nu[6] = {s[7], s[8], s[9], s[10], s[11], s[12]};
  or_quat_rotate(q, s + 7, ds); /* p_dot = R(q) v */
  double wq[4] = {0, s[10], s[11], s[12]}, qd[4];
  or_quat_mul(q, wq, qd);
  for (int i = 0; i < 4; i++) ds[3 + i] = 0.5 * qd[i];
  double c[6], d[6], g[6], r[6];
  coriolis(p->inertia_matrix, nu, c);
  damping(p, nu, d);
  restoring(p, q, g);
  for (int i = 0; i < 6; i++) r[i] = tau[i] - c[i] - d[i] - g[i];
  for (int i = 0; i < 6; i++) {
    double a = 0;
    for (int j = 0; j < 6; j++) a += Minv[i * 6 + j] * r[j];
    ds[7 + i] = a;
  }
}

void or_model_rk4(const uwvk_uwv_params* p, const double Minv[36], const double tau[6], double dt,
                  const double s[13], double o[13]) {
  double k1[13], k2[13], k3[13], k4[13], t[13];
  model_deriv(p, Minv, tau, s, k1);
  for (int i = 0; i < 13; i++) t[i] = s[i] + 0.5 * dt * k1[i];
  model_deriv(p, Minv, tau, t, k2);
  for (int i = 0; i < 13; i++) t[i] = s[i] + 0.5 * dt * k2[i];
  model_deriv(p, Minv, tau, t, k3);
  for (int i = 0; i < 13; i++) t[i] = s[i] + dt * k3[i];
  model_deriv(p, Minv, tau, t, k4);
  for (int i = 0; i < 13; i++) o[i] = s[i] + (dt / 6.0) * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
  double n = sqrt(o[3] * o[3] + o[4] * o[4] + o[5] * o[5] + o[6] * o[6]);
  for (int i = 3; i < 7; i++) o[i] /= n;
}

/* ------------------------------------------------------------------------ */
/* generic UKF core [EXT ukfom::ukf] on a compound manifold                  */
/* ------------------------------------------------------------------------ */
typedef struct manifold {
  int dof, store, has_quat;
  const or_layout* L; /* NULL for the all-vector VelocityState */
} manifold;

static void m_boxplus(const manifold* M, const double* x, const double* d, double s, double* o) {
  if (M->has_quat) { or_boxplus(M->L, x, d, s, o); return; }
  for (int k = 0; k < M->dof; k++) o[k] = x[k] + s * d[k];
}
static void m_boxminus(const manifold* M, const double* a, const double* b, double* o) {
  if (M->has_quat) { or_boxminus(M->L, a, b, o); return; }
  for (int k = 0; k < M->dof; k++) o[k] = a[k] - b[k];
}

#define NPTS (2 * OR_MAXN + 1)

/* generateSigmaPoints: X0 = mu, X_{2j+1} = mu [+] L_j, X_{2j+2} = mu [+] -L_j */
static int sigma_points(const manifold* M, const double* mu, const double* sigma, double* X) {
  int n = M->dof;
  double L[OR_MAXN * OR_MAXN], col[OR_MAXN];
  if (or_cholesky(n, sigma, L) != 0) return -1;
  memcpy(X, mu, sizeof(double) * M->store);
  for (int j = 0; j < n; j++) {
    for (int r = 0; r < n; r++) col[r] = L[r * n + j];
    m_boxplus(M, mu, col, 1.0, X + (2 * j + 1) * OR_MAXS);
    m_boxplus(M, mu, col, -1.0, X + (2 * j + 2) * OR_MAXS);
  }
  return 0;
}

/* meanSigmaPoints on the manifold: Gauss-Newton, |delta| <= 1e-6, max 1e4 it. */
static int mean_points(const manifold* M, const double* X, int N, double* ref) {
  int n = M->dof, it = 0;
  double d[OR_MAXN], dd[OR_MAXN], nrm;
  memcpy(ref, X, sizeof(double) * M->store);
  do {
    for (int k = 0; k < n; k++) d[k] = 0.0;
    for (int p = 0; p < N; p++) {
      m_boxminus(M, X + p * OR_MAXS, ref, dd);
      for (int k = 0; k < n; k++) d[k] += dd[k];
    }
    nrm = 0.0;
    for (int k = 0; k < n; k++) { d[k] /= (double)N; nrm += d[k] * d[k]; }
    m_boxplus(M, ref, d, 1.0, ref);
    nrm = sqrt(nrm);
  } while (nrm > 1e-6 && ++it < 10000);
  return it + 1;
}

/* covSigmaPoints: 0.5 * sum (X_p [-] mean)(X_p [-] mean)^T */
static void cov_points(const manifold* M, const double* mean, const double* X, int N, double* S) {
  int n = M->dof;
  double d[OR_MAXN];
  for (int i = 0; i < n * n; i++) S[i] = 0.0;
  for (int p = 0; p < N; p++) {
    m_boxminus(M, X + p * OR_MAXS, mean, d);
    for (int i = 0; i < n; i++)
      for (int j = 0; j < n; j++) S[i * n + j] += d[i] * d[j];
  }
  for (int i = 0; i < n * n; i++) S[i] = 0.5 * S[i];
}

typedef void (*process_fn)(void* ctx, const double* x, double* out);
typedef void (*meas_fn)(void* ctx, const double* x, double* z);

static int ukf_predict(const manifold* M, double* mu, double* sigma, process_fn g, void* ctx, const double* Qp,
                       int* iters) {
  static __thread double X[NPTS * OR_MAXS];
  int n = M->dof, N = 2 * n + 1;
  if (sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  for (int p = 0; p < N; p++) g(ctx, X + p * OR_MAXS, X + p * OR_MAXS); /* std::transform */
  int it = mean_points(M, X, N, mu);
  if (iters) *iters = it;
  cov_points(M, mu, X, N, sigma);
  for (int i = 0; i < n * n; i++) sigma[i] += Qp[i];
  return UWVK_OK;
}

static int apply_delta(const manifold* M, double* mu, double* sigma, const double* delta) {
  static __thread double X[NPTS * OR_MAXS];
  int n = M->dof, N = 2 * n + 1;
  if (sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  m_boxplus(M, mu, delta, 1.0, mu);
  for (int p = 0; p < N; p++) m_boxplus(M, X + p * OR_MAXS, delta, 1.0, X + p * OR_MAXS);
  cov_points(M, mu, X, N, sigma);
  return UWVK_OK;
}

/* zmode 0: Eigen-vector measurement (plain average); 1: vect manifold (iterative mean)
 * gate: 0 accept any; 1 d2p95 */
static int ukf_update(const manifold* M, double* mu, double* sigma, int m, const double* z, meas_fn h, void* ctx,
                      const double* R, int zmode, int gate, int* accepted) {
  static __thread double X[NPTS * OR_MAXS];
  static __thread double Z[NPTS * 6];
  int n = M->dof, N = 2 * n + 1;
  double zm[6], S[36], Si[36], C[OR_MAXN * 6], K[OR_MAXN * 6], nu[6], dx[OR_MAXN], dz[6];
  *accepted = 0;
  if (sigma_points(M, mu, sigma, X) != 0) return UWVK_ENOTPD;
  for (int p = 0; p < N; p++) h(ctx, X + p * OR_MAXS, Z + p * 6);
  if (zmode == 0) {
    for (int a = 0; a < m; a++) zm[a] = 0.0;
    for (int p = 0; p < N; p++)
      for (int a = 0; a < m; a++) zm[a] += Z[p * 6 + a];
    for (int a = 0; a < m; a++) zm[a] = zm[a] / (double)N;
  } else {
    int it = 0;
    double d[6], nrm;
    for (int a = 0; a < m; a++) zm[a] = Z[a];
    do {
      for (int a = 0; a < m; a++) d[a] = 0.0;
      for (int p = 0; p < N; p++)
        for (int a = 0; a < m; a++) d[a] += Z[p * 6 + a] - zm[a];
      nrm = 0.0;
      for (int a = 0; a < m; a++) { d[a] /= (double)N; nrm += d[a] * d[a]; }
      for (int a = 0; a < m; a++) zm[a] = zm[a] + d[a];
      nrm = sqrt(nrm);
    } while (nrm > 1e-6 && ++it < 10000);
  }
  for (int i = 0; i < m * m; i++) S[i] = 0.0;
  for (int i = 0; i < n * m; i++) C[i] = 0.0;
  for (int p = 0; p < N; p++) {
    for (int a = 0; a < m; a++) dz[a] = Z[p * 6 + a] - zm[a];
    m_boxminus(M, X + p * OR_MAXS, mu, dx);
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
  for (int a = 0; a < m; a++) nu[a] = z[a] - zm[a];
  double d2 = 0.0;
  for (int b = 0; b < m; b++) {
    double t = 0.0;
    for (int a = 0; a < m; a++) t += nu[a] * Si[a * m + b];
    d2 += t * nu[b];
  }
  int ok = gate == 0 ? 1 : !(d2 > D2P95);
  if (!ok) return UWVK_OK;
  *accepted = 1;
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0.0;
      for (int a = 0; a < m; a++) s += C[i * m + a] * K[j * m + a];
      sigma[i * n + j] -= s;
    }
  double delta[OR_MAXN];
  for (int i = 0; i < n; i++) {
    double s = 0.0;
    for (int a = 0; a < m; a++) s += K[i * m + a] * nu[a];
    delta[i] = s;
  }
  return apply_delta(M, mu, sigma, delta);
}

/* ------------------------------------------------------------------------ */
/* PoseUKF                                                                    */
/* ------------------------------------------------------------------------ */
static manifold pose_manifold(const or_pose* f) {
  manifold M = {f->L.dof, f->L.store, 1, &f->L};
  return M;
}

static const int P_IDX[3] = {0, 1, 5}; /* (surge, sway, yaw) rows/cols, PoseUKF.cpp:160-171 */

int or_pose_init_from_config(or_pose* f, int dof, const double pos[3], const double pos_cov[9], const double rot[4],
                             const double rot_cov[9], const uwvk_pose_config* cfg, const uwvk_uwv_params* uwv,
                             const double imu_in_body[7]) {
  memset(f, 0, sizeof(*f));
  or_layout_init(&f->L, dof);
  const or_layout* L = &f->L;
  int n = L->dof;
  double qb[4] = {1, 0, 0, 0}, tb[3] = {0, 0, 0}, Mb[9];
  if (imu_in_body) { memcpy(tb, imu_in_body, 3 * sizeof(double)); memcpy(qb, imu_in_body + 3, 4 * sizeof(double)); }
  or_quat_to_matrix(qb, Mb);
  double* x = f->mu;
  /* PoseUKF.cpp:293-320 */
  memcpy(x + L->s_pos, pos, 3 * sizeof(double));
  memcpy(x + L->s_quat, rot, 4 * sizeof(double));
  for (int i = 0; i < 3; i++) {
    x[L->s_vel + i] = 0.0;
    x[L->s_acc + i] = 0.0;
    double sg = 0, sa = 0;
    for (int k = 0; k < 3; k++) {
      sg += Mb[i * 3 + k] * cfg->rotation_rate.bias_offset[k];
      sa += Mb[i * 3 + k] * cfg->acceleration.bias_offset[k];
    }
    x[L->s_bg + i] = sg;
    x[L->s_ba + i] = sa;
  }
  x[L->s_grav] = or_wgs84_gravity(cfg->location.latitude, cfg->location.altitude);
  if (L->has_params) {
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        x[L->s_inertia + a + 3 * b] = uwv->inertia_matrix[P_IDX[a] * 6 + P_IDX[b]];
        x[L->s_lin + a + 3 * b] = uwv->damping_matrices[0][P_IDX[a] * 6 + P_IDX[b]];
        x[L->s_quad + a + 3 * b] = uwv->damping_matrices[1][P_IDX[a] * 6 + P_IDX[b]];
      }
  }
  for (int i = 0; i < 2; i++) x[L->s_wv + i] = x[L->s_wvb + i] = x[L->s_badcp + i] = 0.0;
  x[L->s_rho] = cfg->hydrostatics.water_density;
  /* PoseUKF.cpp:323-341 */
  double* P = f->sigma;
  for (int i = 0; i < n * n; i++) P[i] = 0.0;
#define PB(d0, r, c, v) P[((d0) + (r)) * n + (d0) + (c)] = (v)
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      PB(L->d_pos, r, c, pos_cov[r * 3 + c]);
      PB(L->d_ori, r, c, rot_cov[r * 3 + c]);
      PB(L->d_vel, r, c, r == c ? 1.0 : 0.0);
      PB(L->d_acc, r, c, r == c ? 10.0 : 0.0);
      double sg = 0, sa = 0;
      for (int k = 0; k < 3; k++) {
        double bg = cfg->rotation_rate.bias_instability[k], ba = cfg->acceleration.bias_instability[k];
        sg += Mb[r * 3 + k] * (bg * bg) * Mb[c * 3 + k];
        sa += Mb[r * 3 + k] * (ba * ba) * Mb[c * 3 + k];
      }
      PB(L->d_bg, r, c, sg);
      PB(L->d_ba, r, c, sa);
    }
  PB(L->d_grav, 0, 0, pow(0.05, 2.));
  if (L->has_params)
    for (int k = 0; k < 9; k++) {
      double a = cfg->model_noise_parameters.inertia_instability[k];
      double b = cfg->model_noise_parameters.lin_damping_instability[k];
      double c = cfg->model_noise_parameters.quad_damping_instability[k];
      PB(L->d_inertia, k, k, a * a);
      PB(L->d_lin, k, k, b * b);
      PB(L->d_quad, k, k, c * c);
    }
  double wl = pow(cfg->water_velocity.limits, 2), al = pow(cfg->water_velocity.adcp_bias_limits, 2);
  for (int k = 0; k < 2; k++) {
    PB(L->d_wv, k, k, wl);
    PB(L->d_wvb, k, k, wl);
    PB(L->d_badcp, k, k, al);
  }
  PB(L->d_rho, 0, 0, pow(cfg->hydrostatics.water_density_limits, 2.));
#undef PB
  /* PoseUKF.cpp:346-371 */
  if (L->has_params) {
    memcpy(f->inertia_offset, x + L->s_inertia, 9 * sizeof(double));
    memcpy(f->lin_damping_offset, x + L->s_lin, 9 * sizeof(double));
    memcpy(f->quad_damping_offset, x + L->s_quad, 9 * sizeof(double));
  }
  f->water_density_offset = x[L->s_rho];
  f->uwv = *uwv;
  f->location = cfg->location;
  uwvk_pose_parameter* p = &f->param;
  memcpy(p->imu_in_body, tb, 3 * sizeof(double));
  p->acc_bias_tau = cfg->acceleration.bias_tau;
  memcpy(p->acc_bias_offset, x + L->s_ba, 3 * sizeof(double));
  p->gyro_bias_tau = cfg->rotation_rate.bias_tau;
  memcpy(p->gyro_bias_offset, x + L->s_bg, 3 * sizeof(double));
  p->inertia_tau = cfg->model_noise_parameters.inertia_tau;
  p->lin_damping_tau = cfg->model_noise_parameters.lin_damping_tau;
  p->quad_damping_tau = cfg->model_noise_parameters.quad_damping_tau;
  p->water_velocity_tau = cfg->water_velocity.tau;
  p->water_velocity_limits = cfg->water_velocity.limits;
  p->water_velocity_scale = cfg->water_velocity.scale;
  p->adcp_bias_tau = cfg->water_velocity.adcp_bias_tau;
  p->atmospheric_pressure = cfg->hydrostatics.atmospheric_pressure;
  p->water_density_tau = cfg->hydrostatics.water_density_tau;
  return UWVK_OK;
}

int or_pose_init_from_state(or_pose* f, int dof, const double* x, const double* P, const uwvk_location* loc,
                            const uwvk_uwv_params* uwv, const uwvk_pose_parameter* param) {
  memset(f, 0, sizeof(*f));
  or_layout_init(&f->L, dof);
  const or_layout* L = &f->L;
  memcpy(f->mu, x, sizeof(double) * L->store);
  memcpy(f->sigma, P, sizeof(double) * L->dof * L->dof);
  f->param = *param;
  f->uwv = *uwv;
  f->location = *loc;
  if (L->has_params) {
    memcpy(f->inertia_offset, x + L->s_inertia, 9 * sizeof(double));
    memcpy(f->lin_damping_offset, x + L->s_lin, 9 * sizeof(double));
    memcpy(f->quad_damping_offset, x + L->s_quad, 9 * sizeof(double));
  }
  f->water_density_offset = x[L->s_rho];
  return UWVK_OK;
}

/* PoseUKF.cpp:393-439 */
void or_pose_set_process_noise_from_config(or_pose* f, const uwvk_pose_config* cfg, double dt,
                                           const double q_imu_in_body[4]) {
  const or_layout* L = &f->L;
  int n = L->dof;
  double qb[4] = {1, 0, 0, 0}, M[9];
  if (q_imu_in_body) memcpy(qb, q_imu_in_body, 4 * sizeof(double));
  or_quat_to_matrix(qb, M);
  double* Q = f->Q;
  for (int i = 0; i < n * n; i++) Q[i] = 0.0;
#define QB(d0, r, c, v) Q[((d0) + (r)) * n + (d0) + (c)] = (v)
  for (int r = 0; r < 3; r++) {
    double j = cfg->max_jerk[r];
    double jp = (1. / 6.) * 0.25 * j, jv = 0.5 * 0.25 * j, ja = 0.25 * j;
    QB(L->d_pos, r, r, 1.5 * (pow(dt, 4.0) * (jp * jp)));
    QB(L->d_vel, r, r, 1.5 * (pow(dt, 2.0) * (jv * jv)));
    QB(L->d_acc, r, r, ja * ja);
  }
  double kg = 2. / (cfg->rotation_rate.bias_tau * dt), ka = 2. / (cfg->acceleration.bias_tau * dt);
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double so = 0, sg = 0, sa = 0;
      for (int k = 0; k < 3; k++) {
        double rw = cfg->rotation_rate.randomwalk[k];
        double bg = cfg->rotation_rate.bias_instability[k], ba = cfg->acceleration.bias_instability[k];
        so += M[r * 3 + k] * (rw * rw) * M[c * 3 + k];
        sg += M[r * 3 + k] * (kg * (bg * bg)) * M[c * 3 + k];
        sa += M[r * 3 + k] * (ka * (ba * ba)) * M[c * 3 + k];
      }
      QB(L->d_ori, r, c, so);
      QB(L->d_bg, r, c, sg);
      QB(L->d_ba, r, c, sa);
    }
  QB(L->d_grav, 0, 0, 1.e-12);
  if (L->has_params) {
    const uwvk_model_noise* mn = &cfg->model_noise_parameters;
    for (int k = 0; k < 9; k++) {
      QB(L->d_inertia, k, k, (2. / (mn->inertia_tau * dt)) * (mn->inertia_instability[k] * mn->inertia_instability[k]));
      QB(L->d_lin, k, k,
         (2. / (mn->lin_damping_tau * dt)) * (mn->lin_damping_instability[k] * mn->lin_damping_instability[k]));
      QB(L->d_quad, k, k,
         (2. / (mn->quad_damping_tau * dt)) * (mn->quad_damping_instability[k] * mn->quad_damping_instability[k]));
    }
  }
  double qwv = (2. / (cfg->water_velocity.tau * dt)) * pow(cfg->water_velocity.limits, 2);
  double qad = (2. / (cfg->water_velocity.adcp_bias_tau * dt)) * pow(cfg->water_velocity.adcp_bias_limits, 2);
  for (int k = 0; k < 2; k++) {
    QB(L->d_wv, k, k, qwv);
    QB(L->d_wvb, k, k, qwv);
    QB(L->d_badcp, k, k, qad);
  }
  QB(L->d_rho, 0, 0, (2. / (cfg->hydrostatics.water_density_tau * dt)) * pow(cfg->hydrostatics.water_density_limits, 2.));
#undef QB
}

void or_pose_set_process_noise(or_pose* f, const double* Q) {
  memcpy(f->Q, Q, sizeof(double) * f->L.dof * f->L.dof);
}

int or_pose_set_rotation_rate(or_pose* f, const double w[3], const double* cov) {
  if (!finite_arr(w, 3) || (cov && !finite_arr(cov, 9))) return UWVK_ENAN;
  memcpy(f->rotation_rate, w, 3 * sizeof(double)); /* PoseUKF.cpp:492-496 */
  return UWVK_OK;
}

/* processModel, PoseUKF.cpp:12-84 */
static void pose_process(void* ctx, const double* x, double* o) {
  const or_pose* f = (const or_pose*)((void**)ctx)[0];
  double dt = *(const double*)((void**)ctx)[1];
  const or_layout* L = &f->L;
  const uwvk_pose_parameter* P = &f->param;
  double s[OR_MAXS];
  memcpy(s, x, sizeof(double) * L->store);
  for (int i = 0; i < 3; i++) s[L->s_pos + i] = x[L->s_pos + i] + dt * x[L->s_vel + i];
  double er[3], wb[3], wn[3];
  earth_rotation(&f->location, x[L->s_pos], x[L->s_pos + 1], er);
  for (int i = 0; i < 3; i++) wb[i] = f->rotation_rate[i] - x[L->s_bg + i];
  or_quat_rotate(x + L->s_quat, wb, wn);
  for (int i = 0; i < 3; i++) wn[i] = (wn[i] - er[i]) * dt;
  so3_plus(x + L->s_quat, wn, s + L->s_quat); /* new_state.orientation.boxplus(w, dt), :32 */
  for (int i = 0; i < 3; i++) s[L->s_vel + i] = x[L->s_vel + i] + dt * x[L->s_acc + i];
  for (int i = 0; i < 3; i++) {
    double dg = (-1.0 / P->gyro_bias_tau) * (x[L->s_bg + i] - P->gyro_bias_offset[i]);
    s[L->s_bg + i] = x[L->s_bg + i] + dt * dg;
    double da = (-1.0 / P->acc_bias_tau) * (x[L->s_ba + i] - P->acc_bias_offset[i]);
    s[L->s_ba + i] = x[L->s_ba + i] + dt * da;
  }
  if (L->has_params)
    for (int k = 0; k < 9; k++) {
      double di = (-1.0 / P->inertia_tau) * (x[L->s_inertia + k] - f->inertia_offset[k]);
      s[L->s_inertia + k] = x[L->s_inertia + k] + dt * di;
      double dl = (-1.0 / P->lin_damping_tau) * (x[L->s_lin + k] - f->lin_damping_offset[k]);
      s[L->s_lin + k] = x[L->s_lin + k] + dt * dl;
      double dq = (-1.0 / P->quad_damping_tau) * (x[L->s_quad + k] - f->quad_damping_offset[k]);
      s[L->s_quad + k] = x[L->s_quad + k] + dt * dq;
    }
  for (int k = 0; k < 2; k++) {
    double dw = (-1.0 / P->water_velocity_tau) * x[L->s_wv + k];
    s[L->s_wv + k] = x[L->s_wv + k] + dt * dw;
    double db = (-1.0 / P->water_velocity_tau) * x[L->s_wvb + k];
    s[L->s_wvb + k] = x[L->s_wvb + k] + dt * db;
    double da = (-1.0 / P->adcp_bias_tau) * x[L->s_badcp + k];
    s[L->s_badcp + k] = x[L->s_badcp + k] + dt * da;
  }
  double dr = (-1.0 / P->water_density_tau) * (x[L->s_rho] - f->water_density_offset);
  s[L->s_rho] = x[L->s_rho] + dt * dr;
  memcpy(o, s, sizeof(double) * L->store);
}

/* predictionStepImpl, PoseUKF.cpp:446-465 */
int or_pose_predict(or_pose* f, double dt) {
  const or_layout* L = &f->L;
  int n = L->dof;
  double Qp[OR_MAXN * OR_MAXN], R[9];
  memcpy(Qp, f->Q, sizeof(double) * n * n);
  or_quat_to_matrix(f->mu + L->s_quat, R);
  int o = L->d_ori;
  for (int r = 0; r < 3; r++)
    for (int c = 0; c < 3; c++) {
      double s = 0.0;
      for (int k = 0; k < 3; k++) {
        double t = 0.0;
        for (int l = 0; l < 3; l++) t += R[r * 3 + l] * f->Q[(o + l) * n + o + k];
        s += t * R[c * 3 + k];
      }
      Qp[(o + r) * n + o + c] = s;
    }
  double vs[3] = {f->mu[L->s_vel], f->mu[L->s_vel + 1], 10 * f->mu[L->s_vel + 2]};
  double add = f->param.water_velocity_scale * (vs[0] * vs[0] + vs[1] * vs[1] + vs[2] * vs[2]) * dt;
  for (int k = 0; k < 2; k++) {
    Qp[(L->d_wv + k) * n + L->d_wv + k] = f->Q[(L->d_wv + k) * n + L->d_wv + k] + add;
    Qp[(L->d_wvb + k) * n + L->d_wvb + k] = f->Q[(L->d_wvb + k) * n + L->d_wvb + k] + add;
  }
  double dt2 = pow(dt, 2.);
  for (int i = 0; i < n * n; i++) Qp[i] = dt2 * Qp[i];
  manifold M = pose_manifold(f);
  void* ctx[2] = {f, &dt};
  return ukf_predict(&M, f->mu, f->sigma, pose_process, ctx, Qp, &f->last_mean_iterations);
}

typedef struct meas_ctx {
  const or_pose* f;
  double v3[3], w3[3], wb[3], ab[3], q[4];
  double cw;
  const uwvk_uwv_params* uwv;
  uwvk_uwv_params* uwv_mut;
} meas_ctx;

static void h_acc(void* c, const double* x, double* z) { /* PoseUKF.cpp:125-131 */
  const or_layout* L = &((meas_ctx*)c)->f->L;
  double a[3] = {x[L->s_acc], x[L->s_acc + 1], x[L->s_acc + 2] + x[L->s_grav]}, r[3];
  or_quat_rotate_inv(x + L->s_quat, a, r);
  for (int i = 0; i < 3; i++) z[i] = r[i] + x[L->s_ba + i];
}
static void h_vel(void* c, const double* x, double* z) { /* PoseUKF.cpp:117-123 */
  const or_layout* L = &((meas_ctx*)c)->f->L;
  or_quat_rotate_inv(x + L->s_quat, x + L->s_vel, z);
}
static void h_pressure(void* c, const double* x, double* z) { /* PoseUKF.cpp:107-115 */
  meas_ctx* m = (meas_ctx*)c;
  const or_layout* L = &m->f->L;
  double r[3];
  or_quat_rotate(x + L->s_quat, m->v3, r);
  double pz = x[L->s_pos + 2] + r[2];
  z[0] = m->f->param.atmospheric_pressure - pz * x[L->s_grav] * x[L->s_rho];
}
static void h_water(void* c, const double* x, double* z) { /* PoseUKF.cpp:133-151 */
  meas_ctx* m = (meas_ctx*)c;
  const or_layout* L = &m->f->L;
  double vb[3] = {x[L->s_vel] - x[L->s_wvb], x[L->s_vel + 1] - x[L->s_wvb + 1], x[L->s_vel + 2] - 0.0};
  double vw[3] = {x[L->s_vel] - x[L->s_wv], x[L->s_vel + 1] - x[L->s_wv + 1], x[L->s_vel + 2] - 0.0};
  double rb[3], rw[3];
  or_quat_rotate_inv(x + L->s_quat, vb, rb);
  or_quat_rotate_inv(x + L->s_quat, vw, rw);
  for (int i = 0; i < 2; i++) z[i] = m->cw * rb[i] + (1 - m->cw) * rw[i] + x[L->s_badcp + i];
}
static void h_xy(void* c, const double* x, double* z) {
  const or_layout* L = &((meas_ctx*)c)->f->L;
  z[0] = x[L->s_pos];
  z[1] = x[L->s_pos + 1];
}
static void h_z(void* c, const double* x, double* z) {
  const or_layout* L = &((meas_ctx*)c)->f->L;
  z[0] = x[L->s_pos + 2];
}
/* measurementEfforts, PoseUKF.cpp:153-196 (mutates the shared model, :173) */
static void h_efforts(void* c, const double* x, double* z) {
  meas_ctx* m = (meas_ctx*)c;
  const or_layout* L = &m->f->L;
  uwvk_uwv_params* P = m->uwv_mut;
  if (L->has_params)
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) {
        P->inertia_matrix[P_IDX[a] * 6 + P_IDX[b]] = x[L->s_inertia + a + 3 * b];
        P->damping_matrices[0][P_IDX[a] * 6 + P_IDX[b]] = x[L->s_lin + a + 3 * b];
        P->damping_matrices[1][P_IDX[a] * 6 + P_IDX[b]] = x[L->s_quad + a + 3 * b];
      }
  const double* imu = m->f->param.imu_in_body;
  const double* wbd = m->wb;
  double wv[3] = {x[L->s_wv], x[L->s_wv + 1], 0.0};
  double vb[3], cr[3], rw[3], vel6[6], acc6[6], ab[3], cc[3];
  or_quat_rotate_inv(x + L->s_quat, x + L->s_vel, vb);
  cross3(wbd, imu, cr);
  for (int i = 0; i < 3; i++) vb[i] = vb[i] - cr[i];
  or_quat_rotate_inv(x + L->s_quat, wv, rw);
  for (int i = 0; i < 3; i++) vel6[i] = vb[i] - rw[i];
  for (int i = 0; i < 3; i++) vel6[3 + i] = wbd[i];
  or_quat_rotate_inv(x + L->s_quat, x + L->s_acc, ab);
  cross3(wbd, cr, cc);
  for (int i = 0; i < 3; i++) { acc6[i] = ab[i] - cc[i]; acc6[3 + i] = 0.0; }
  or_calc_efforts(P, acc6, vel6, x + L->s_quat, z);
}
/* constrainVelocity, PoseUKF.cpp:199-219 */
static void h_constrain(void* c, const double* x, double* z) {
  meas_ctx* m = (meas_ctx*)c;
  const or_layout* L = &m->f->L;
  const double* imu = m->f->param.imu_in_body;
  double vb[3], cr[3], rw[3], vel6[6], acc6[6];
  or_quat_rotate_inv(m->q, x + L->s_vel, vb);
  cross3(m->wb, imu, cr);
  for (int i = 0; i < 3; i++) vb[i] = vb[i] - cr[i];
  or_quat_rotate_inv(m->q, m->w3, rw);
  for (int i = 0; i < 3; i++) { vel6[i] = vb[i] - rw[i]; vel6[3 + i] = m->wb[i]; }
  for (int i = 0; i < 3; i++) { acc6[i] = m->ab[i]; acc6[3 + i] = 0.0; }
  or_calc_efforts(m->uwv, acc6, vel6, m->q, z);
}

static int check(const double* mu, int m, const double* cov) {
  if (!finite_arr(mu, m) || !finite_arr(cov, m * m)) return UWVK_ENAN;
  return UWVK_OK;
}

static int upd(or_pose* f, int m, const double* z, meas_fn h, meas_ctx* c, const double* R, int zmode, int gate,
               int* acc) {
  manifold M = pose_manifold(f);
  c->f = f;
  return ukf_update(&M, f->mu, f->sigma, m, z, h, c, R, zmode, gate, acc);
}

int or_pose_update_acceleration(or_pose* f, const double mu[3], const double cov[9], int* a) {
  int e = check(mu, 3, cov);
  if (e) return e;
  meas_ctx c;
  return upd(f, 3, mu, h_acc, &c, cov, 1, 0, a);
}
int or_pose_update_velocity(or_pose* f, const double mu[3], const double cov[9], int* a) {
  int e = check(mu, 3, cov);
  if (e) return e;
  meas_ctx c;
  return upd(f, 3, mu, h_vel, &c, cov, 1, 0, a);
}
int or_pose_update_pressure(or_pose* f, const double mu[1], const double cov[1], const double s[3], int* a) {
  int e = check(mu, 1, cov);
  if (e) return e;
  meas_ctx c;
  memcpy(c.v3, s, 3 * sizeof(double));
  return upd(f, 1, mu, h_pressure, &c, cov, 0, 0, a);
}
int or_pose_update_water_velocity(or_pose* f, const double mu[2], const double cov[4], double cw, int* a) {
  int e = check(mu, 2, cov);
  if (e) return e;
  meas_ctx c;
  c.cw = cw;
  return upd(f, 2, mu, h_water, &c, cov, 1, 1, a);
}
int or_pose_update_xy(or_pose* f, const double mu[2], const double cov[4], int* a) {
  int e = check(mu, 2, cov);
  if (e) return e;
  meas_ctx c;
  return upd(f, 2, mu, h_xy, &c, cov, 0, 0, a);
}
int or_pose_update_z(or_pose* f, const double mu[1], const double cov[1], int* a) {
  int e = check(mu, 1, cov);
  if (e) return e;
  meas_ctx c;
  return upd(f, 1, mu, h_z, &c, cov, 0, 0, a);
}
/* PoseUKF.cpp:567-579 */
int or_pose_update_geographic(or_pose* f, const double mu[2], const double cov[4], const double gps[3], int* a) {
  int e = check(mu, 2, cov);
  if (e) return e;
  double z[2], r[3];
  or_world_to_nav(&f->location, mu[0], mu[1], &z[0], &z[1]);
  or_quat_rotate(f->mu + f->L.s_quat, gps, r);
  z[0] = z[0] - r[0];
  z[1] = z[1] - r[1];
  meas_ctx c;
  return upd(f, 2, z, h_xy, &c, cov, 0, 1, a);
}
/* PoseUKF.cpp:514-527 */
int or_pose_update_delayed_xy(or_pose* f, const double mu[2], const double cov[4], const double dp[2], int* a) {
  double z[2];
  for (int i = 0; i < 2; i++) z[i] = mu[i] + (f->mu[f->L.s_pos + i] - dp[i]);
  int e = check(z, 2, cov);
  if (e) return e;
  meas_ctx c;
  return upd(f, 2, z, h_xy, &c, cov, 0, 0, a);
}

/* getRotationRate, PoseUKF.cpp:693-699 */
void or_pose_get_rotation_rate(const or_pose* f, double out[3]) {
  const or_layout* L = &f->L;
  double er[3], r[3];
  earth_rotation(&f->location, f->mu[L->s_pos], f->mu[L->s_pos + 1], er);
  or_quat_rotate_inv(f->mu + L->s_quat, er, r);
  for (int i = 0; i < 3; i++) out[i] = (f->rotation_rate[i] - f->mu[L->s_bg + i]) - r[i];
}

/* PoseUKF.cpp:581-602 */
int or_pose_update_efforts(or_pose* f, const double mu[6], const double cov[36], int only_vel, int* a) {
  int e = check(mu, 6, cov);
  if (e) return e;
  const or_layout* L = &f->L;
  meas_ctx c;
  memset(&c, 0, sizeof(c));
  or_pose_get_rotation_rate(f, c.wb);
  if (only_vel) {
    c.w3[0] = f->mu[L->s_wv]; c.w3[1] = f->mu[L->s_wv + 1]; c.w3[2] = 0.0;
    memcpy(c.q, f->mu + L->s_quat, 4 * sizeof(double));
    double ra[3], cr[3], cc[3];
    or_quat_rotate_inv(c.q, f->mu + L->s_acc, ra);
    cross3(c.wb, f->param.imu_in_body, cr);
    cross3(c.wb, cr, cc);
    for (int i = 0; i < 3; i++) c.ab[i] = ra[i] - cc[i];
    c.uwv = &f->uwv;
    return upd(f, 6, mu, h_constrain, &c, cov, 0, 0, a);
  }
  c.uwv_mut = &f->uwv;
  return upd(f, 6, mu, h_efforts, &c, cov, 0, 0, a);
}

/* PoseUKF.cpp:685-691 */
void or_pose_reset_with_external_pose(or_pose* f, const double pose[7]) {
  memcpy(f->mu + f->L.s_pos, pose, 3 * sizeof(double));
  memcpy(f->mu + f->L.s_quat, pose + 3, 4 * sizeof(double));
}

/* ------------------------------------------------------------------------ */
/* VelocityUKF (VelocityUKF.cpp)                                             */
/* ------------------------------------------------------------------------ */
static const manifold VEL_M = {4, 4, 0, NULL};

void or_vel_init(or_vel* f, const double x[4], const double P[16]) { /* VelocityUKF.cpp:49-56 */
  memset(f, 0, sizeof(*f));
  memcpy(f->mu, x, 4 * sizeof(double));
  memcpy(f->sigma, P, 16 * sizeof(double));
  for (int i = 0; i < 3; i++) f->Q[i * 4 + i] = 0.0001;
}

/* setProcessNoiseCovariance [EXT pose_estimation base] */
void or_vel_set_process_noise(or_vel* f, const double Q[16]) { memcpy(f->Q, Q, 16 * sizeof(double)); }

void or_vel_setup_motion_model(or_vel* f, const uwvk_uwv_params* uwv) { /* VelocityUKF.cpp:58-77 */
  f->uwv = *uwv;
  or_invert(6, uwv->inertia_matrix, f->Minv);
  f->has_model = 1;
  double* s = f->model_state;
  s[0] = s[1] = s[2] = 0.0;
  s[3] = 1.0; s[4] = s[5] = s[6] = 0.0;
  memcpy(s + 7, f->mu, 3 * sizeof(double));
  memcpy(s + 10, f->gyro, 3 * sizeof(double));
}

int or_vel_set_gyro(or_vel* f, const double w[3], const double* cov) { /* VelocityUKF.cpp:87-98 */
  if (!finite_arr(w, 3) || (cov && !finite_arr(cov, 9))) return UWVK_ENAN;
  if (f->has_model) memcpy(f->model_state + 10, w, 3 * sizeof(double));
  memcpy(f->gyro, w, 3 * sizeof(double));
  return UWVK_OK;
}

int or_vel_set_efforts(or_vel* f, const double t[6], const double* cov) {
  if (!finite_arr(t, 6) || (cov && !finite_arr(cov, 36))) return UWVK_ENAN;
  memcpy(f->efforts, t, 6 * sizeof(double));
  return UWVK_OK;
}

typedef struct vel_ctx {
  const or_vel* f;
  double q[4];
  double dt;
} vel_ctx;

/* processMotionModel, VelocityUKF.cpp:6-33 */
static void vel_process(void* c, const double* x, double* o) {
  vel_ctx* v = (vel_ctx*)c;
  double s[13], n[13], r[3], t[4];
  s[0] = s[1] = s[2] = 0.0;
  memcpy(s + 3, v->q, 4 * sizeof(double));
  memcpy(s + 7, x, 3 * sizeof(double));
  memcpy(s + 10, v->f->gyro, 3 * sizeof(double));
  or_model_rk4(&v->f->uwv, v->f->Minv, v->f->efforts, v->dt, s, n);
  for (int i = 0; i < 3; i++) t[i] = x[i] + (n[7 + i] - x[i]);
  or_quat_rotate(v->q, t, r);
  t[3] = x[3] + v->dt * r[2];
  memcpy(o, t, 4 * sizeof(double));
}

int or_vel_predict(or_vel* f, double dt) { /* VelocityUKF.cpp:114-130 */
  if (!f->has_model) return UWVK_ENOMODEL;
  vel_ctx c;
  c.f = f;
  memcpy(c.q, f->model_state + 3, 4 * sizeof(double));
  c.dt = dt;
  double Qp[16];
  for (int i = 0; i < 16; i++) Qp[i] = dt * f->Q[i];
  int e = ukf_predict(&VEL_M, f->mu, f->sigma, vel_process, &c, Qp, NULL);
  double n[13];
  or_model_rk4(&f->uwv, f->Minv, f->efforts, dt, f->model_state, n);
  memcpy(f->model_state, n, sizeof(n));
  return e;
}

static void h_vel_dvl(void* c, const double* x, double* z) { (void)c; memcpy(z, x, 3 * sizeof(double)); }
static void h_vel_z(void* c, const double* x, double* z) { (void)c; z[0] = x[3]; }

int or_vel_update_dvl(or_vel* f, const double mu[3], const double cov[9]) {
  if (!finite_arr(mu, 3) || !finite_arr(cov, 9)) return UWVK_ENAN;
  int a;
  return ukf_update(&VEL_M, f->mu, f->sigma, 3, mu, h_vel_dvl, NULL, cov, 1, 0, &a);
}
int or_vel_update_pressure(or_vel* f, const double mu[1], const double cov[1]) {
  if (!finite_arr(mu, 1) || !finite_arr(cov, 1)) return UWVK_ENAN;
  int a;
  return ukf_update(&VEL_M, f->mu, f->sigma, 1, mu, h_vel_z, NULL, cov, 1, 0, &a);
}

/* ------------------------------------------------------------------------ */
/* batched log runner (threads over independent instances)                   */
/* ------------------------------------------------------------------------ */
typedef struct run_job {
  or_pose* filters;
  const or_pose_run_args* a;
  int64_t first, count, i0, i1;
  uint32_t* accept;
  int err;
} run_job;

static void* run_worker(void* p) {
  run_job* j = (run_job*)p;
  const or_pose_run_args* a = j->a;
  int64_t B = a->batch;
  for (int64_t i = j->i0; i < j->i1; i++) {
    or_pose* f = &j->filters[i];
    uint32_t* ac = j->accept ? j->accept + i * 4 : NULL;
    for (int64_t e = j->first; e < j->first + j->count; e++) {
      int acc, st;
      uint32_t fl = a->flags[e];
      st = or_pose_set_rotation_rate(f, a->gyro + (e * B + i) * 3, NULL);
      if (!st) st = or_pose_predict(f, a->dt);
      if (!st && (fl & UWVK_EV_ACC)) st = or_pose_update_acceleration(f, a->acc + (e * B + i) * 3, a->acc_cov, &acc);
      if (!st && (fl & UWVK_EV_DVL)) {
        st = or_pose_update_velocity(f, a->dvl + ((int64_t)a->dvl_index[e] * B + i) * 3, a->dvl_cov, &acc);
        if (ac) ac[0] += acc;
      }
      if (!st && (fl & UWVK_EV_PRESSURE)) {
        st = or_pose_update_pressure(f, a->pressure + (int64_t)a->pressure_index[e] * B + i, &a->pressure_cov,
                                     a->pressure_sensor_in_imu, &acc);
        if (ac) ac[1] += acc;
      }
      if (!st && (fl & UWVK_EV_ADCP))
        for (int c = 0; c < a->adcp_cells && !st; c++) {
          const double* z = a->adcp + (((int64_t)a->adcp_index[e] * a->adcp_cells + c) * B + i) * 2;
          st = or_pose_update_water_velocity(f, z, a->adcp_cov, a->adcp_cell_weighting[c], &acc);
          if (ac) ac[2] += acc;
        }
      if (!st && (fl & UWVK_EV_EFFORTS)) {
        st = or_pose_update_efforts(f, a->efforts + ((int64_t)a->efforts_index[e] * B + i) * 6, a->efforts_cov,
                                    (fl & UWVK_EV_EFFORTS_VELOCITY_ONLY) ? 1 : 0, &acc);
        if (ac) ac[3] += acc;
      }
      if (st) { j->err = st; return NULL; }
    }
  }
  return NULL;
}

int or_pose_run_log(or_pose* filters, const or_pose_run_args* a, int64_t first, int64_t count, int nthreads,
                    uint32_t* accept) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > a->batch) nthreads = (int)a->batch;
  run_job* jobs = (run_job*)calloc((size_t)nthreads, sizeof(run_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].filters = filters; jobs[t].a = a; jobs[t].first = first; jobs[t].count = count; jobs[t].accept = accept;
    jobs[t].i0 = a->batch * t / nthreads;
    jobs[t].i1 = a->batch * (t + 1) / nthreads;
    if (nthreads == 1) run_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, run_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    if (jobs[t].err && !err) err = jobs[t].err;
  }
  free(jobs);
  free(th);
  return err;
}

typedef struct vel_job {
  or_vel* filters;
  const or_vel_run_args* a;
  int64_t first, count, i0, i1;
  int err;
} vel_job;

/* the epoch order of the reference's users (VelocityUKF.cpp:79-130) */
static void* vel_worker(void* p) {
  vel_job* j = (vel_job*)p;
  const or_vel_run_args* a = j->a;
  const int64_t B = a->batch;
  for (int64_t i = j->i0; i < j->i1 && !j->err; i++) {
    or_vel* f = &j->filters[i];
    for (int64_t e = j->first; e < j->first + j->count; e++) {
      int r = or_vel_set_gyro(f, a->gyro + (e * B + i) * 3, NULL);
      if (!r) r = or_vel_set_efforts(f, a->efforts + (e * B + i) * 6, NULL);
      if (!r) r = or_vel_predict(f, a->dt);
      if (!r && (a->flags[e] & UWVK_EV_DVL))
        r = or_vel_update_dvl(f, a->dvl + ((int64_t)a->dvl_index[e] * B + i) * 3, a->dvl_cov);
      if (!r && (a->flags[e] & UWVK_EV_PRESSURE)) {
        const double pc[1] = {a->pressure_cov};
        r = or_vel_update_pressure(f, a->pressure + (int64_t)a->pressure_index[e] * B + i, pc);
      }
      if (r) {
        j->err = r;
        break;
      }
    }
  }
  return NULL;
}

int or_vel_run_log(or_vel* filters, const or_vel_run_args* a, int64_t first, int64_t count, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > a->batch) nthreads = (int)a->batch;
  vel_job* jobs = (vel_job*)calloc((size_t)nthreads, sizeof(vel_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    jobs[t].filters = filters; jobs[t].a = a; jobs[t].first = first; jobs[t].count = count;
    jobs[t].i0 = a->batch * t / nthreads;
    jobs[t].i1 = a->batch * (t + 1) / nthreads;
    if (nthreads == 1) vel_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, vel_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(th[t], NULL);
    if (jobs[t].err && !err) err = jobs[t].err;
  }
  free(jobs);
  free(th);
  return err;
}

size_t or_pose_sizeof(void) { return sizeof(or_pose); }
size_t or_vel_sizeof(void) { return sizeof(or_vel); }

void or_pose_get_state(const or_pose* f, double* x, double* P) {
  memcpy(x, f->mu, sizeof(double) * f->L.store);
  if (P) memcpy(P, f->sigma, sizeof(double) * f->L.dof * f->L.dof);
}
void or_vel_get_state(const or_vel* f, double* x, double* P, double* ms) {
  memcpy(x, f->mu, 4 * sizeof(double));
  if (P) memcpy(P, f->sigma, 16 * sizeof(double));
  if (ms) memcpy(ms, f->model_state, 13 * sizeof(double));
}
