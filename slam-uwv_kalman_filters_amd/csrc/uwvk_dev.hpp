// uwvk_dev.hpp — device-side building blocks of the batched UKF engine (gfx950).
//
// Everything here runs inside ONE wavefront (64 lanes) that owns ONE filter
// instance (PoseUKF) — the north-star "one filter per wavefront" layout — or,
// for the 4-DOF VelocityUKF, inside one lane.  fp64 throughout (SURVEY.md K8:
// the covariance spans 1e-10..1e2, Cholesky needs fp64).
//
// Conventions shared with the CPU oracle (oracle/uwvk_oracle.c) and the frozen
// [EXT] spec:
//   quaternion (w,x,y,z); SO3 boxplus is nav-frame (left): q <- exp(d) * q;
//   boxminus a [-] b = log(a * conj(b)); vect boxplus x + s*d.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define UWVK_DEV __device__ __forceinline__

namespace uwvk {

// Host side: every C-ABI entry point that takes a handle makes the handle's
// device current for the duration of the call (allocations, launches, copies)
// and restores the caller's device on return, so one thread may drive handles
// on several GPUs.  device < 0 (a null handle): no-op.
// clears the calling thread's uwvk_last_device_error text (uwvk_rt.hip): every
// public entry point starts with a DeviceGuard, so the text always belongs to
// the current call's UWVK_EDEVICE, never an earlier, unrelated failure
void clear_hip_error();
void note_hip_error(int err, const char* where);
// UWVK_EDEVICE with the text of the first failing HIP call (uwvk_last_device_error)
inline int edevice_status(hipError_t e, const char* where) {
  note_hip_error((int)e, where);
  return 5;  // UWVK_EDEVICE (include/uwvk.h; static_assert in uwvk_rt.hip)
}
// a launch's error, else its stream synchronisation's; 0 when both succeeded
inline int launch_sync_status(hipError_t launch, hipStream_t st, const char* where) {
  const hipError_t s = hipStreamSynchronize(st);
  if (launch != hipSuccess) return edevice_status(launch, where);
  if (s != hipSuccess) return edevice_status(s, where);
  return 0;
}
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int device) {
    clear_hip_error();
    int cur = -1;
    if (device < 0 || hipGetDevice(&cur) != hipSuccess || cur == device) return;
    if (hipSetDevice(device) == hipSuccess) prev = cur;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define UWVK_DEVICE_GUARD(h) ::uwvk::DeviceGuard uwvk_device_guard_((h) ? (h)->device : -1)

constexpr double kEarthW = 7.292115e-5;  // pose_estimation::EARTHW [EXT] (PoseUKF.cpp:30)
constexpr double kD2P95 = 5.991;         // PoseUKF.cpp:275-286

// ---------------------------------------------------------------------------
// PoseState layout (PoseState.hpp:29-45) as a compile-time descriptor.
// DOF = 53: full state; DOF = 26: kinematic subset (no model-parameter blocks).
// ---------------------------------------------------------------------------
template <int DOF>
struct Lay;

template <>
struct Lay<53> {
  static constexpr int dof = 53, store = 54, has_params = 1;
  static constexpr int s_pos = 0, s_quat = 3, s_vel = 7, s_acc = 10, s_bg = 13, s_ba = 16, s_grav = 19,
                       s_inertia = 20, s_lin = 29, s_quad = 38, s_wv = 47, s_wvb = 49, s_badcp = 51, s_rho = 53;
  static constexpr int d_pos = 0, d_ori = 3, d_vel = 6, d_acc = 9, d_bg = 12, d_ba = 15, d_grav = 18,
                       d_inertia = 19, d_lin = 28, d_quad = 37, d_wv = 46, d_wvb = 48, d_badcp = 50, d_rho = 52;
};
template <>
struct Lay<26> {
  static constexpr int dof = 26, store = 27, has_params = 0;
  static constexpr int s_pos = 0, s_quat = 3, s_vel = 7, s_acc = 10, s_bg = 13, s_ba = 16, s_grav = 19,
                       s_inertia = -1, s_lin = -1, s_quad = -1, s_wv = 20, s_wvb = 22, s_badcp = 24, s_rho = 26;
  static constexpr int d_pos = 0, d_ori = 3, d_vel = 6, d_acc = 9, d_bg = 12, d_ba = 15, d_grav = 18,
                       d_inertia = -1, d_lin = -1, d_quad = -1, d_wv = 19, d_wvb = 21, d_badcp = 23, d_rho = 25;
};

// tangent index -> storage index for non-orientation DOFs
UWVK_DEV constexpr int d2s(int d) { return d < 3 ? d : d + 1; }

// ---------------------------------------------------------------------------
// small vector / quaternion algebra (Eigen conventions, see oracle)
// ---------------------------------------------------------------------------
UWVK_DEV void cross3(const double a[3], const double b[3], double o[3]) {
  double x = a[1] * b[2] - a[2] * b[1];
  double y = a[2] * b[0] - a[0] * b[2];
  double z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}

UWVK_DEV void qmul(const double a[4], const double b[4], double o[4]) {
  double w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  double x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  double y = a[0] * b[2] + a[2] * b[0] + a[3] * b[1] - a[1] * b[3];
  double z = a[0] * b[3] + a[3] * b[0] + a[1] * b[2] - a[2] * b[1];
  o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}

// Eigen _transformVector: uv = 2 (q.vec x v); v + w uv + q.vec x uv
UWVK_DEV void qrot(const double q[4], const double v[3], double o[3]) {
  double uv[3], t[3];
  cross3(q + 1, v, uv);
  uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
  cross3(q + 1, uv, t);
#pragma unroll
  for (int i = 0; i < 3; i++) o[i] = v[i] + q[0] * uv[i] + t[i];
}
UWVK_DEV void qrot_inv(const double q[4], const double v[3], double o[3]) {
  double c[4] = {q[0], -q[1], -q[2], -q[3]};
  qrot(c, v, o);
}
UWVK_DEV void qmatrix(const double q[4], double R[9]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  double twx = tx * w, twy = ty * w, twz = tz * w;
  double txx = tx * x, txy = ty * x, txz = tz * x;
  double tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1 - (txx + tyy);
}

// SO3 exp of an already-scaled rotation vector [EXT MTK]
UWVK_DEV void so3_exp(const double v[3], double o[4]) {
  double t = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (t == 0.0) { o[0] = 1; o[1] = o[2] = o[3] = 0; return; }
  double s, c;
  sincos(0.5 * t, &s, &c);
  s = s / t;
  o[0] = c; o[1] = s * v[0]; o[2] = s * v[1]; o[3] = s * v[2];
}
// SO3 log, shortest rotation (|theta| <= pi) [EXT MTK]
UWVK_DEV void so3_log(const double q[4], double o[3]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  if (w < 0) { w = -w; x = -x; y = -y; z = -z; }
  double nv = sqrt(x * x + y * y + z * z);
  if (nv == 0.0) { o[0] = o[1] = o[2] = 0; return; }
  double k = 2.0 * atan2(nv, w) / nv;
  o[0] = k * x; o[1] = k * y; o[2] = k * z;
}
// log(a * conj(b))
UWVK_DEV void qboxminus(const double a[4], const double b[4], double o[3]) {
  double bc[4] = {b[0], -b[1], -b[2], -b[3]}, r[4];
  qmul(a, bc, r);
  so3_log(r, o);
}

// SO3 [+] / [-] of either side [EXT MTK] (SURVEY 8(c) item
// 5): right = 0 is the nav-frame (left) convention, q [+] d = exp(d) q and
// a [-] b = log(a b^-1), the default everywhere; right = 1 the body-frame
// (classic MTK SO3::boxplus) one, q [+] d = q exp(d) and a [-] b = log(b^-1 a).
// The literal kernels take the side from the handle (UWVK_OPT_SO3_RIGHT); the
// PSP kernels are left-only.  e = exp(d) is passed in; the branch is uniform.
// One product with the operand order selected (no duplicated code paths: the
// literal kernels are at the VGPR limit): q1 q2 = (w1 w2 - v1.v2, w1 v2 + w2 v1
// + v1 x v2), so swapping the operands only flips the sign of the cross term.
UWVK_DEV void qmul_side(const double a[4], const double b[4], double o[4], int swap) {
  const double sg = swap ? -1.0 : 1.0;
  const double cx = a[2] * b[3] - a[3] * b[2], cy = a[3] * b[1] - a[1] * b[3], cz = a[1] * b[2] - a[2] * b[1];
  o[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  o[1] = a[0] * b[1] + a[1] * b[0] + sg * cx;
  o[2] = a[0] * b[2] + a[2] * b[0] + sg * cy;
  o[3] = a[0] * b[3] + a[3] * b[0] + sg * cz;
}
UWVK_DEV void qplus_side(const double e[4], const double q[4], double o[4], int right) {
  if (!right) {  // the default keeps qmul's exact expressions (bitwise the r02 results)
    qmul(e, q, o);
    return;
  }
  qmul_side(e, q, o, 1);  // q e
}
UWVK_DEV void qboxminus_side(const double a[4], const double b[4], double o[3], int right) {
  double bc[4] = {b[0], -b[1], -b[2], -b[3]}, r[4];
  if (!right) {
    qmul(a, bc, r);
  } else {
    qmul_side(a, bc, r, 1);  // b^-1 a
  }
  so3_log(r, o);
}

// ---------------------------------------------------------------------------
// wave-level primitives
// ---------------------------------------------------------------------------
UWVK_DEV int lane_id() { return threadIdx.x & 63; }

// filter instance of this workgroup (one workgroup per instance).  Workgroups
// are dealt round-robin to the 8 XCDs (workgroup w runs on XCD w % 8), so XCD
// x is given the contiguous instances [x n, (x+1) n): neighbouring instances'
// per-epoch input rows (24 B, five to a 128-B line) then meet in one L2
// instead of being fetched once per XCD.  The tail past 8n maps to itself.
UWVK_DEV int64_t xcd_instance(int64_t batch) {
  const int64_t w = blockIdx.x, n = batch >> 3;
  return w < (n << 3) ? (w & 7) * n + (w >> 3) : w;
}

// Packed lower triangle (row i at i (i + 1) / 2): Sigma's layout in HBM
// ([batch][dof (dof + 1) / 2], every kernel) and in the PSP kernels' LDS.
UWVK_DEV constexpr int pidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }
template <int DOF>
constexpr int tri_n() { return DOF * (DOF + 1) / 2; }

// flat packed index e -> (i, j), i >= j
UWVK_DEV void unpack(int e, int& i, int& j) {
  int r = (int)((__builtin_sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if ((r + 1) * (r + 2) / 2 <= e) r++;
  if (r * (r + 1) / 2 > e) r--;
  i = r;
  j = e - r * (r + 1) / 2;
}

UWVK_DEV double shfl_d(double v, int src) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __shfl(lo, src, 64);
  hi = __shfl(hi, src, 64);
  return __hiloint2double(hi, lo);
}
UWVK_DEV double readlane_d(double v, int lane) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
UWVK_DEV double shfl_xor_d(double v, int m) {
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __shfl_xor(lo, m, 64);
  hi = __shfl_xor(hi, m, 64);
  return __hiloint2double(hi, lo);
}
// butterfly sum over the 64 lanes, result in every lane
UWVK_DEV double wave_sum(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += shfl_xor_d(v, m);
  return v;
}

// accumulator type of v_mfma_f64_16x16x4_f64 (4 results per lane; C/D map
// col = lane & 15, row = (lane >> 4) + 4 * reg — verified on gfx950 by
// tools/probe_fp64.hip, profiles/r01_probe_fp64.txt)
typedef double d4_t __attribute__((ext_vector_type(4)));

UWVK_DEV d4_t mfma_f64(double a, double b, d4_t c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }

// ---------------------------------------------------------------------------
// Diagnostic phase stamps (build with -DUWVK_STAMPS; never in the product .so).
// Thread 0 of every 64th workgroup adds the s_memtime delta since its previous
// stamp to a per-phase sum (sampling keeps the atomics from serialising the
// kernel); read back with uwvk_debug_read_stamps().
// ---------------------------------------------------------------------------
#ifdef UWVK_STAMPS
static __device__ unsigned long long uwvk_stamp_sum[64];  // per translation unit
static __device__ unsigned long long uwvk_stamp_cnt[64];
UWVK_DEV unsigned long long stamp_now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
struct Stamper {
  unsigned long long last;
  UWVK_DEV Stamper() : last(stamp_now()) {}
  UWVK_DEV void mark(int ph) {
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = stamp_now();
    __builtin_amdgcn_sched_barrier(0);
    if (threadIdx.x == 0 && (blockIdx.x & 63) == 0) {
      atomicAdd(&uwvk_stamp_sum[ph], t - last);
      atomicAdd(&uwvk_stamp_cnt[ph], 1ull);
    }
    last = t;
  }
};
#else
struct Stamper {
  UWVK_DEV void mark(int) {}
};
#endif
#define UWVK_STAMP(ph) \
  do {                 \
    if (st) st->mark(ph); \
  } while (0)

}  // namespace uwvk
