// uwvk_small.hip — BottomUKF (src/BottomUKF.hpp:26-53) and IndirectPoseUKF
// (src/IndirectPoseUKF.hpp:28-86) on gfx950, batched, and their uwvk_bottom_* /
// uwvk_ipose_* C ABI.
//
// Both are small-state filters: one instance per lane group, one sigma point
// per lane (uwvk_aug_dev.hpp): BottomUKF 8 lanes (8 instances per wave),
// IndirectPoseUKF 16 lanes (4 per wave), its marker-augmented visual update
// 32 lanes (2 per wave).  Sigma lives in LDS for the duration of a call.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <vector>

#include "uwvk_aug_dev.hpp"
#include "../../include/uwvk.h"
#include "uwvk_host.hpp"

using namespace uwvk;
using namespace uwvk::aug;

namespace {

using BottomM = Manifold<Seg<SEG_V, 1>, Seg<SEG_S2>>;                        // BottomUKF.hpp:18-21
// IndirectPoseUKF's orientation_error is an MTK::SO3 like PoseUKF's orientation:
// SR = 1 the body-frame [+] q exp(d) (MTK's SO3::boxplus, the default), 0 nav-frame
template <int SR>
using SO3Seg = Seg<SR ? SEG_SO3R : SEG_SO3>;
template <int SR>
using IPoseM = Manifold<Seg<SEG_V, 3>, SO3Seg<SR>>;                          // IndirectPoseUKF.hpp:19-22
template <int SR>
using IPoseMarkerM = Manifold<Seg<SEG_V, 3>, SO3Seg<SR>, Seg<SEG_V, 3>, SO3Seg<SR>>;  // IndirectPoseUKF.cpp:25-29
using BE = Engine<BottomM>;
template <int SR>
using IE = Engine<IPoseM<SR>>;
template <int SR>
using IAE = Engine<IPoseMarkerM<SR>>;

struct SmallBufs {
  int64_t batch;
  double* mu;        // [batch][store]
  double* sigma;     // [batch][n*n]
  uint32_t* status;  // [batch]
};

struct M9 { double v[9]; };
struct M36 { double v[36]; };

// load / store one instance's (mu, Sigma) between HBM and its LDS words
template <class E>
__device__ void load(E& e, const SmallBufs& b, int64_t inst) {
  if (e.live) {
    for (int i = e.g; i < E::n * E::n; i += E::G) e.sm[E::o_sig + i] = b.sigma[inst * E::n * E::n + i];
    for (int k = e.g; k < E::S; k += E::G) e.sm[E::o_mu + k] = b.mu[inst * E::S + k];
  }
  __syncthreads();
}
template <class E>
__device__ void store(E& e, const SmallBufs& b, int64_t inst, bool ok) {
  if (e.live && ok) {
    for (int i = e.g; i < E::n * E::n; i += E::G) b.sigma[inst * E::n * E::n + i] = e.sm[E::o_sig + i];
    for (int k = e.g; k < E::S; k += E::G) b.mu[inst * E::S + k] = e.sm[E::o_mu + k];
  }
  if (e.live && !ok && e.g == 0) b.status[inst] |= UWVK_ST_NOTPD;
}

template <class E>
__device__ E make_engine(double* smem, const SmallBufs& b, const uint8_t* mask, int64_t* inst) {
  const int gi = threadIdx.x / E::G;
  E e;
  e.g = threadIdx.x % E::G;
  e.sm = smem + gi * E::words;
  *inst = (int64_t)blockIdx.x * E::IPB + gi;
  e.live = *inst < b.batch && (!mask || mask[*inst]);
  return e;
}

// ---- BottomUKF -----------------------------------------------------------
// predictionStepImpl (BottomUKF.cpp:48-54) + processModel (:5-16)
__global__ __launch_bounds__(BE::BLOCK) void k_bottom_predict(SmallBufs b, const double* vel, M9 Q, double dt) {
  __shared__ double smem[BE::IPB * BE::words];
  int64_t inst;
  BE e = make_engine<BE>(smem, b, nullptr, &inst);
  load(e, b, inst);
  double vz = 0.0, s = 0.0;
  if (e.live) {
    const double vx = vel[inst * 3], vy = vel[inst * 3 + 1];
    vz = vel[inst * 3 + 2];
    const double nrm = sqrt(vx * vx + vy * vy);
    s = (nrm * nrm) * (dt * dt);  // pow(|v_xy|, 2) * pow(dt, 2)
  }
  const bool ok = e.predict([&](double* x) { x[0] = x[0] + (-1.0 * vz) * dt; },
                            [&](int r, int c) { return s * Q.v[r * 3 + c]; });
  store(e, b, inst, ok);
}

// measurementDistance (BottomUKF.cpp:18-30)
struct RangeH {
  double dir[3], origin[3];
  UWVK_DEV void operator()(const double* x, double* z) const {
    const double bottom[3] = {0.0, 0.0, -x[0]};
    const double v = dir[0] * x[1] + dir[1] * x[2] + dir[2] * x[3];
    if (v != 0.0)
      z[0] = ((bottom[0] - origin[0]) * x[1] + (bottom[1] - origin[1]) * x[2] + (bottom[2] - origin[2]) * x[3]) / v;
    else
      z[0] = 0.0;
  }
};

// integrateMeasurement(RangeMeasurement, unit_direction, origin) (BottomUKF.cpp:56-61):
// DistanceType (mtkwrap<Scalar>) measurement -> iterative vect mean
__global__ __launch_bounds__(BE::BLOCK) void k_bottom_range(SmallBufs b, const double* z, const double* cov,
                                                            double shared_cov, RangeH h, const uint8_t* mask) {
  __shared__ double smem[BE::IPB * BE::words];
  int64_t inst;
  BE e = make_engine<BE>(smem, b, mask, &inst);
  load(e, b, inst);
  double zz[3] = {0.0, 0.0, 0.0}, R[1] = {1.0};
  if (e.live) {
    zz[0] = z[inst];
    R[0] = cov ? cov[inst] : shared_cov;
  }
  const bool ok = e.template update<Z_VECT, 1>(zz, R, h);
  store(e, b, inst, ok);
}

// measurementNormal (BottomUKF.cpp:32-37)
struct NormalH {
  UWVK_DEV void operator()(const double* x, double* z) const { z[0] = x[1]; z[1] = x[2]; z[2] = x[3]; }
};

// integrateMeasurement(NormalType, cov) (BottomUKF.cpp:63-67): S2 measurement
__global__ __launch_bounds__(BE::BLOCK) void k_bottom_normal(SmallBufs b, const double* z, const double* cov,
                                                             M9 shared_cov, const uint8_t* mask) {
  __shared__ double smem[BE::IPB * BE::words];
  int64_t inst;
  BE e = make_engine<BE>(smem, b, mask, &inst);
  load(e, b, inst);
  double zz[3] = {0.0, 0.0, 1.0}, R[4] = {1.0, 0.0, 0.0, 1.0};
  if (e.live) {
    s2_from(z + inst * 3, zz);
#pragma unroll
    for (int k = 0; k < 4; k++) R[k] = cov ? cov[inst * 4 + k] : shared_cov.v[k];
  }
  const bool ok = e.template update<Z_S2, 2>(zz, R, NormalH{});
  store(e, b, inst, ok);
}

// ---- IndirectPoseUKF -------------------------------------------------------
// predictionStepImpl (IndirectPoseUKF.cpp:80-92) + processModel (:7-20)
template <int SR>
__global__ __launch_bounds__(IE<SR>::BLOCK) void k_ipose_predict(SmallBufs b, M36 Q, double tau, double dt) {
  using E = IE<SR>;
  __shared__ double smem[E::IPB * E::words];
  int64_t inst;
  E e = make_engine<E>(smem, b, nullptr, &inst);
  load(e, b, inst);
  // Q' = dt^2 (Q with the orientation block R (2/(tau dt) Q_o) R^T), R = mu's rotation
  double Rm[9];
  {
    const double q[4] = {e.sm[E::o_mu + 3], e.sm[E::o_mu + 4], e.sm[E::o_mu + 5], e.sm[E::o_mu + 6]};
    qmatrix(q, Rm);
  }
  const double s = 2.0 / (tau * dt), dt2 = dt * dt;
  auto qf = [&](int r, int c) {
    if (r < 3 || c < 3) return dt2 * Q.v[r * 6 + c];
    const int i = r - 3, j = c - 3;
    double A[3];
#pragma unroll
    for (int l = 0; l < 3; l++) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < 3; k++) t += Rm[i * 3 + k] * (s * Q.v[(k + 3) * 6 + l + 3]);
      A[l] = t;
    }
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) t += A[k] * Rm[j * 3 + k];
    return dt2 * t;
  };
  const double ntau = -1.0 / tau;
  const bool ok = e.predict(
      [&](double* x) {
        double l[3], d[3], ex[4], r[4];
        so3_log(x + 3, l);
#pragma unroll
        for (int k = 0; k < 3; k++) d[k] = ntau * l[k] * dt;
        so3_exp(d, ex);
        // orientation_error.boxplus(d, dt) (:17); d is a multiple of log(q), so
        // exp(d) commutes with q and both sides give the same product
        if constexpr (SR) qmul(x + 3, ex, r);
        else qmul(ex, x + 3, r);
#pragma unroll
        for (int k = 0; k < 4; k++) x[3 + k] = r[k];
      },
      qf);
  store(e, b, inst, ok);
}

// integrateMeasurement(marker features, ...) (IndirectPoseUKF.cpp:94-135):
// augment with the marker pose, one S2 update per feature, keep the filter block
template <int SR>
__global__ __launch_bounds__(IAE<SR>::BLOCK) void k_ipose_visual(SmallBufs b, VisArgs va) {
  using E = IAE<SR>;
  __shared__ double smem[E::IPB * E::words];
  int64_t inst;
  E e = make_engine<E>(smem, b, va.mask, &inst);
  if (e.live) {
    for (int i = e.g; i < 144; i += E::G) {
      const int r = i / 12, c = i % 12;
      double v = 0.0;
      if (r < 6 && c < 6) v = b.sigma[inst * 36 + r * 6 + c];
      else if (r >= 6 && c >= 6) v = va.cov_marker[(r - 6) * 6 + (c - 6)];
      e.sm[E::o_sig + i] = v;
    }
    for (int k = e.g; k < 14; k += E::G)
      e.sm[E::o_mu + k] = k < 7 ? b.mu[inst * 7 + k] : va.marker[inst * va.marker_stride + (k - 7)];
  }
  __syncthreads();
  const bool ok = visual_loop<E, 7, true>(e, va, inst);
  if (e.live && ok) {
    for (int i = e.g; i < 36; i += E::G) b.sigma[inst * 36 + i] = e.sm[E::o_sig + (i / 6) * 12 + (i % 6)];
    for (int k = e.g; k < 7; k += E::G) b.mu[inst * 7 + k] = e.sm[E::o_mu + k];
  }
  if (e.live && !ok && e.g == 0) b.status[inst] |= UWVK_ST_NOTPD;
}

int64_t grid_of(int64_t batch, int ipb) { return (batch + ipb - 1) / ipb; }

bool finite_all(const double* a, size_t n) {
  for (size_t k = 0; k < n; k++)
    if (!std::isfinite(a[k])) return false;
  return true;
}

}  // namespace

#define HIPCHK(x)                                  \
  do {                                             \
    const hipError_t e_ = (x);                     \
    if (e_ != hipSuccess) {                        \
      ::uwvk::note_hip_error((int)e_, __func__);   \
      return UWVK_EDEVICE;                         \
    }                                              \
  } while (0)

// ===========================================================================
// host handles
// ===========================================================================
struct SmallHandle {
  int64_t batch = 0;
  int device = 0, n = 0, store = 0;
  hipStream_t stream = nullptr;
  double *d_mu = nullptr, *d_sigma = nullptr, *d_aux = nullptr, *d_meas = nullptr;
  uint32_t* d_status = nullptr;
  uint8_t* d_mask = nullptr;
  size_t meas_words = 0;
  VisStage vis;  // visual-update staging (IndirectPoseUKF)
  bool has_state = false;
  SmallBufs bufs() const { return SmallBufs{batch, d_mu, d_sigma, d_status}; }
};

struct uwvk_bottom : SmallHandle {
  M9 Q{};
};
struct uwvk_ipose : SmallHandle {
  M36 Q{};
  double tau = 1.0;
  int so3_right = 1;  // UWVK_OPT_SO3_RIGHT (uwvk_ipose_set_option), default body frame
};

static void small_destroy(SmallHandle* h) {
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : {(void*)h->d_mu, (void*)h->d_sigma, (void*)h->d_aux, (void*)h->d_meas, (void*)h->d_status,
                  (void*)h->d_mask})
    if (p) (void)hipFree(p);
  h->vis.release();
  if (h->stream) (void)hipStreamDestroy(h->stream);
}

// aux: BottomUKF velocity [batch][3]; IndirectPoseUKF pose_ref [batch][7]
static uwvk_status small_create(SmallHandle* h, int64_t batch, int device, int n, int store, int aux_w,
                                size_t meas_words) {
  h->batch = batch;
  h->device = device;
  h->n = n;
  h->store = store;
  h->meas_words = meas_words;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return UWVK_EDEVICE;
  const size_t B = (size_t)batch;
  const bool ok = hipMalloc(&h->d_mu, B * store * 8) == hipSuccess &&
                  hipMalloc(&h->d_sigma, B * n * n * 8) == hipSuccess &&
                  hipMalloc(&h->d_aux, B * aux_w * 8) == hipSuccess &&
                  hipMalloc(&h->d_meas, meas_words * 8) == hipSuccess && hipMalloc(&h->d_mask, B) == hipSuccess &&
                  hipMalloc(&h->d_status, B * 4) == hipSuccess;
  if (!ok) return UWVK_ENOMEM;
  (void)hipMemsetAsync(h->d_aux, 0, B * aux_w * 8, h->stream);
  (void)hipMemsetAsync(h->d_status, 0, B * 4, h->stream);
  return hipStreamSynchronize(h->stream) == hipSuccess ? UWVK_OK : UWVK_EDEVICE;
}

static uwvk_status small_get_state(SmallHandle* h, double* x, double* P) {
  if (!h || !x) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(x, h->d_mu, (size_t)h->batch * h->store * 8, hipMemcpyDeviceToHost, h->stream));
  if (P) HIPCHK(hipMemcpyAsync(P, h->d_sigma, (size_t)h->batch * h->n * h->n * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

static uwvk_status small_get_status(SmallHandle* h, uint32_t* st, int clear) {
  if (!h || !st) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(st, h->d_status, (size_t)h->batch * 4, hipMemcpyDeviceToHost, h->stream));
  if (clear) HIPCHK(hipMemsetAsync(h->d_status, 0, (size_t)h->batch * 4, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

static uwvk_status upload_mask(SmallHandle* h, const uint8_t* mask, const uint8_t** dmask) {
  *dmask = nullptr;
  if (mask) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)h->batch, hipMemcpyHostToDevice, h->stream));
    *dmask = h->d_mask;
  }
  return UWVK_OK;
}

extern "C" {

// ---- BottomUKF -----------------------------------------------------------
uwvk_status uwvk_bottom_create(int64_t batch, int device, uwvk_bottom** out) {
  ::uwvk::DeviceGuard uwvk_device_guard_(device);
  if (!out || batch <= 0) return UWVK_EINVAL;
  *out = nullptr;
  if (!uwvk_device_available(device)) return UWVK_EDEVICE;
  uwvk_bottom* h = new uwvk_bottom();
  const uwvk_status st = small_create(h, batch, device, 3, 4, 3, (size_t)batch * 8 + 16);
  if (st != UWVK_OK) {
    small_destroy(h);
    delete h;
    return st;
  }
  for (int k = 0; k < 3; k++) h->Q.v[k * 3 + k] = 1.0;  // Covariance::Identity() (BottomUKF.cpp:45)
  *out = h;
  return UWVK_OK;
}

void uwvk_bottom_destroy(uwvk_bottom* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return;
  small_destroy(h);
  delete h;
}

void* uwvk_bottom_stream(const uwvk_bottom* h) { return h ? (void*)h->stream : nullptr; }

uwvk_status uwvk_bottom_init(uwvk_bottom* h, const double* x, const double* P) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !x || !P) return UWVK_EINVAL;
  const int64_t B = h->batch;
  if (!finite_all(x, (size_t)B * 4) || !finite_all(P, (size_t)B * 9)) return UWVK_ENAN;
  std::vector<double> xs((size_t)B * 4);
  for (int64_t i = 0; i < B; i++) {  // MTK::S2 constructor normalises the normal
    const double* v = x + i * 4;
    const double nn = std::sqrt(v[1] * v[1] + v[2] * v[2] + v[3] * v[3]);
    if (!(nn > 0.0)) return UWVK_EINVAL;
    xs[i * 4] = v[0];
    for (int k = 1; k < 4; k++) xs[i * 4 + k] = v[k] / nn;
  }
  HIPCHK(hipMemcpyAsync(h->d_mu, xs.data(), xs.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_sigma, P, (size_t)B * 9 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return UWVK_OK;
}

uwvk_status uwvk_bottom_set_process_noise(uwvk_bottom* h, const double Q[9]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !Q) return UWVK_EINVAL;
  if (!finite_all(Q, 9)) return UWVK_ENAN;
  std::memcpy(h->Q.v, Q, sizeof(h->Q.v));
  return UWVK_OK;
}

uwvk_status uwvk_bottom_set_velocity(uwvk_bottom* h, const double* v) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !v) return UWVK_EINVAL;
  if (!finite_all(v, (size_t)h->batch * 3)) return UWVK_ENAN;
  HIPCHK(hipMemcpyAsync(h->d_aux, v, (size_t)h->batch * 3 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_bottom_predict(uwvk_bottom* h, double dt) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  hipLaunchKernelGGL(k_bottom_predict, dim3(grid_of(h->batch, BE::IPB)), dim3(BE::BLOCK), 0, h->stream, h->bufs(),
                     h->d_aux, h->Q, dt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_bottom_update_range(uwvk_bottom* h, const double* mu, const double* cov, double shared_cov,
                                     const double unit_direction[3], const double origin[3], const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !mu || !unit_direction || !origin) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  const int64_t B = h->batch;
  for (int64_t i = 0; i < B; i++) {  // checkMeasurment (BottomUKF.cpp:58)
    if (mask && !mask[i]) continue;
    if (!std::isfinite(mu[i]) || (cov && !std::isfinite(cov[i]))) return UWVK_ENAN;
  }
  if (!cov && !std::isfinite(shared_cov)) return UWVK_ENAN;
  double* dz = h->d_meas;
  double* dc = h->d_meas + B;
  HIPCHK(hipMemcpyAsync(dz, mu, (size_t)B * 8, hipMemcpyHostToDevice, h->stream));
  if (cov) HIPCHK(hipMemcpyAsync(dc, cov, (size_t)B * 8, hipMemcpyHostToDevice, h->stream));
  const uint8_t* dm;
  if (upload_mask(h, mask, &dm) != UWVK_OK) return UWVK_EDEVICE;
  RangeH rh;
  for (int k = 0; k < 3; k++) {
    rh.dir[k] = unit_direction[k];
    rh.origin[k] = origin[k];
  }
  hipLaunchKernelGGL(k_bottom_range, dim3(grid_of(B, BE::IPB)), dim3(BE::BLOCK), 0, h->stream, h->bufs(), dz,
                     cov ? dc : nullptr, shared_cov, rh, dm);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_bottom_update_normal(uwvk_bottom* h, const double* mu, const double* cov, const double* shared_cov,
                                      const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !mu || (!cov && !shared_cov)) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  const int64_t B = h->batch;
  // the reference does not check this measurement (BottomUKF.cpp:63-67); a
  // zero / non-finite normal cannot be normalised into S2
  for (int64_t i = 0; i < B; i++) {
    if (mask && !mask[i]) continue;
    const double* v = mu + i * 3;
    if (!finite_all(v, 3) || !(v[0] * v[0] + v[1] * v[1] + v[2] * v[2] > 0.0)) return UWVK_EINVAL;
  }
  double* dz = h->d_meas;
  double* dc = h->d_meas + B * 3;
  HIPCHK(hipMemcpyAsync(dz, mu, (size_t)B * 3 * 8, hipMemcpyHostToDevice, h->stream));
  if (cov) HIPCHK(hipMemcpyAsync(dc, cov, (size_t)B * 4 * 8, hipMemcpyHostToDevice, h->stream));
  M9 sc{};
  if (!cov) std::memcpy(sc.v, shared_cov, 4 * 8);
  const uint8_t* dm;
  if (upload_mask(h, mask, &dm) != UWVK_OK) return UWVK_EDEVICE;
  hipLaunchKernelGGL(k_bottom_normal, dim3(grid_of(B, BE::IPB)), dim3(BE::BLOCK), 0, h->stream, h->bufs(), dz,
                     cov ? dc : nullptr, sc, dm);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_bottom_get_state(uwvk_bottom* h, double* x, double* P) { UWVK_DEVICE_GUARD(h); return small_get_state(h, x, P); }
uwvk_status uwvk_bottom_get_status(uwvk_bottom* h, uint32_t* status, int clear) {
  UWVK_DEVICE_GUARD(h);
  return small_get_status(h, status, clear);
}

// ---- IndirectPoseUKF -------------------------------------------------------
uwvk_status uwvk_ipose_create(int64_t batch, int device, uwvk_ipose** out) {
  ::uwvk::DeviceGuard uwvk_device_guard_(device);
  if (!out || batch <= 0) return UWVK_EINVAL;
  *out = nullptr;
  if (!uwvk_device_available(device)) return UWVK_EDEVICE;
  uwvk_ipose* h = new uwvk_ipose();
  const uwvk_status st = small_create(h, batch, device, 6, 7, 7, 0);
  if (st != UWVK_OK) {
    small_destroy(h);
    delete h;
    return st;
  }
  std::vector<double> ref((size_t)batch * 7, 0.0);  // Affine3d::Identity() (IndirectPoseUKF.cpp:58)
  for (int64_t i = 0; i < batch; i++) ref[i * 7 + 3] = 1.0;
  if (hipMemcpy(h->d_aux, ref.data(), ref.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
    small_destroy(h);
    delete h;
    return UWVK_EDEVICE;
  }
  *out = h;
  return UWVK_OK;
}

void uwvk_ipose_destroy(uwvk_ipose* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return;
  small_destroy(h);
  delete h;
}

void* uwvk_ipose_stream(const uwvk_ipose* h) { return h ? (void*)h->stream : nullptr; }

uwvk_status uwvk_ipose_set_option(uwvk_ipose* h, int option, int value) {
  if (!h) return UWVK_EINVAL;
  if (option == UWVK_OPT_SO3_RIGHT) {
    h->so3_right = value ? 1 : 0;
    return UWVK_OK;
  }
  return UWVK_EINVAL;
}

uwvk_status uwvk_ipose_init(uwvk_ipose* h, const double position_error_std[3], const double orientation_error_std[3],
                            double orientation_error_tau, const double* initial_position_error,
                            const double initial_position_error_std[3]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !position_error_std || !orientation_error_std) return UWVK_EINVAL;
  if (!(orientation_error_tau > 0.0)) return UWVK_EINVAL;
  const int64_t B = h->batch;
  std::vector<double> x((size_t)B * 7, 0.0), P((size_t)B * 36, 0.0);
  double Q[36] = {0};
  for (int k = 0; k < 3; k++) {
    const double s0 = initial_position_error_std ? initial_position_error_std[k] : 1.0;
    for (int64_t i = 0; i < B; i++) {
      P[i * 36 + k * 6 + k] = std::fabs(s0) * std::fabs(s0);
      P[i * 36 + (k + 3) * 6 + k + 3] = std::fabs(orientation_error_std[k]) * std::fabs(orientation_error_std[k]);
    }
    Q[k * 6 + k] = std::fabs(position_error_std[k]) * std::fabs(position_error_std[k]);
    Q[(k + 3) * 6 + k + 3] = std::fabs(orientation_error_std[k]) * std::fabs(orientation_error_std[k]);
  }
  for (int64_t i = 0; i < B; i++) {
    for (int k = 0; k < 3; k++) x[i * 7 + k] = initial_position_error ? initial_position_error[i * 3 + k] : 0.0;
    x[i * 7 + 3] = 1.0;
  }
  if (!finite_all(x.data(), x.size()) || !finite_all(P.data(), P.size()) || !finite_all(Q, 36)) return UWVK_ENAN;
  std::memcpy(h->Q.v, Q, sizeof(Q));
  h->tau = orientation_error_tau;
  HIPCHK(hipMemcpyAsync(h->d_mu, x.data(), x.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_sigma, P.data(), P.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return UWVK_OK;
}

uwvk_status uwvk_ipose_set_process_noise(uwvk_ipose* h, const double Q[36]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !Q) return UWVK_EINVAL;
  if (!finite_all(Q, 36)) return UWVK_ENAN;
  std::memcpy(h->Q.v, Q, sizeof(h->Q.v));
  return UWVK_OK;
}

uwvk_status uwvk_ipose_set_pose_reference(uwvk_ipose* h, const double* pose) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !pose) return UWVK_EINVAL;
  if (!finite_all(pose, (size_t)h->batch * 7)) return UWVK_ENAN;
  HIPCHK(hipMemcpyAsync(h->d_aux, pose, (size_t)h->batch * 7 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_ipose_predict(uwvk_ipose* h, double dt) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !(dt > 0.0)) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  if (h->so3_right)
    hipLaunchKernelGGL(k_ipose_predict<1>, dim3(grid_of(h->batch, IE<1>::IPB)), dim3(IE<1>::BLOCK), 0, h->stream,
                       h->bufs(), h->Q, h->tau, dt);
  else
    hipLaunchKernelGGL(k_ipose_predict<0>, dim3(grid_of(h->batch, IE<0>::IPB)), dim3(IE<0>::BLOCK), 0, h->stream,
                       h->bufs(), h->Q, h->tau, dt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_ipose_update_visual(uwvk_ipose* h, int32_t n_features, const double* features,
                                     const double* feature_cov, int feature_cov_per_instance,
                                     const double* feature_positions, const double* marker_pose,
                                     int marker_pose_per_instance, const double cov_marker_pose[36],
                                     const double camera[4], const double camera_in_body[7], const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  VisArgs va{};
  const int st = stage_visual(h->stream, h->batch, n_features, features, feature_cov, feature_cov_per_instance,
                              feature_positions, marker_pose, marker_pose_per_instance, cov_marker_pose, camera,
                              camera_in_body, mask, &va, &h->vis);
  if (st != 0 || va.nf == 0) {
    (void)hipStreamSynchronize(h->stream);
    return (uwvk_status)st;
  }
  va.ref = h->d_aux;
  if (h->so3_right)
    hipLaunchKernelGGL(k_ipose_visual<1>, dim3(grid_of(h->batch, IAE<1>::IPB)), dim3(IAE<1>::BLOCK), 0, h->stream,
                       h->bufs(), va);
  else
    hipLaunchKernelGGL(k_ipose_visual<0>, dim3(grid_of(h->batch, IAE<0>::IPB)), dim3(IAE<0>::BLOCK), 0, h->stream,
                       h->bufs(), va);
  const hipError_t e = hipGetLastError();
  return (uwvk_status)::uwvk::launch_sync_status(e, h->stream, "k_ipose_visual");
}

// getCorrectedPose (IndirectPoseUKF.cpp:137-142): pose_ref * pose_error, t(3) q(4)
uwvk_status uwvk_ipose_get_corrected_pose(uwvk_ipose* h, double* out) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !out) return UWVK_EINVAL;
  const int64_t B = h->batch;
  std::vector<double> x((size_t)B * 7), ref((size_t)B * 7);
  HIPCHK(hipMemcpyAsync(x.data(), h->d_mu, x.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipMemcpyAsync(ref.data(), h->d_aux, ref.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int64_t i = 0; i < B; i++) {
    const double* r = &ref[i * 7];
    const double* e = &x[i * 7];
    double* o = out + i * 7;
    // t = t_ref + R_ref p_err (Eigen _transformVector), q = q_ref * q_err
    const double* q = r + 3;
    double uv[3] = {2 * (q[2] * e[2] - q[3] * e[1]), 2 * (q[3] * e[0] - q[1] * e[2]), 2 * (q[1] * e[1] - q[2] * e[0])};
    double t2[3] = {q[2] * uv[2] - q[3] * uv[1], q[3] * uv[0] - q[1] * uv[2], q[1] * uv[1] - q[2] * uv[0]};
    for (int k = 0; k < 3; k++) o[k] = r[k] + (e[k] + q[0] * uv[k] + t2[k]);
    const double* b = e + 3;
    o[3] = q[0] * b[0] - q[1] * b[1] - q[2] * b[2] - q[3] * b[3];
    o[4] = q[0] * b[1] + q[1] * b[0] + q[2] * b[3] - q[3] * b[2];
    o[5] = q[0] * b[2] + q[2] * b[0] + q[3] * b[1] - q[1] * b[3];
    o[6] = q[0] * b[3] + q[3] * b[0] + q[1] * b[2] - q[2] * b[1];
  }
  return UWVK_OK;
}

uwvk_status uwvk_ipose_get_state(uwvk_ipose* h, double* x, double* P) { UWVK_DEVICE_GUARD(h); return small_get_state(h, x, P); }
uwvk_status uwvk_ipose_get_status(uwvk_ipose* h, uint32_t* status, int clear) {
  UWVK_DEVICE_GUARD(h);
  return small_get_status(h, status, clear);
}

}  // extern "C"
