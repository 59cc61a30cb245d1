// uwvk_pose.hip — PoseUKF kernels (gfx950) and the uwvk_pose_* C ABI.
//
// Grid: one 64-thread workgroup (= one wavefront) per filter instance.
// Every kernel loads (mu, Sigma) of its instance into LDS once, runs one or
// more predict / update steps on it and writes it back.  The fused epoch
// kernel (k_pose_epoch) is the hot path of uwvk_pose_run_log:
//   RotationRate -> predictionStep(dt) -> Acceleration update
//   [-> Velocity (DVL) -> Pressure -> ADCP cells -> BodyEfforts]
// with Sigma resident in LDS across all steps of the epoch.
#include <array>
#include <map>
#include "uwvk_pose_kernels.hpp"
#include "uwvk_psp.hpp"
#include "uwvk_host.hpp"
#include "uwvk_aug_dev.hpp"

namespace uwvk {
hipError_t launch_pose_visual(int dof, int right, hipStream_t st, const PoseBufs& b, const aug::VisArgs& va);
}

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

using namespace uwvk;


// ===========================================================================
// host side
// ===========================================================================
// ensemble statistics per instance group: 3 store + 1 doubles (store <= 54)
constexpr int64_t kStatsMaxOut = 3 * 54 + 2;

struct uwvk_pose {
  int64_t batch = 0;
  int dof = 53, store = 54, device = 0;
  hipStream_t stream = nullptr;
  double *d_mu = nullptr, *d_sigma = nullptr, *d_Q = nullptr, *d_rot = nullptr, *d_off = nullptr,
         *d_model = nullptr, *d_uwv = nullptr;
  uint32_t* d_status = nullptr;
  double* d_meas = nullptr;  // staging: batch*36 (mu) + batch*36 (cov) + batch*2 (extra)
  uint8_t* d_mask = nullptr;
  uint8_t* d_accepted = nullptr;
  double* d_scratch = nullptr;  // [0, 256): stats out + truth; [0, 3 batch): rotation rate; then stats partials
  PoseShared* d_shared = nullptr;  // device copy of sh for the PSP kernels
  PoseShared sh_dev{};             // what d_shared holds (valid when sh_dev_ok)
  bool sh_dev_ok = false;
  double* d_Qp = nullptr;          // {A_ii A_jj, dt^2 Q_ij} per packed entry (PSP)
  double* d_qband = nullptr;       // [128] dt^2 Q band of rows >= 9 (PSP)
  double qp_dt = -1.0;             // dt d_Qp was made for (-1: stale)
  std::vector<double> Qh;          // host copy of Q
  PoseShared sh{};
  uwvk_location loc{};
  uwvk_uwv_params uwv{};
  bool has_state = false, has_Q = false;
  int dense = 0;  // UWVK_OPT_DENSE_SIGMA
  // last-generation spreading of the PSP epoch launch (UWVK_OPT_TAIL_SLOTS)
  int64_t tail_slots = 0;  // resident blocks per XCD to plan for: 0 auto, < 0 off
  int tail_force = 0;      // UWVK_OPT_TAIL_CHUNKS: >= 2 forces that many chunks (tests)
  std::map<std::array<int64_t, 3>, int> tail_chunks;  // (instances per XCD, slots, epochs) -> chunks
  uint32_t* d_tail_flag = nullptr;  // per tail instance (batch / 8 - 1 per XCD at most)
  double* d_tail_carry = nullptr;   // per tail instance: 64 x (ds, ids)
  int64_t tail_inst_cap = 0;
  uint32_t tail_tag = 0;
  // persistent epoch kernel (UWVK_OPT_PERSIST): ticket counter and the value
  // it holds when the next launch starts (every launch takes units + grid)
  int persist = 1;  // UWVK_OPT_PERSIST (default since r06)
  uint32_t lds_pad = 0;  // UWVK_OPT_LDS_PAD (diagnostic occupancy sweep)
  // the parameter-decoupled epoch kernel (psp::PspSmemPD):
  // pdec = the 27 model-parameter DOFs' rows of Sigma are zero off the diagonal
  // (checked on the host at init; cleared by the full BodyEfforts update and by
  // any literal-kernel step, which do not keep those zeros exact)
  int pd_opt = 1;  // UWVK_OPT_PARAM_BLOCK
  int pair_opt = 1;  // UWVK_OPT_PAIR (default on): the PD kernel with two instances per wave (uwvk_psp_pair.hip)
  bool pdec = false;
  double* d_Qp_pd = nullptr;  // the PD table: the 26-DOF subset's {A A, dt^2 Q}, then the parameters' diagonal
  int wait_bound = -1;   // UWVK_OPT_WAIT_BOUND: < 0 the planner's bound, else that many sleeps (tests)
  uint32_t* d_ticket = nullptr;
  // hand-off fault word: pinned, coherent host memory the epoch kernel writes
  // directly (no copy on the stream); read after the stream has drained
  uint32_t* h_fault = nullptr;
  uint32_t* d_fault = nullptr;  // its device address
  uint32_t ticket_next = 0;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  aug::VisStage vis;  // visual-landmark update staging
};

// literal (all 2n+1 sigma points) kernels requested?
// (and the body-frame SO3 side, which only the literal kernels implement)
// the literal kernels: on request, or for ukfom's literal apply_delta re-spread
// (the PSP kernels run both SO3 sides, sh.so3_right, since r04)
static bool use_dense(const uwvk_pose* h) { return h->dense || h->sh.literal_apply_delta; }

static PoseBufs bufs(const uwvk_pose* h) {
  PoseBufs b;
  b.batch = h->batch; b.mu = h->d_mu; b.sigma = h->d_sigma; b.Q = h->d_Q; b.rot = h->d_rot; b.off = h->d_off;
  b.model = h->d_model; b.uwv = h->d_uwv; b.status = h->d_status;
  b.shared = h->d_shared;
  b.Qp = h->d_Qp;
  b.qband = h->d_qband;
  return b;
}

static void set_shared(uwvk_pose* h, const uwvk_pose_parameter& p, const uwvk_location& loc,
                       const uwvk_uwv_params& uwv) {
  h->loc = loc;
  h->uwv = uwv;
  h->sh.p = p;
  double rm, rn;
  host::wgs84_radii(loc.latitude, &rm, &rn);
  h->sh.lat0 = loc.latitude;
  h->sh.lon0 = loc.longitude;
  h->sh.rm = rm;
  h->sh.inv_rm = 1.0 / rm;
  h->sh.slat0 = std::sin(loc.latitude);
  h->sh.clat0 = std::cos(loc.latitude);
  h->sh.rn_cos = rn * std::cos(loc.latitude);
  const double taus[8] = {p.gyro_bias_tau, p.acc_bias_tau, p.inertia_tau, p.lin_damping_tau, p.quad_damping_tau,
                          p.water_velocity_tau, p.adcp_bias_tau, p.water_density_tau};
  for (int k = 0; k < 8; k++) h->sh.ntau[k] = -1.0 / taus[k];
  h->qp_dt = -1.0;  // the packed {A_ii A_jj, dt^2 Q} table depends on the taus
  h->sh.uwv_weight = uwv.weight;
  h->sh.uwv_buoyancy = uwv.buoyancy;
  for (int k = 0; k < 3; k++) {
    h->sh.cog[k] = uwv.distance_body2centerofgravity[k];
    h->sh.cob[k] = uwv.distance_body2centerofbuoyancy[k];
  }
}

// PSP kernels read the batch-shared parameters and dt^2 Q (packed) from device memory
// lane-resident Q (psp::LaneQ): no coupling of the rewritten rows (< 9) with
// anything but their own diagonal / the orientation block, and a band of at
// most 2 below the diagonal in rows >= 9 (the epoch kernel's QM = 1)
static bool q_is_simple(const uwvk_pose* h) {
  const int n = h->dof;
  auto Qij = [&](int i, int j) { return h->Qh.empty() ? 0.0 : h->Qh[(size_t)i * n + j]; };
  for (int i = 0; i < n; i++)
    for (int j = 0; j < i; j++) {
      if (Qij(i, j) == 0.0) continue;
      const bool ori = i >= 3 && i < 6 && j >= 3 && j < 6;
      if ((i < 9 || j < 9) ? !ori : (i - j > 2)) return false;
    }
  return true;
}

// the process noise leaves the parameter block decoupled: no Q entry in a
// parameter row / column (tangent 19..45) off the diagonal
static bool q_params_diag(const uwvk_pose* h) {
  if (h->dof != 53) return false;
  if (h->Qh.empty()) return true;
  for (int i = 0; i < 53; i++)
    for (int j = 0; j < 53; j++)
      if (i != j && ((i >= 19 && i <= 45) || (j >= 19 && j <= 45)) && h->Qh[(size_t)i * 53 + j] != 0.0) return false;
  return true;
}
// the next PSP epoch launch runs the parameter-decoupled kernel (after
// upload_shared: q_simple is the current Q's)
static bool use_pd(const uwvk_pose* h) {
  return h->pd_opt && h->pdec && h->dof == 53 && h->sh.q_simple && q_params_diag(h);
}

// the two-instances-per-wave kernel (UWVK_OPT_PAIR): the parameter-decoupled
// state of a 53-DOF handle, or a 26-DOF handle's own state (r06), on the
// persistent scheduler, an even batch, the lane-resident Q and no LDS pad
static bool pair_eligible(uwvk_pose* h) {
  if (!h->pair_opt || !h->persist || h->batch % 2 != 0 || h->lds_pad != 0 || use_dense(h)) return false;
  if (h->dof == 26) return q_is_simple(h);
  return h->pd_opt && h->pdec && h->dof == 53 && q_is_simple(h) && q_params_diag(h);  // (uwvk_pose_param_block)
}

static hipError_t upload_shared(uwvk_pose* h, double dt) {
  hipError_t e = hipSuccess;
  if (dt != h->qp_dt) {
    const int n = h->dof;
    // A_ii: the diagonal of the process model's Jacobian, the same expressions as
    // psp::proc_diag (1 + dt (-1/tau) per Markov block, 1 otherwise)
    std::vector<double> ad(n, 1.0);
    auto block = [&](int d0, int len, double nt) {
      for (int d = d0; d < d0 + len; d++) ad[d] = 1.0 + dt * nt;
    };
    const double* nt = h->sh.ntau;
    if (n == 53) {
      using L = Lay<53>;
      block(L::d_bg, 3, nt[0]); block(L::d_ba, 3, nt[1]); block(L::d_inertia, 9, nt[2]);
      block(L::d_lin, 9, nt[3]); block(L::d_quad, 9, nt[4]); block(L::d_wv, 4, nt[5]);
      block(L::d_badcp, 2, nt[6]); block(L::d_rho, 1, nt[7]);
    } else {
      using L = Lay<26>;
      block(L::d_bg, 3, nt[0]); block(L::d_ba, 3, nt[1]); block(L::d_wv, 4, nt[5]);
      block(L::d_badcp, 2, nt[6]); block(L::d_rho, 1, nt[7]);
    }
    auto rewritten = [](int d) { return d < 9; };  // pos, ori, vel rows: rewritten by the kernel
    auto Qij = [&](int i, int j) { return h->Qh.empty() ? 0.0 : h->Qh[(size_t)i * n + j]; };
    std::vector<double> qp((size_t)n * (n + 1));
    const double dt2 = dt * dt;
    for (int i = 0, k = 0; i < n; i++)
      for (int j = 0; j <= i; j++, k++) {
        qp[2 * k] = (rewritten(i) || rewritten(j)) ? 0.0 : ad[i] * ad[j];
        qp[2 * k + 1] = dt2 * Qij(i, j);
      }
    // band of rows >= 9: first nonzero column >= 9 .. diagonal
    std::vector<double> band(128, 0.0);
    int off = 0;
    bool fits = true;
    for (int i = 0; i < n; i++) {
      int lo = i + 1;
      if (i >= 9)
        for (int j = 9; j <= i; j++)
          if (Qij(i, j) != 0.0) { lo = j; break; }
      h->sh.qlo[i] = lo;
      h->sh.qoff[i] = off;
      for (int j = lo; j <= i; j++, off++) {
        if (off < 128) band[off] = dt2 * Qij(i, j);
        else fits = false;
      }
    }
    h->sh.q_band = fits ? 1 : 0;
    int bw = 0;
    for (int i = 9; i < n; i++) bw = std::max(bw, i - h->sh.qlo[i]);
    h->sh.q_bw = bw;
    h->sh.q_simple = q_is_simple(h) ? 1 : 0;
    e = hipMemcpyAsync(h->d_Qp, qp.data(), qp.size() * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h->d_qband, band.data(), 128 * 8, hipMemcpyHostToDevice, h->stream);
    // the PD kernel's table: the 26-DOF subset's entries in its packed order,
    // then parameter t's (19 + t, 19 + t) entry at 351 + t (psp::lane_q PD)
    std::vector<double> qpd((351 + 32) * 2, 0.0);
    if (n == 53) {
      auto m = [](int d) { return d < 19 ? d : d + 27; };
      for (int i = 0, k = 0; i < 26; i++)
        for (int j = 0; j <= i; j++, k++) {
          const int I = m(i), J = m(j), k53 = I * (I + 1) / 2 + J;
          qpd[2 * k] = qp[2 * k53];
          qpd[2 * k + 1] = qp[2 * k53 + 1];
        }
      for (int t = 0; t < 27; t++) {
        const int d = 19 + t, k53 = d * (d + 1) / 2 + d;
        qpd[2 * (351 + t)] = qp[2 * k53];
        qpd[2 * (351 + t) + 1] = qp[2 * k53 + 1];
      }
    }
    if (e == hipSuccess) e = hipMemcpyAsync(h->d_Qp_pd, qpd.data(), qpd.size() * 8, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);  // qp, band are locals
    if (e != hipSuccess) return e;
    h->qp_dt = dt;
  }
  // unchanged since the last upload (a run_log after another): no copy in
  // front of the launch (a pageable 2-KB copy cost ~10 us of the timed window)
  if (h->sh_dev_ok && std::memcmp(&h->sh_dev, &h->sh, sizeof(PoseShared)) == 0) return hipSuccess;
  e = hipMemcpyAsync(h->d_shared, &h->sh, sizeof(PoseShared), hipMemcpyHostToDevice, h->stream);
  h->sh_dev_ok = e == hipSuccess;
  if (h->sh_dev_ok) h->sh_dev = h->sh;
  return e;
}

#define HIPCHK(x)                                  \
  do {                                             \
    const hipError_t e_ = (x);                     \
    if (e_ != hipSuccess) {                        \
      ::uwvk::note_hip_error((int)e_, __func__);   \
      return UWVK_EDEVICE;                         \
    }                                              \
  } while (0)


static bool finite_all(const double* a, size_t n) {
  for (size_t k = 0; k < n; k++)
    if (!std::isfinite(a[k])) return false;
  return true;
}

extern "C" {

uwvk_status uwvk_pose_create(int64_t batch, int dof, int device, uwvk_pose** out) {
  ::uwvk::DeviceGuard uwvk_device_guard_(device);
  if (!out || batch <= 0 || (dof != 53 && dof != 26)) return UWVK_EINVAL;
  *out = nullptr;
  if (!uwvk_device_available(device)) return UWVK_EDEVICE;
  uwvk_pose* h = new uwvk_pose();
  h->batch = batch;
  h->dof = dof;
  h->store = dof == 53 ? 54 : 27;
  h->device = device;
  h->sh.so3_right = 1;  // MTK's SO3::boxplus, q exp(d): the default side since r05 (UWVK_OPT_SO3_RIGHT)
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    return UWVK_EDEVICE;
  }
  const size_t B = (size_t)batch, n = (size_t)dof;
  // Sigma: packed lower triangle per instance (B n (n + 1) / 2 doubles)
  bool ok = hipMalloc(&h->d_mu, B * h->store * 8) == hipSuccess &&
            hipMalloc(&h->d_sigma, B * (n * (n + 1) / 2) * 8) == hipSuccess &&
            hipMalloc(&h->d_Q, n * n * 8) == hipSuccess && hipMalloc(&h->d_rot, B * 3 * 8) == hipSuccess &&
            hipMalloc(&h->d_off, B * 28 * 8) == hipSuccess && hipMalloc(&h->d_model, B * 27 * 8) == hipSuccess &&
            hipMalloc(&h->d_uwv, 108 * 8) == hipSuccess && hipMalloc(&h->d_status, B * 4) == hipSuccess &&
            hipMalloc(&h->d_meas, B * 74 * 8) == hipSuccess && hipMalloc(&h->d_mask, B) == hipSuccess &&
            hipMalloc(&h->d_accepted, B) == hipSuccess && hipMalloc(&h->d_scratch, (B * 3 + 256 + ((B + 63) / 64) * kStatsMaxOut) * 8) == hipSuccess &&
            hipMalloc(&h->d_shared, sizeof(PoseShared)) == hipSuccess &&
            hipMalloc(&h->d_Qp, n * (n + 1) * 8) == hipSuccess && hipMalloc(&h->d_qband, 128 * 8) == hipSuccess &&
            hipMalloc(&h->d_Qp_pd, (351 + 32) * 2 * 8) == hipSuccess &&
            hipMalloc(&h->d_ticket, 4) == hipSuccess &&
            hipHostMalloc((void**)&h->h_fault, 4, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer((void**)&h->d_fault, h->h_fault, 0) == hipSuccess &&
            hipEventCreate(&h->ev0) == hipSuccess && hipEventCreate(&h->ev1) == hipSuccess;
  if (!ok) {
    uwvk_pose_destroy(h);
    return UWVK_ENOMEM;
  }
  (void)hipMemsetAsync(h->d_status, 0, B * 4, h->stream);
  (void)hipMemsetAsync(h->d_rot, 0, B * 3 * 8, h->stream);
  (void)hipMemsetAsync(h->d_Q, 0, n * n * 8, h->stream);
  (void)hipMemsetAsync(h->d_ticket, 0, 4, h->stream);
  *h->h_fault = 0;
  if (hipStreamSynchronize(h->stream) != hipSuccess) {
    uwvk_pose_destroy(h);
    return UWVK_EDEVICE;
  }
  *out = h;
  return UWVK_OK;
}

void uwvk_pose_destroy(uwvk_pose* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return;
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  for (void* p : {(void*)h->d_mu, (void*)h->d_sigma, (void*)h->d_Q, (void*)h->d_rot, (void*)h->d_off,
                  (void*)h->d_model, (void*)h->d_uwv, (void*)h->d_status, (void*)h->d_meas, (void*)h->d_mask,
                  (void*)h->d_accepted, (void*)h->d_scratch, (void*)h->d_shared, (void*)h->d_Qp, (void*)h->d_qband,
                  (void*)h->d_Qp_pd,
                  (void*)h->d_tail_flag, (void*)h->d_tail_carry, (void*)h->d_ticket})
    if (p) (void)hipFree(p);
  if (h->h_fault) (void)hipHostFree(h->h_fault);
  h->vis.release();
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

int64_t uwvk_pose_batch(const uwvk_pose* h) { return h ? h->batch : 0; }
int uwvk_pose_dof(const uwvk_pose* h) { return h ? h->dof : 0; }
void* uwvk_pose_stream(const uwvk_pose* h) { return h ? (void*)h->stream : nullptr; }
// a tail-chunk hand-off that timed out in a launch that has completed (the
// kernel wrote the handle's host-mapped fault word); reported once
static bool take_fault(uwvk_pose* h) {
  if (!__atomic_load_n(h->h_fault, __ATOMIC_ACQUIRE)) return false;
  __atomic_store_n(h->h_fault, 0u, __ATOMIC_RELEASE);
  return true;
}

uwvk_status uwvk_pose_synchronize(uwvk_pose* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  const hipError_t e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return (uwvk_status)::uwvk::edevice_status(e, "uwvk_pose_synchronize");
  return take_fault(h) ? UWVK_ESCHEDULE : UWVK_OK;
}

// Both init calls replace the reference's constructors (PoseUKF.cpp:288-391):
// the filter object is new, so the process noise is zero until it is set again
// and the stored rotation rate is zero (:380); the handle keeps its stream,
// buffers and options.
static uwvk_status upload_state(uwvk_pose* h, const std::vector<double>& x, const std::vector<double>& P,
                                const std::vector<double>& off, const std::vector<double>& model) {
  const size_t n = (size_t)h->dof;
  h->Qh.assign(n * n, 0.0);
  h->qp_dt = -1.0;
  for (double& v : h->sh.q_ori) v = 0.0;
  for (double& v : h->sh.q_wv) v = 0.0;
  HIPCHK(hipMemsetAsync(h->d_Q, 0, n * n * 8, h->stream));
  HIPCHK(hipMemsetAsync(h->d_rot, 0, (size_t)h->batch * 3 * 8, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_mu, x.data(), x.size() * 8, hipMemcpyHostToDevice, h->stream));
  // HBM keeps the packed lower triangle (the caller's P is the full matrix;
  // its lower triangle is taken, like the Cholesky-based ukfom reads it)
  const int tn = h->dof * (h->dof + 1) / 2;
  std::vector<double> Pp((size_t)h->batch * tn);
  for (int64_t b = 0; b < h->batch; b++)
    for (int i = 0, k = 0; i < h->dof; i++)
      for (int j = 0; j <= i; j++, k++) Pp[b * tn + k] = P[(b * h->dof + i) * h->dof + j];
  HIPCHK(hipMemcpyAsync(h->d_sigma, Pp.data(), Pp.size() * 8, hipMemcpyHostToDevice, h->stream));
  // the parameter block decoupled (PD kernel): every lower-triangle entry in a
  // parameter row or column (tangent 19..45) off the diagonal is zero
  h->pdec = false;
  if (h->dof == 53) {
    bool dec = true;
    for (int64_t b = 0; b < h->batch && dec; b++)
      for (int i = 19, k0 = 19 * 20 / 2; i < 53 && dec; k0 += ++i)
        for (int j = 0; j < i; j++)
          if ((i <= 45 || (j >= 19 && j <= 45)) && Pp[b * tn + k0 + j] != 0.0) {
            dec = false;
            break;
          }
    h->pdec = dec;
  }
  HIPCHK(hipMemcpyAsync(h->d_off, off.data(), off.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemcpyAsync(h->d_model, model.data(), model.size() * 8, hipMemcpyHostToDevice, h->stream));
  double uw[108];
  std::memcpy(uw, h->uwv.inertia_matrix, 36 * 8);
  std::memcpy(uw + 36, h->uwv.damping_matrices[0], 36 * 8);
  std::memcpy(uw + 72, h->uwv.damping_matrices[1], 36 * 8);
  HIPCHK(hipMemcpyAsync(h->d_uwv, uw, sizeof(uw), hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipMemsetAsync(h->d_status, 0, (size_t)h->batch * 4, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_state = true;
  return UWVK_OK;
}

uwvk_status uwvk_pose_init_from_config(uwvk_pose* h, const double* pos, const double* pos_cov, const double* rot,
                                       const double* rot_cov, const uwvk_pose_config* cfg, const uwvk_uwv_params* uwv,
                                       const double imu_in_body[7]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !pos || !pos_cov || !rot || !rot_cov || !cfg || !uwv) return UWVK_EINVAL;
  const int64_t B = h->batch;
  const int n = h->dof, s = h->store;
  std::vector<double> x(B * s), P(B * n * n), off(B * 28), model(B * 27);
  uwvk_pose_parameter par{};
  for (int64_t i = 0; i < B; i++) {
    host::pose_initial_state(n, pos + 3 * i, pos_cov + 9 * i, rot + 4 * i, rot_cov + 9 * i, *cfg, *uwv, imu_in_body,
                             &x[i * s], &P[i * n * n], &par);
    host::pose_offsets(n, &x[i * s], &off[i * 28]);
    host::model_blocks(*uwv, &model[i * 27]);
  }
  set_shared(h, par, cfg->location, *uwv);
  return upload_state(h, x, P, off, model);
}

uwvk_status uwvk_pose_init_from_state(uwvk_pose* h, const double* x, const double* P, const uwvk_location* loc,
                                      const uwvk_uwv_params* uwv, const uwvk_pose_parameter* param) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !x || !P || !loc || !uwv || !param) return UWVK_EINVAL;
  const int64_t B = h->batch;
  const int n = h->dof, s = h->store;
  std::vector<double> xs(x, x + B * s), Ps(P, P + B * n * n), off(B * 28), model(B * 27);
  for (int64_t i = 0; i < B; i++) {
    host::pose_offsets(n, &xs[i * s], &off[i * 28]);
    host::model_blocks(*uwv, &model[i * 27]);
  }
  set_shared(h, *param, *loc, *uwv);
  return upload_state(h, xs, Ps, off, model);
}

uwvk_status uwvk_pose_set_process_noise_from_config(uwvk_pose* h, const uwvk_pose_config* cfg, double imu_delta_t,
                                                    const double q_imu_in_body[4]) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !cfg || !(imu_delta_t > 0)) return UWVK_EINVAL;
  std::vector<double> Q(h->dof * h->dof);
  host::pose_process_noise(h->dof, *cfg, imu_delta_t, q_imu_in_body, Q.data());
  return uwvk_pose_set_process_noise(h, Q.data());
}

uwvk_status uwvk_pose_set_process_noise(uwvk_pose* h, const double* Q) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !Q) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(h->d_Q, Q, (size_t)h->dof * h->dof * 8, hipMemcpyHostToDevice, h->stream));
  h->Qh.assign(Q, Q + (size_t)h->dof * h->dof);
  h->qp_dt = -1.0;
  {
    const int n = h->dof, o = 3, wv = n == 53 ? 46 : 19;
    for (int r = 0; r < 3; r++)
      for (int c = 0; c < 3; c++) h->sh.q_ori[r * 3 + c] = Q[(o + r) * n + o + c];
    for (int k = 0; k < 4; k++) h->sh.q_wv[k] = Q[(wv + k) * n + wv + k];
  }
  HIPCHK(hipStreamSynchronize(h->stream));
  h->has_Q = true;
  return UWVK_OK;
}

uwvk_status uwvk_pose_set_rotation_rate(uwvk_pose* h, const double* w, const double* cov) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !w) return UWVK_EINVAL;
  if (!finite_all(w, (size_t)h->batch * 3) || (cov && !finite_all(cov, (size_t)h->batch * 9))) return UWVK_ENAN;
  HIPCHK(hipMemcpyAsync(h->d_rot, w, (size_t)h->batch * 3 * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_pose_predict(uwvk_pose* h, double dt) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  PoseBufs b = bufs(h);
  if (use_dense(h)) {
    h->pdec = false;  // the literal covariance GEMM does not keep the parameter block's zeros exact
    HIPCHK(launch_pose_predict(h->dof, h->stream, b, h->sh, dt));
  }
  else {
    // upload_shared recomputes the Q shape (q_bw, q_simple, qlo, qoff) for this dt:
    // the by-value PoseShared handed to the kernel must be taken after it
    HIPCHK(upload_shared(h, dt));
    const PoseShared sh = h->sh;
    HIPCHK(launch_psp_predict(h->dof, h->stream, b, sh, dt));
  }
  return UWVK_OK;
}

}  // extern "C"

template <int K>
static uwvk_status launch_update(uwvk_pose* h, int m, const double* mu, const double* cov, const double* shared_cov,
                                 const uint8_t* mask, uint8_t* accepted, const double* extra, int extra_w,
                                 const double* v3, int only_vel) {
  if (!h || !mu || (!cov && !shared_cov)) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  const int64_t B = h->batch;
  // checkMeasurment [EXT] (PoseUKF.cpp:478): NaN -> error, nothing applied
  for (int64_t i = 0; i < B; i++) {
    if (mask && !mask[i]) continue;
    if (!finite_all(mu + i * m, m) || (cov && !finite_all(cov + i * m * m, (size_t)m * m))) return UWVK_ENAN;
  }
  if (!cov && !finite_all(shared_cov, (size_t)m * m)) return UWVK_ENAN;
  MeasArgs ma{};
  double* dmu = h->d_meas;
  double* dcov = h->d_meas + B * 36;
  double* dext = h->d_meas + B * 72;
  HIPCHK(hipMemcpyAsync(dmu, mu, (size_t)B * m * 8, hipMemcpyHostToDevice, h->stream));
  ma.mu = dmu;
  if (cov) {
    HIPCHK(hipMemcpyAsync(dcov, cov, (size_t)B * m * m * 8, hipMemcpyHostToDevice, h->stream));
    ma.cov = dcov;
  } else {
    std::memcpy(ma.shared_cov, shared_cov, (size_t)m * m * 8);
  }
  if (mask) {
    HIPCHK(hipMemcpyAsync(h->d_mask, mask, (size_t)B, hipMemcpyHostToDevice, h->stream));
    ma.mask = h->d_mask;
  }
  if (extra) {
    HIPCHK(hipMemcpyAsync(dext, extra, (size_t)B * extra_w * 8, hipMemcpyHostToDevice, h->stream));
    ma.extra = dext;
  }
  if (v3)
    for (int k = 0; k < 3; k++) ma.v3[k] = v3[k];
  ma.only_vel = only_vel;
  ma.accepted = h->d_accepted;
  PoseBufs b = bufs(h);
  // BodyEfforts on PSP too (r05): the full model with k = 48 (psp_update_eff),
  // its velocity-only form (constrainVelocity) with k = 9
  // the literal kernels, and the full BodyEfforts model (non-affine in the
  // parameters), couple the parameter block: no PD kernel afterwards
  if (use_dense(h) || (K == MK_EFFORTS && !only_vel)) h->pdec = false;
  if (use_dense(h))
    HIPCHK(launch_pose_update(h->dof, K, h->stream, b, h->sh, ma, m));
  else {
    HIPCHK(upload_shared(h, h->qp_dt));
    const PoseShared sh = h->sh;  // after upload_shared (it refreshes the Q shape)
    HIPCHK(launch_psp_update(h->dof, K, h->stream, b, sh, ma, m));
  }
  if (accepted) HIPCHK(hipMemcpyAsync(accepted, h->d_accepted, (size_t)B, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

extern "C" {

uwvk_status uwvk_pose_update_acceleration(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                          const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  return launch_update<MK_ACC>(h, 3, mu, cov, sc, mask, acc, nullptr, 0, nullptr, 0);
}
uwvk_status uwvk_pose_update_velocity(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                      const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  return launch_update<MK_VEL>(h, 3, mu, cov, sc, mask, acc, nullptr, 0, nullptr, 0);
}
uwvk_status uwvk_pose_update_pressure(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                      const double sensor_in_imu[3], const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  const double zero[3] = {0, 0, 0};
  return launch_update<MK_PRESSURE>(h, 1, mu, cov, sc, mask, acc, nullptr, 0, sensor_in_imu ? sensor_in_imu : zero, 0);
}
uwvk_status uwvk_pose_update_water_velocity(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                            const double* cw, const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  if (!cw) return UWVK_EINVAL;
  return launch_update<MK_WATER>(h, 2, mu, cov, sc, mask, acc, cw, 1, nullptr, 0);
}
uwvk_status uwvk_pose_update_efforts(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                     int only_affect_velocity, const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  return launch_update<MK_EFFORTS>(h, 6, mu, cov, sc, mask, acc, nullptr, 0, nullptr, only_affect_velocity ? 1 : 0);
}
uwvk_status uwvk_pose_update_xy(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  return launch_update<MK_XY>(h, 2, mu, cov, sc, mask, acc, nullptr, 0, nullptr, 0);
}
uwvk_status uwvk_pose_update_z(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                               const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  return launch_update<MK_Z>(h, 1, mu, cov, sc, mask, acc, nullptr, 0, nullptr, 0);
}
uwvk_status uwvk_pose_update_geographic(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                        const double gps_in_body[3], const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  const double zero[3] = {0, 0, 0};
  return launch_update<MK_GEO>(h, 2, mu, cov, sc, mask, acc, nullptr, 0, gps_in_body ? gps_in_body : zero, 0);
}
// integrateMeasurement(vector<VisualFeatureMeasurement>, feature_positions, marker_pose,
// cov_marker_pose, camera_config, camera_in_IMU) (PoseUKF.cpp:613-654)
uwvk_status uwvk_pose_update_visual_landmark(uwvk_pose* h, int32_t n_features, const double* features,
                                             const double* feature_cov, int feature_cov_per_instance,
                                             const double* feature_positions, const double* marker_pose,
                                             int marker_pose_per_instance, const double cov_marker_pose[36],
                                             const double camera[4], const double camera_in_imu[7],
                                             const uint8_t* mask) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  aug::VisArgs va{};
  const int st = aug::stage_visual(h->stream, h->batch, n_features, features, feature_cov, feature_cov_per_instance,
                                   feature_positions, marker_pose, marker_pose_per_instance, cov_marker_pose, camera,
                                   camera_in_imu, mask, &va, &h->vis);
  if (st != 0 || va.nf == 0) {
    (void)hipStreamSynchronize(h->stream);
    return (uwvk_status)st;
  }
  h->pdec = false;  // the literal augmented update (all sigma points)
  const hipError_t e = launch_pose_visual(h->dof, h->sh.so3_right, h->stream, bufs(h), va);
  return (uwvk_status)::uwvk::launch_sync_status(e, h->stream, "launch_pose_visual");
}

uwvk_status uwvk_pose_update_delayed_xy(uwvk_pose* h, const double* mu, const double* cov, const double* sc,
                                        const double* delayed_xy, const uint8_t* mask, uint8_t* acc) {
  UWVK_DEVICE_GUARD(h);
  if (!delayed_xy) return UWVK_EINVAL;
  return launch_update<MK_DELAYED>(h, 2, mu, cov, sc, mask, acc, delayed_xy, 2, nullptr, 0);
}

uwvk_status uwvk_pose_reset_with_external_pose(uwvk_pose* h, const double* pose) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !pose) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  const int64_t B = h->batch;
  std::vector<double> x(B * h->store);
  HIPCHK(hipMemcpyAsync(x.data(), h->d_mu, x.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int64_t i = 0; i < B; i++) std::memcpy(&x[i * h->store], pose + 7 * i, 7 * 8);  // PoseUKF.cpp:687-690
  HIPCHK(hipMemcpyAsync(h->d_mu, x.data(), x.size() * 8, hipMemcpyHostToDevice, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_pose_get_state(uwvk_pose* h, double* x, double* P) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !x) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(x, h->d_mu, (size_t)h->batch * h->store * 8, hipMemcpyDeviceToHost, h->stream));
  if (!P) {
    HIPCHK(hipStreamSynchronize(h->stream));
    return UWVK_OK;
  }
  // packed lower triangle -> the full symmetric matrix
  const int n = h->dof, tn = n * (n + 1) / 2;
  std::vector<double> Pp((size_t)h->batch * tn);
  HIPCHK(hipMemcpyAsync(Pp.data(), h->d_sigma, Pp.size() * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  for (int64_t b = 0; b < h->batch; b++) {
    const double* s = &Pp[b * tn];
    double* d = P + (size_t)b * n * n;
    for (int i = 0, k = 0; i < n; i++)
      for (int j = 0; j <= i; j++, k++) d[i * n + j] = d[j * n + i] = s[k];
  }
  return UWVK_OK;
}

uwvk_status uwvk_pose_get_rotation_rate(uwvk_pose* h, double* out) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !out) return UWVK_EINVAL;
  PoseBufs b = bufs(h);
  PoseShared sh = h->sh;
  double* d = h->d_scratch;
  HIPCHK(launch_pose_rotation_rate(h->dof, h->stream, b, sh, d));
  HIPCHK(hipMemcpyAsync(out, d, (size_t)h->batch * 3 * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_pose_get_status(uwvk_pose* h, uint32_t* status, int clear) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !status) return UWVK_EINVAL;
  HIPCHK(hipMemcpyAsync(status, h->d_status, (size_t)h->batch * 4, hipMemcpyDeviceToHost, h->stream));
  if (clear) HIPCHK(hipMemsetAsync(h->d_status, 0, (size_t)h->batch * 4, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

// flags and carries for `need` tail instances (sized once for the largest
// plan: 8 chunks of these slots), and this launch's flag tag
static hipError_t tail_buffers(uwvk_pose* h, int64_t need, int64_t cap) {
  if (need > h->tail_inst_cap) {
    // the previous buffers may still be read by a queued launch
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return e;
    if (h->d_tail_flag) (void)hipFree(h->d_tail_flag);
    if (h->d_tail_carry) (void)hipFree(h->d_tail_carry);
    h->d_tail_flag = nullptr;
    h->d_tail_carry = nullptr;
    h->tail_inst_cap = 0;
    cap = std::max(cap, need);
    e = hipMalloc(&h->d_tail_flag, (size_t)cap * 4);
    if (e == hipSuccess) e = hipMalloc(&h->d_tail_carry, (size_t)cap * 128 * 8);
    if (e == hipSuccess) e = hipMemsetAsync(h->d_tail_flag, 0, (size_t)cap * 4, h->stream);
    if (e != hipSuccess) return e;
    h->tail_inst_cap = cap;
    h->tail_tag = 0;
  }
  if (++h->tail_tag >= (1u << 27)) {  // flags hold tag * 16 + chunks done: restart on zeroed flags
    hipError_t e = hipMemsetAsync(h->d_tail_flag, 0, (size_t)h->tail_inst_cap * 4, h->stream);
    if (e != hipSuccess) return e;
    h->tail_tag = 1;
  }
  return hipSuccess;
}

// chunk count of a launch: the planner's (cached per shape), or the forced one
static int tail_plan(uwvk_pose* h, int64_t n, int64_t s, int64_t count) {
  const std::array<int64_t, 3> key{n, s, count};
  auto it = h->tail_chunks.find(key);
  if (it == h->tail_chunks.end()) {
    if (h->tail_chunks.size() >= 64) h->tail_chunks.clear();
    it = h->tail_chunks.emplace(key, plan_tail(n, s, count)).first;
  }
  int c = it->second;
  if (h->tail_force >= 2)  // forced (tests): every chunk count, where the shape allows it
    c = (s > 0 && h->tail_force <= 8 && h->tail_force * s <= n && h->tail_force <= count) ? h->tail_force : 1;
  return c;
}

// Persistent launch (UWVK_OPT_PERSIST): grid = resident blocks (or fewer
// units); the last r = chunks x slots instances run as epoch chunks, claimed
// in chunk order (uwvk_psp_k.hip, k_psp_epoch_p).  UWVK_OPT_TAIL_SLOTS < 0
// turns the chunks off, > 0 plans for that many slots per XCD.
// pair: the two-instances-per-wave kernel, whose units are pairs of instances
static hipError_t prepare_persist(uwvk_pose* h, EpochArgs& ea, int64_t& grid, int pd, int pair = 0) {
  const int64_t B = pair ? h->batch / 2 : h->batch;
  const int64_t slots = pair ? psp_pair_slots(h->device) : psp_epoch_slots(h->dof, h->device, true, pd);
  const int64_t s = h->tail_slots > 0 ? 8 * h->tail_slots : slots;
  if (slots <= 0) return hipErrorInvalidValue;
  ea.chunks = 1;
  ea.tail0 = B;
  ea.r_x = 0;
  int c = h->tail_slots < 0 || h->lds_pad > 0 || s <= 0 ? 1 : tail_plan(h, B, s, ea.count);
  // the pair kernel's default: no spreading (r06v, interleaved: off +2.4% at 20
  // epochs, a tie at 200; forced 3 / 4 chunks -6% / -18% at 20); an explicit
  // UWVK_OPT_TAIL_SLOTS > 0 or UWVK_OPT_TAIL_CHUNKS still spreads (tests)
  if (pair && h->tail_slots == 0 && h->tail_force < 2) c = 1;
  if (c > 1) {
    const int64_t r = c * s;
    hipError_t e = tail_buffers(h, r, 8 * s);
    if (e != hipSuccess) return e;
    ea.tail_flag = h->d_tail_flag;
    ea.tail_carry = h->d_tail_carry;
    ea.tail0 = B - r;
    ea.r_x = r;
    ea.chunks = c;
    ea.tag = h->tail_tag;
    // a chunk waits at most for its predecessor's unit and the unit its block
    // held before it: ~2 of the launch's epochs per wave, see prepare_tail
    ea.wait_bound = (uint32_t)std::min<uint64_t>(0xffffffffull, (1ull << 20) + 128ull * (uint64_t)ea.count);
    if (h->wait_bound >= 0) ea.wait_bound = (uint32_t)h->wait_bound;
  }
  const int64_t units = ea.tail0 + (int64_t)ea.chunks * ea.r_x;
  grid = std::min<int64_t>(units, slots);
  ea.units = (uint32_t)units;
  ea.ticket = h->d_ticket;
  ea.ticket_base = h->ticket_next;
  // the first grid units are the blocks' own; the counter then numbers units
  // grid .. units - 1 and one failing ticket per block: units - grid + grid.
  // ticket_next advances only once the launch is queued (commit_persist): a
  // launch that fails leaves the device counter where it was
  return hipSuccess;
}

// the tail layout of one PSP epoch launch (uwvk_psp_k.hip, plan_tail), cached
// per (instances per XCD, slots, epochs); fills ea's tail fields and the grid
static hipError_t prepare_tail(uwvk_pose* h, EpochArgs& ea, int64_t& grid, int pd) {
  ea.chunks = 1;
  ea.ticket = nullptr;
  grid = 0;
  if (h->persist) return prepare_persist(h, ea, grid, pd);
  // an LDS pad lowers the resident blocks below what the tail plan assumes:
  // no spreading then (UWVK_OPT_LDS_PAD is a diagnostic of the unspread launch)
  if (h->tail_slots < 0 || h->lds_pad > 0 || h->batch % 8 != 0) return hipSuccess;
  // placement not the round-robin the XCD-ordered tail plan needs (a
  // partitioned device, another runtime): the ticket-ordered persistent
  // launch spreads the tail without any placement assumption
  if (!xcd_round_robin(h->device)) return prepare_persist(h, ea, grid, pd);
  const int64_t n = h->batch / 8;
  const int64_t s = h->tail_slots > 0 ? h->tail_slots : psp_epoch_slots_per_xcd(h->dof, h->device, pd);
  const int c = tail_plan(h, n, s, ea.count);
  if (c <= 1) return hipSuccess;
  const int64_t r = c * s;
  hipError_t e = tail_buffers(h, 8 * r, 8 * std::max<int64_t>(r, 8 * s));
  if (e != hipSuccess) return e;
  ea.tail_flag = h->d_tail_flag;
  ea.tail_carry = h->d_tail_carry;
  ea.n_x = n;
  ea.tail0 = n - r;
  ea.r_x = r;
  ea.chunks = c;
  ea.tag = h->tail_tag;
  // a chunk waits at most for its predecessors' (c - 1) / c of the launch's
  // epochs; one sleep is ~1.7 us and an epoch ~20 us per wave at full
  // occupancy: 64 sleeps per epoch is a wide margin, plus ~2 s of slack
  ea.wait_bound = (uint32_t)std::min<uint64_t>(0xffffffffull, (1ull << 20) + 64ull * (uint64_t)ea.count);
  if (h->wait_bound >= 0) ea.wait_bound = (uint32_t)h->wait_bound;
  grid = 8 * (n + (c - 1) * r);
  return hipSuccess;
}

uwvk_status uwvk_pose_run_log(uwvk_pose* h, const uwvk_pose_log* log, int64_t first, int64_t count,
                              uint32_t* accept_counts) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !log || first < 0 || count < 0 || first + count > log->epochs || log->adcp_cells > 8) return UWVK_EINVAL;
  if (!h->has_state) return UWVK_ENOTINIT;
  // ABI 3: a hand-off timeout of an earlier, completed launch is reported here
  // (or by uwvk_pose_synchronize), before any new work is queued
  if (take_fault(h)) return UWVK_ESCHEDULE;
  EpochArgs ea{};
  ea.flags = log->flags; ea.gyro = log->gyro; ea.acc = log->acc;
  std::memcpy(ea.acc_cov, log->acc_cov, sizeof(ea.acc_cov));
  ea.dvl_index = log->dvl_index; ea.dvl = log->dvl;
  std::memcpy(ea.dvl_cov, log->dvl_cov, sizeof(ea.dvl_cov));
  ea.p_index = log->pressure_index; ea.pressure = log->pressure; ea.p_cov = log->pressure_cov;
  std::memcpy(ea.p_sens, log->pressure_sensor_in_imu, sizeof(ea.p_sens));
  ea.a_index = log->adcp_index; ea.adcp = log->adcp; ea.cells = log->adcp_cells;
  std::memcpy(ea.cw, log->adcp_cell_weighting, sizeof(ea.cw));
  std::memcpy(ea.adcp_cov, log->adcp_cov, sizeof(ea.adcp_cov));
  ea.e_index = log->efforts_index; ea.efforts = log->efforts;
  std::memcpy(ea.e_cov, log->efforts_cov, sizeof(ea.e_cov));
  ea.dt = log->dt;
  ea.accept_counts = accept_counts;
  PoseBufs b = bufs(h);
  if (use_dense(h)) {  // literal kernels: one fused launch per epoch
    h->pdec = false;
    for (int64_t e = first; e < first + count; e++) {
      ea.first = e;
      ea.count = 1;
      HIPCHK(launch_pose_epoch(h->dof, h->stream, b, h->sh, ea));
    }
    return UWVK_OK;
  }
  // PSP: one launch per run of epochs up to and including the next BodyEfforts
  // epoch (its predict and other updates); that epoch's efforts update alone
  // then runs in its own one-wave PSP kernel (k_psp_efforts: the full model or
  // its velocity-only form; its own register / LDS budget).  Efforts is the
  // last update of an epoch (the fused literal order), so the split is exact.
  std::vector<uint32_t> fl;
  const uint32_t* hf = log->host_flags ? log->host_flags + first : nullptr;
  if (!hf && count > 0) {
    fl.resize((size_t)count);
    HIPCHK(hipMemcpyAsync(fl.data(), log->flags + first, (size_t)count * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    hf = fl.data();
  }
  std::memcpy(h->sh.log_acc_cov, log->acc_cov, sizeof(h->sh.log_acc_cov));
  std::memcpy(h->sh.log_dvl_cov, log->dvl_cov, sizeof(h->sh.log_dvl_cov));
  HIPCHK(upload_shared(h, log->dt));
  const PoseShared sh = h->sh;  // after upload_shared (it refreshes the Q shape)
  ea.fault = h->d_fault;
  // one epoch-kernel launch over [s0, s1): the pair kernel or the one-instance
  // PSP kernel (parameter-decoupled while eligible)
  auto launch_seg = [&](int64_t s0, int64_t s1, bool use_pair) -> uwvk_status {  // (pair or one-instance)
    ea.first = s0;
    ea.count = s1 - s0;
    ea.efforts_only = 0;
    int64_t grid = 0;
    uint32_t ev_any = 0;  // the event kinds of this launch's epochs (kernel choice)
    for (int64_t k = s0; k < s1; k++) ev_any |= hf[k - first];
    const int pd = use_pd(h) ? 1 : 0;
    PoseBufs bl = b;
    if (pd) bl.Qp = h->d_Qp_pd;
    if (h->dof == 53 && !pd) use_pair = false;  // (the pair kernel runs a 53-DOF state decoupled only)
    hipError_t le;
    if (use_pair) {
      ea.chunks = 1;
      ea.ticket = nullptr;
      HIPCHK(prepare_persist(h, ea, grid, pd, 1));
      le = launch_psp_epoch_pair(h->stream, bl, sh, ea, grid, ev_any, pd);
    } else {
      HIPCHK(prepare_tail(h, ea, grid, pd));
      le = launch_psp_epoch(h->dof, h->stream, bl, sh, ea, grid, ev_any, h->lds_pad, pd);
    }
    if (le != hipSuccess) {
      ::uwvk::note_hip_error((int)le, use_pair ? "launch_psp_epoch_pair" : "launch_psp_epoch");
      // a persistent launch that did not run took no tickets: restart the
      // counter from zero (stream-ordered, before any later launch)
      if (ea.ticket) {
        h->ticket_next = 0;
        (void)hipMemsetAsync(h->d_ticket, 0, 4, h->stream);
      }
      return UWVK_EDEVICE;
    }
    if (ea.ticket) h->ticket_next += ea.units;  // the tickets the launch takes
    return UWVK_OK;
  };
  int64_t e = first;
  while (e < first + count) {
    int64_t r = e;
    while (r < first + count && !(hf[r - first] & UWVK_EV_EFFORTS)) r++;
    const int64_t last = r < first + count ? r + 1 : r;
    // the two-instances-per-wave form of the parameter-decoupled kernel
    // (UWVK_OPT_PAIR; persistent, even batch) runs the epochs without a
    // pressure update (its 39 sigma points do not fit a half-wave): a launch
    // with pressure epochs is split around them when the runs between them are
    // long (kPairMinRun epochs: each extra launch costs a Sigma round trip and
    // a ramp), the pressure epochs and short runs on the one-instance kernel
    const bool pair_ok = pair_eligible(h);
    if (!pair_ok) {
      const uwvk_status st = launch_seg(e, last, false);
      if (st != UWVK_OK) return st;
    } else {
      constexpr int64_t kPairMinRun = 48;
      int64_t s0 = e;  // start of the pending one-instance segment
      int64_t k = e;
      while (k < last) {
        if (hf[k - first] & UWVK_EV_PRESSURE) { k++; continue; }
        int64_t q = k;  // a run of epochs without pressure: [k, q)
        while (q < last && !(hf[q - first] & UWVK_EV_PRESSURE)) q++;
        if (q - k >= kPairMinRun || (k == e && q == last)) {
          if (k > s0) {
            const uwvk_status st = launch_seg(s0, k, false);
            if (st != UWVK_OK) return st;
          }
          const uwvk_status st = launch_seg(k, q, true);
          if (st != UWVK_OK) return st;
          s0 = q;
        }
        k = q;
      }
      if (last > s0) {
        const uwvk_status st = launch_seg(s0, last, false);
        if (st != UWVK_OK) return st;
      }
    }
    if (r < first + count) {
      ea.first = r;
      ea.count = 1;
      ea.efforts_only = 0;
      // constrainVelocity (PEffVO) or the full measurementEfforts (psp_update_eff)
      const int vo = (hf[r - first] & UWVK_EV_EFFORTS_VELOCITY_ONLY) ? 1 : 0;
      if (!vo) h->pdec = false;  // the full model couples the parameters (PD off from here)
      HIPCHK(launch_psp_efforts(h->dof, vo, h->stream, b, sh, ea));
    }
    e = last;
  }
  return UWVK_OK;
}

uwvk_status uwvk_pose_ensemble_stats(uwvk_pose* h, const double* truth, double* out) {
  UWVK_DEVICE_GUARD(h);
  return uwvk_pose_ensemble_allreduce(h, truth, out, nullptr);
}

uwvk_status uwvk_pose_ensemble_allreduce(uwvk_pose* h, const double* truth, double* out, void* comm) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !out) return UWVK_EINVAL;
  const int s = h->store;
  const int nout = 3 * s + 2;
  double* d_out = h->d_scratch;
  StatTruth t{};  // by value in the kernel arguments: no upload in front of the kernel
  if (truth) std::memcpy(t.v, truth, s * 8);
  else t.v[3] = 1.0;
  t.right = h->sh.so3_right;
  // ensemble partials after the rotation-rate area: d_scratch + 256 + 3 batch
  double* d_part = h->d_scratch + 256 + 3 * h->batch;
  PoseBufs b = bufs(h);
  HIPCHK(launch_pose_stats(h->dof, h->stream, b, t, d_out, d_part));
  if (comm) {  // RCCL sum across the ranks' shards, stream-ordered after the stats kernel
    const uwvk_status st = uwvk_comm_allreduce_sum_device(comm, d_out, nout, (void*)h->stream);
    if (st != UWVK_OK) return st;
  }
  HIPCHK(hipMemcpyAsync(out, d_out, nout * 8, hipMemcpyDeviceToHost, h->stream));
  HIPCHK(hipStreamSynchronize(h->stream));
  return UWVK_OK;
}

uwvk_status uwvk_pose_set_option(uwvk_pose* h, int option, int value) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  if (option == UWVK_OPT_LITERAL_APPLY_DELTA) {
    h->sh.literal_apply_delta = value ? 1 : 0;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_DENSE_SIGMA) {
    h->dense = value ? 1 : 0;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_TAIL_SLOTS) {
    h->tail_slots = value;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_SO3_RIGHT) {
    h->sh.so3_right = value ? 1 : 0;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_TAIL_CHUNKS) {
    if (value < 0 || value > 8) return UWVK_EINVAL;
    h->tail_force = value;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_PERSIST) {
    h->persist = value ? 1 : 0;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_LDS_PAD) {  // diagnostic: occupancy sweep of the epoch kernel
    // the pad plus the kernel's static PspSmem<53> must fit gfx950's 160 KiB
    if (value < 0 || value > 160 * 1024 - (int)psp_epoch_lds_bytes(53)) return UWVK_EINVAL;
    h->lds_pad = (uint32_t)value;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_WAIT_BOUND) {  // tests: force hand-off timeouts (0 = every one)
    h->wait_bound = value;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_PARAM_BLOCK) {
    h->pd_opt = value ? 1 : 0;
    return UWVK_OK;
  }
  if (option == UWVK_OPT_PAIR) {
    h->pair_opt = value ? 1 : 0;
    return UWVK_OK;
  }
  return UWVK_EINVAL;
}

int64_t uwvk_pose_resident_slots(int dof, int device) {
  if (dof != 53 && dof != 26) return 0;
  return psp_epoch_slots_per_xcd(dof, device);
}

int uwvk_pose_param_block(uwvk_pose* h) {
  if (!h) return 0;
  // q_simple is refreshed by upload_shared; evaluate it on the current Q
  return (h->pd_opt && h->pdec && h->dof == 53 && q_is_simple(h) && q_params_diag(h)) ? 1 : 0;
}

int uwvk_pose_pair_active(uwvk_pose* h) { return (h && pair_eligible(h)) ? 1 : 0; }

int uwvk_xcd_round_robin(int device) { return xcd_round_robin(device); }

int uwvk_pose_epoch_qshape(const uwvk_pose* h) { return h ? (q_is_simple(h) ? 1 : 2) : 0; }

int uwvk_pose_tail_chunks(int64_t instances_per_xcd, int64_t slots_per_xcd, int64_t epochs) {
  return plan_tail(instances_per_xcd, slots_per_xcd, epochs);
}

uwvk_status uwvk_pose_timer_start(uwvk_pose* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  HIPCHK(hipEventRecord(h->ev0, h->stream));
  return UWVK_OK;
}
uwvk_status uwvk_pose_timer_stop(uwvk_pose* h, float* ms) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !ms) return UWVK_EINVAL;
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  HIPCHK(hipEventSynchronize(h->ev1));
  HIPCHK(hipEventElapsedTime(ms, h->ev0, h->ev1));
  return UWVK_OK;
}
uwvk_status uwvk_pose_timer_mark(uwvk_pose* h) {
  UWVK_DEVICE_GUARD(h);
  if (!h) return UWVK_EINVAL;
  HIPCHK(hipEventRecord(h->ev1, h->stream));
  return UWVK_OK;
}
uwvk_status uwvk_pose_timer_elapsed(uwvk_pose* h, float* ms) {
  UWVK_DEVICE_GUARD(h);
  if (!h || !ms) return UWVK_EINVAL;
  HIPCHK(hipEventSynchronize(h->ev1));
  HIPCHK(hipEventElapsedTime(ms, h->ev0, h->ev1));
  return UWVK_OK;
}

}  // extern "C"
