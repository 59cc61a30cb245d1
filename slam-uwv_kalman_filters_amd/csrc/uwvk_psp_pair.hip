// uwvk_psp_pair.hip — the parameter-decoupled PSP epoch kernel with TWO
// instances per wave (r06).
//
// The parameter-decoupled kernel (uwvk_psp_dev.hpp PspSmemPD) runs a 53-DOF
// instance on the 26-DOF layout: its row phases use 26 of 64 lanes and its
// sigma-point phases 31 (predict) or 13 (update).  Every phase fits 32 lanes,
// so here instance h = lane >> 5 of a wave owns lanes [32 h, 32 h + 32) and its
// own PspSmemPD: one wave instruction serves both instances.  The PSP routines
// are the same source compiled with PSP_PAIR = 1 (namespace psp2): lane masks
// on the 32 local lanes of both halves, per-half broadcasts (hread) and sums,
// and Sigma~ -= C~ K~^T as a lane-per-row FMA sweep instead of the MFMA tile
// (one v_mfma_f64_16x16x4 spans 64 lanes).  A work unit is a PAIR of
// instances (2u, 2u + 1) over an epoch range: the persistent scheduler, tail
// chunks and their hand-offs work on pair units exactly as k_psp_epoch_p on
// instances.  The arithmetic per instance is the single kernel's except for the
// rank-M update's summation order (FMA chain per entry instead of the MFMA's).
#define PSP_PAIR 1
#define PSP_NS psp2
// waves per SIMD of the pair kernel (PSP_PAIR_WAVES=... for occupancy A/Bs)
#ifndef PSP_PAIR_WAVES
#define PSP_PAIR_WAVES 3
#endif
#include <algorithm>
#include <atomic>

#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"
#include "uwvk_psp_dev.hpp"
#include "uwvk_psp.hpp"

namespace uwvk {
namespace psp2 {

// instance h of the wave's pair
UWVK_DEV int half() { return (int)(threadIdx.x >> 5) & 1; }

// ---- scheduling (as uwvk_psp_k.hip's persistent kernel, on pair units) ----
struct PUnit {
  int64_t unit, e0, e1, tslot;
  int chunk;  // >= 0: a chunk of a tail unit
};
UWVK_DEV PUnit ticket_unit(const EpochArgs& ea, uint32_t u) {
  PUnit t{(int64_t)u, ea.first, ea.first + ea.count, 0, -1};
  if (ea.chunks > 1 && (int64_t)u >= ea.tail0) {
    const uint32_t q = u - (uint32_t)ea.tail0, m = (uint32_t)ea.r_x;
    const uint32_t k = q / m, r = q - k * m;
    t.unit = ea.tail0 + r;
    t.chunk = (int)k;
    t.tslot = r;
    t.e0 = ea.first + ea.count * k / ea.chunks;
    t.e1 = ea.first + ea.count * (k + 1) / ea.chunks;
  }
  return t;
}
UWVK_DEV uint32_t ticket_issue(const EpochArgs& ea) {
  uint32_t v = 0;
  if (lane_id() == 0) v = __hip_atomic_fetch_add(ea.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}
UWVK_DEV uint32_t ticket_value(const EpochArgs& ea, uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v) - ea.ticket_base;
}
// predecessor chunk's hand-off (see uwvk_psp_k.hip tail_wait_t)
UWVK_DEV bool tail_wait(uint32_t* f, uint32_t want, uint32_t bound) {
  uint32_t n = 0;
  if (lane_id() == 0) {
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want && ++n < bound)
      __builtin_amdgcn_s_sleep(64);
  }
  n = __builtin_amdgcn_readfirstlane(n);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return n < bound;
}
UWVK_DEV void tail_signal(const EpochArgs& ea, int64_t t, int chunk) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_wave_barrier();
  if (lane_id() == 0)
    __hip_atomic_store(ea.tail_flag + t, ea.tag * 16u + (uint32_t)(chunk + 1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// ---- the parameter-decoupled state through the 26-DOF layout (uwvk_psp_k.hip's, per half) ----
UWVK_DEV int pd_pidx(int e) {
  int i = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if (((i + 1) * (i + 2)) / 2 <= e) i++;
  if ((i * (i + 1)) / 2 > e) i--;
  const int j = e - (i * (i + 1)) / 2;
  const int I = pd_dof(i), J = pd_dof(j);
  return (I * (I + 1)) / 2 + J;
}
UWVK_DEV constexpr int pd_diag53(int t) { return ((19 + t) * (20 + t)) / 2 + 19 + t; }

// per-lane process-model constants of the 26-DOF layout (uwvk_psp_k.hip
// lane_proc<26>), s = the local lane
UWVK_DEV void lane_proc(const PoseBufs& b, const PoseShared& sh, int64_t inst, int s, ProcCtx& pc) {
  using L = Lay<26>;
  const uwvk_pose_parameter& P = sh.p;
  pc.vpart = s < 3 ? L::s_vel + s : ((s >= L::s_vel && s < L::s_vel + 3) ? L::s_acc + s - L::s_vel : -1);
  pc.nt_lane = 0.0;
  pc.off_lane = 0.0;
  int k = -1;
  if (s >= L::s_bg && s < L::s_bg + 3) { pc.nt_lane = sh.ntau[0]; pc.off_lane = P.gyro_bias_offset[s - L::s_bg]; }
  if (s >= L::s_ba && s < L::s_ba + 3) { pc.nt_lane = sh.ntau[1]; pc.off_lane = P.acc_bias_offset[s - L::s_ba]; }
  if (s >= L::s_wv && s < L::s_wv + 4) pc.nt_lane = sh.ntau[5];
  if (s >= L::s_badcp && s < L::s_badcp + 2) pc.nt_lane = sh.ntau[6];
  if (s == L::s_rho) { k = 27; pc.nt_lane = sh.ntau[7]; }
  if (k >= 0) pc.off_lane = b.off[inst * 28 + k];
  pc.nt_tan = 0.0;
  if (s < 26 && scaled_dof(s)) pc.nt_tan = tan_ntau_sel<26>(s, sh);
}

// The 27 model parameters of the pair layout: local lane t < 27 owns parameter
// t's plain Sigma_ii (no time scale: Sigma_ii <- A_ii^2 Sigma_ii + dt^2 Q_ii,
// the process model's A_ii = 1 + dt (-1/tau), PoseUKF.cpp:50-72 / :460) and
// its mean (decay toward the offset), in the instance's PspSmemPD (pS, pm).
// Only lane t touches entry t: no ordering with the other phases.
struct ParLane {
  double q;    // dt^2 Q_ii (the PD table's entry 351 + t)
  double off;  // the mean's offset
  double nt;   // -1/tau of its block
};
UWVK_DEV ParLane par_lane(const PoseBufs& b, const PoseShared& sh, int64_t inst, int t) {
  ParLane p{0.0, 0.0, 0.0};
  if (t < kPdN) {
    p.q = reinterpret_cast<const double2*>(b.Qp)[PG<26>::NP + t].y;
    p.off = b.off[inst * 28 + t];
    p.nt = t < 9 ? sh.ntau[2] : (t < 18 ? sh.ntau[3] : sh.ntau[4]);
  }
  return p;
}
UWVK_DEV void par_epoch(double* px, int t, double dt, const ParLane& p) {
  if (t < kPdN) {
    const double a = 1.0 + dt * p.nt;
    const double v = px[t], m = px[32 + t];
    px[t] = a * (a * v) + p.q;
    px[32 + t] = m + dt * (p.nt * (m - p.off));  // proc_vect_lane's expression
  }
}

// the pair's state through the 26-DOF layout: instance inst's Sigma~ subset,
// 27 stored means, the parameters' diagonal and means (local lanes, 32 per instance)
UWVK_DEV void load_pair(PspSmem<26>& sm, double* px, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  const double* gs = b.sigma + inst * (int64_t)PG<53>::NP;
  const double* gm = b.mu + inst * (int64_t)Lay<53>::store;
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    v[t] = e < G::NP ? gs[pd_pidx(e)] : 0.0;
  }
  const double m = l < Lay<26>::store ? gm[pd_store(l)] : 0.0;
  const bool pl = l < kPdN;
  const double ps = pl ? gs[pd_diag53(l)] : 0.0, pm = pl ? gm[20 + l] : 0.0;
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    if (e < G::NP) sm.S[e] = v[t];
  }
  if (l < Lay<26>::store) sm.mu[l] = m;
  if (pl) {
    px[l] = ps;
    px[32 + l] = pm;
  }
  psync();
}
UWVK_DEV void store_pair(const PspSmem<26>& sm, const double* px, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  double* gs = b.sigma + inst * (int64_t)PG<53>::NP;
  double* gm = b.mu + inst * (int64_t)Lay<53>::store;
  static_assert(G::NSLOT * kLanes <= G::NP + Lay<26>::store + PG<26>::STG, "slot over-read stays in PspSmem");
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) v[t] = flat(sm)[l + kLanes * t];
  const double m = flat(sm)[kFlatMu<26> + l];
  const bool pl = l < kPdN;
  const double ps = px[l], pm = px[32 + l];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    if (e < G::NP) gs[pd_pidx(e)] = v[t];
  }
  if (l < Lay<26>::store) gm[pd_store(l)] = m;
  if (pl) {
    gs[pd_diag53(l)] = ps;
    gm[20 + l] = pm;
  }
}

// a 26-DOF handle's own state (PD = 0): the packed 26-DOF triangle and mean
// (uwvk_psp_k.hip load_psp<26> / store_psp<26>, on 32 lanes per instance)
UWVK_DEV void load_pair26(PspSmem<26>& sm, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  const double* gs = b.sigma + inst * (int64_t)G::NP;
  const double* gm = b.mu + inst * (int64_t)Lay<26>::store;
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    v[t] = e < G::NP ? gs[e] : 0.0;
  }
  const double m = l < Lay<26>::store ? gm[l] : 0.0;
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    if (e < G::NP) sm.S[e] = v[t];
  }
  if (l < Lay<26>::store) sm.mu[l] = m;
  psync();
}
UWVK_DEV void store_pair26(const PspSmem<26>& sm, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  double* gs = b.sigma + inst * (int64_t)G::NP;
  double* gm = b.mu + inst * (int64_t)Lay<26>::store;
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) v[t] = flat(sm)[l + kLanes * t];
  const double m = flat(sm)[kFlatMu<26> + l];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + kLanes * t;
    if (e < G::NP) gs[e] = v[t];
  }
  if (l < Lay<26>::store) gm[l] = m;
}

template <int M>
UWVK_DEV void copy_zr(const double* zin, const double* Rin, double (&z)[M], double (&R)[M * M]) {
#pragma unroll
  for (int k = 0; k < M; k++) z[k] = zin[k];
#pragma unroll
  for (int k = 0; k < M * M; k++) R[k] = Rin[k];
}
UWVK_DEV bool finite_n(const double* a, int n) {
  bool ok = true;
  for (int i = 0; i < n; i++) ok = ok && __builtin_isfinite(a[i]);
  return ok;
}
UWVK_DEV const PoseShared& shared_for_epoch(const PoseBufs& b) {
  using CP = const __attribute__((address_space(4))) PoseShared*;
  CP p = (CP)b.shared;
  asm volatile("" : "+s"(p));
  return *(const PoseShared*)p;
}

// The pair kernel's persistent work loop: block b runs pair unit b first, then
// takes units from the ticket counter (k_psp_epoch_p's scheme); unit u is
// instances 2u (lanes 0..31) and 2u + 1 (lanes 32..63).
// Launches without pressure epochs only (EpochArgs flags host-checked): the
// pressure update's nonlinear prefix is k = 19 (pos .. gravity;
// PoseUKF.cpp:107-115), 39 sigma points, more than a half-wave holds; run_log
// runs those epochs on the one-instance PD kernel.  EVS = 1: no ADCP epoch in
// the launch either (the ADCP update, k = 6, not compiled in).
// PD = 1: a 53-DOF handle's parameter-decoupled state (NW = 53, the 27
// parameters in pS / pm); PD = 0 (r06): a 26-DOF kinematic handle's own state
// (NW = 26, no parameter lanes).
template <int SR, int EVS, int PD>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PSP_PAIR_WAVES, PSP_PAIR_WAVES)))
void k_psp_epoch_pair(PoseBufs b, PoseShared sh0, EpochArgs ea) {
  __shared__ PspSmemPD<26> smx[2];
  const int h = half();
  PspSmem<26>& sm = smx[h];
  double* const px = smx[h].pS;
  constexpr int NW = PD ? 53 : 26;
  const int64_t B = b.batch;
  const uint32_t grid = gridDim.x;
  uint32_t u = blockIdx.x;
#pragma unroll 1
  while (u < ea.units) {
    const PUnit tu = ticket_unit(ea, u);
    if (tu.chunk > 0 && !tail_wait(ea.tail_flag + tu.tslot, ea.tag * 16u + (uint32_t)tu.chunk, ea.wait_bound)) {
      if ((threadIdx.x & 31) == 0) {
        __hip_atomic_fetch_or(b.status + 2 * tu.unit + h, UWVK_ST_SCHEDULE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ea.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-mapped word
      }
      u = grid + ticket_value(ea, ticket_issue(ea));
      psync();
      continue;
    }
    const int l = olane();
    const int64_t inst = 2 * tu.unit + h;
    const int64_t e_begin = tu.e0, e_end = tu.e1;
    bool ok = true, nan = false;
    uint32_t cnt[4] = {0, 0, 0, 0};
    ProcCtx pc;
    for (int k = 0; k < 3; k++) pc.w[k] = b.rot[inst * 3 + k];
    {
      double dtv = ea.dt;
      asm volatile("" : "+v"(dtv));
      pc.dt = dtv;
    }
    pc.off = nullptr;
    lane_proc(b, *b.shared, inst, l, pc);
    const ParLane pl = PD ? par_lane(b, *b.shared, inst, l) : ParLane{0.0, 0.0, 0.0};
    const LaneQ lq = lane_q<26, 0>(b.Qp, l);
    uint32_t fl_n = 0;
    double g_n[3] = {0, 0, 0}, a_n[3] = {0, 0, 0};
    auto fetch = [&](int64_t e) {
      fl_n = ea.flags[e];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        g_n[k] = ea.gyro[(e * B + inst) * 3 + k];
        a_n[k] = ea.acc[(e * B + inst) * 3 + k];
      }
    };
    if (e_end > e_begin) fetch(e_begin);
    if constexpr (PD) load_pair(sm, px, b, inst, l);
    else load_pair26(sm, b, inst, l);
    double ds = 1.0, ids = 1.0;  // time scale of the 26-DOF layout's Markov DOFs
    if (tu.chunk > 0) {
      const double2 c = reinterpret_cast<const double2*>(ea.tail_carry)[tu.tslot * 64 + lane_id()];
      ds = c.x;
      ids = c.y;
    }
    uint32_t vn = ticket_issue(ea);  // the next unit's ticket, claimed early
#pragma unroll 1
    for (int64_t e = e_begin; e < e_end; e++) {
      const uint32_t fl = fl_n;
      const double g[3] = {g_n[0], g_n[1], g_n[2]}, za[3] = {a_n[0], a_n[1], a_n[2]};
      if (e + 1 < e_end) fetch(e + 1);
      if (finite_n(g, 3)) {
        for (int k = 0; k < 3; k++) pc.w[k] = g[k];
      } else {
        nan = true;
      }
      const PoseShared& sh = shared_for_epoch(b);
      if (((e - ea.first) & 1023) == 1023) psp_fold<26, 0>(sm, ds, ids);
      bool sok = psp_predict<26, 1, SR, PD>(sm, sh, pc, b.Q, b.Qp, ds, ids, lq, nullptr, px);
      if constexpr (PD) par_epoch(px, l, pc.dt, pl);
      ok = ok && sok;
      if (fl & UWVK_EV_ACC) {
        if (finite_n(za, 3)) {
          double z[3], R[9];
          copy_zr<3>(za, sh.log_acc_cov, z, R);
          psp_update<26, SR, PAcc<26>, NW>(sm, z, R, 0, PAcc<26>{}, &sok, ds, ids);
          ok = ok && sok;
        } else {
          nan = true;
        }
      }
      if (fl & UWVK_EV_DVL) {
        const double* zp = ea.dvl + ((int64_t)ea.dvl_index[e] * B + inst) * 3;
        if (finite_n(zp, 3)) {
          double z[3], R[9];
          copy_zr<3>(zp, sh.log_dvl_cov, z, R);
          cnt[0] += psp_update<26, SR, PVel<26>, NW>(sm, z, R, 0, PVel<26>{}, &sok, ds, ids);
          ok = ok && sok;
        } else {
          nan = true;
        }
      }
      if constexpr (EVS == 0) {
        if (fl & UWVK_EV_ADCP) {  // measurementWaterCurrents per cell (PoseUKF.cpp:133-151, :514-527)
          for (int c = 0; c < ea.cells; c++) {
            const double* zp = ea.adcp + (((int64_t)ea.a_index[e] * ea.cells + c) * B + inst) * 2;
            if (!finite_n(zp, 2)) {
              nan = true;
              continue;
            }
            double z[2] = {zp[0], zp[1]}, R[4] = {ea.adcp_cov[0], ea.adcp_cov[1], ea.adcp_cov[2], ea.adcp_cov[3]};
            PWater<26> hw;
            hw.cw = ea.cw[c];
            cnt[2] += psp_update<26, SR, PWater<26>, NW>(sm, z, R, 1, hw, &sok, ds, ids);
            ok = ok && sok;
          }
        }
      }
    }
    if (l == 0) {  // local lane 0 of each half: its instance's bookkeeping
      const uint32_t bits = (ok ? 0u : UWVK_ST_NOTPD) | (nan ? UWVK_ST_NAN : 0u);
      if (bits) __hip_atomic_fetch_or(b.status + inst, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e_end > e_begin) {
        b.rot[inst * 3] = pc.w[0]; b.rot[inst * 3 + 1] = pc.w[1]; b.rot[inst * 3 + 2] = pc.w[2];
      }
      if (ea.accept_counts)
        for (int k = 0; k < 4; k++) ea.accept_counts[inst * 4 + k] += cnt[k];
    }
    const uint32_t un = grid + ticket_value(ea, vn);
    const PUnit tn = ticket_unit(ea, u);  // re-derived: not kept live through the epochs
    const bool hand = tn.chunk >= 0 && tn.chunk + 1 < ea.chunks;
    if (hand) {  // hand on: Sigma~ and d unfolded (both halves' 64 lanes)
      double* c = ea.tail_carry + (tn.tslot * 64 + lane_id()) * 2;
      c[0] = ds;
      c[1] = ids;
      psync();
    } else {
      psp_fold<26, 0>(sm, ds, ids);
    }
    if constexpr (PD) store_pair(sm, px, b, inst, l);
    else store_pair26(sm, b, inst, l);
    if (hand) tail_signal(ea, tn.tslot, tn.chunk);
    u = un;
    psync();  // the next unit's LDS writes after this unit's reads
  }
}

}  // namespace psp2

template <int SR, int PD>
static hipError_t launch_pair_sr(hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                                 int64_t grid, uint32_t ev_any) {
  const dim3 g((unsigned)grid), t(64);
  if (ev_any & UWVK_EV_PRESSURE) return hipErrorInvalidValue;  // (run_log splits those epochs off)
  if (ev_any & UWVK_EV_ADCP) hipLaunchKernelGGL((psp2::k_psp_epoch_pair<SR, 0, PD>), g, t, 0, st, b, sh, ea);
  else hipLaunchKernelGGL((psp2::k_psp_epoch_pair<SR, 1, PD>), g, t, 0, st, b, sh, ea);
  return hipGetLastError();
}

hipError_t launch_psp_epoch_pair(hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                                 int64_t grid, uint32_t ev_any, int pd) {
  if (!sh.q_simple || !ea.ticket || grid <= 0) return hipErrorInvalidValue;
  if (pd) return sh.so3_right ? launch_pair_sr<1, 1>(st, b, sh, ea, grid, ev_any)
                              : launch_pair_sr<0, 1>(st, b, sh, ea, grid, ev_any);
  return sh.so3_right ? launch_pair_sr<1, 0>(st, b, sh, ea, grid, ev_any)
                      : launch_pair_sr<0, 0>(st, b, sh, ea, grid, ev_any);
}

int64_t psp_pair_slots(int device) {
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)psp2::k_psp_epoch_pair<1, 1, 1>, 64, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return (int64_t)per_cu * cus;
}

}  // namespace uwvk
