// uwvk_psp_k.hip — PSP PoseUKF kernels (one wavefront per filter instance).
//
// k_psp_epoch is the hot path of uwvk_pose_run_log: each workgroup (one wave)
// loads its instance's (mu, Sigma) from HBM once, runs every epoch of the
// requested range with Sigma packed in LDS, and writes it back once:
//   RotationRate -> predictionStep(dt) -> Acceleration update
//   [-> Velocity (DVL) -> Pressure -> ADCP cells]
// The host splits a launch after each BodyEfforts epoch (this kernel runs that
// epoch's predict and other updates) and runs the efforts update alone on the
// literal k_pose_efforts_epoch, whose HBM layout is shared.  With tail
// spreading (EpochArgs::chunks > 1, plan_tail below) the last instances of
// each XCD run as a few epoch chunks, one block each, handed on in order.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

// PSP_SIDE: the SO3 side this translation unit instantiates the kernels for
// (0 here; uwvk_psp_k_r.hip includes this file with 1).  The two sides are
// separate objects so the build parallelises; the host dispatchers, the
// placement probe and the occupancy helpers live in the side-0 object.
#ifndef PSP_SIDE
#define PSP_SIDE 0
#endif

#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"
#include "uwvk_psp_dev.hpp"
#include "uwvk_psp.hpp"


namespace uwvk {
namespace psp {

#ifdef UWVK_TIMELINE
// diagnostic build only (tools/timeline.py): per-wave wall-clock marks of the
// epoch kernel (entry, Sigma loaded, epochs done, stored) and the CU it ran on
static __device__ unsigned long long uwvk_timeline[8 * 131072];  // per side's translation unit
UWVK_DEV void tl_mark(int64_t w, int k) {
  const unsigned long long t = wall_clock64();
  if (lane_id() == 0 && w < 131072) uwvk_timeline[w * 8 + k] = t;
}
#endif

// tail-chunk hand-off (EpochArgs::chunks > 1).  Chunk k of a tail instance is
// placed later in its XCD's block order than chunk k - 1 (plan_tail), and
// blocks are dispatched in order, so the block waited for is resident or done:
// the wait cannot deadlock.  The host enables spreading only after
// xcd_round_robin() has seen, on this device, that block b runs on XCC b % 8
// (the hardware XCC_ID register), the placement the plan relies on.
struct TailUnit {
  int64_t inst, e0, e1, tslot;
  int chunk;  // >= 0: a chunk of a tail instance
};
UWVK_DEV TailUnit tail_unit(const EpochArgs& ea, int64_t B) {
  TailUnit u{xcd_instance(B), ea.first, ea.first + ea.count, 0, -1};
  if (ea.chunks > 1) {
    const int64_t x = blockIdx.x & 7, i = blockIdx.x >> 3;
    if (i < ea.tail0) {
      u.inst = x * ea.n_x + i;
    } else {
      const uint32_t q = (uint32_t)(i - ea.tail0), m = (uint32_t)ea.r_x;
      const uint32_t k = q / m, t = q - k * m;
      u.inst = x * ea.n_x + ea.tail0 + t;
      u.chunk = (int)k;
      u.tslot = x * ea.r_x + t;
      u.e0 = ea.first + ea.count * k / ea.chunks;
      u.e1 = ea.first + ea.count * (k + 1) / ea.chunks;
    }
  }
  return u;
}

// Waits for the predecessor chunk's signal.  The bound (ea.wait_bound sleeps
// of ~1.7 us, scaled by the host with the launch's epoch count) only keeps a
// broken ordering from hanging the device: past it the instance is flagged
// UWVK_ST_SCHEDULE and false is returned, and the caller skips the whole chunk
// (no load, no epochs, no store, no signal), so nothing races the late
// predecessor; every later chunk of the instance then times out the same way.
// (scalar arguments: with the EpochArgs reference the caller kept a copy of
// the kernel arguments in scratch, 150 -> 173 VGPRs and 800 B/lane)
template <bool INL>
UWVK_DEV bool tail_wait_t(uint32_t* f, uint32_t want, uint32_t bound) {
  uint32_t n = 0;
  if (lane_id() == 0) {
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want && ++n < bound)
      __builtin_amdgcn_s_sleep(64);
  }
  n = __builtin_amdgcn_readfirstlane(n);  // lane 0's count, wave-uniform
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the previous chunk's stores, from any CU
  return n < bound;
}
__device__ __attribute__((noinline)) bool tail_wait(uint32_t* f, uint32_t want, uint32_t bound) {
  return tail_wait_t<false>(f, want, bound);
}
__device__ __attribute__((noinline)) double2 tail_carry_in(const EpochArgs& ea, int64_t t) {
  return reinterpret_cast<const double2*>(ea.tail_carry)[t * 64 + lane_id()];
}
UWVK_DEV void tail_signal(const EpochArgs& ea, int64_t t, int chunk) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // every lane's Sigma~ / mu / carry / rot stores first
  __builtin_amdgcn_wave_barrier();
  if (lane_id() == 0)
    __hip_atomic_store(ea.tail_flag + t, ea.tag * 16u + (uint32_t)(chunk + 1), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}


template <int DOF>
UWVK_DEV void load_psp(PspSmem<DOF>& sm, const PoseBufs& b, int64_t inst, int l = lane_id()) {
  using G = PG<DOF>;
  const double* gs = b.sigma + inst * (int64_t)G::NP;  // packed in HBM as in LDS: one coalesced copy
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {  // all loads in flight before the LDS stores
    const int e = l + 64 * t;
    v[t] = e < G::NP ? gs[e] : 0.0;
  }
  const double m = l < Lay<DOF>::store ? b.mu[inst * Lay<DOF>::store + l] : 0.0;
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + 64 * t;
    if (e < G::NP) sm.S[e] = v[t];
  }
  if (l < Lay<DOF>::store) sm.mu[l] = m;
  psync();
}

// per-lane process-model constants of storage component s (PoseUKF.cpp:24-79):
// the state it integrates (pos <- vel, vel <- acc), or its Markov decay -1/tau
// and the offset it decays towards
template <int DOF, int PD = 0>
UWVK_DEV void lane_proc(const PoseBufs& b, const PoseShared& sh, int64_t inst, int s, ProcCtx& pc) {
  using L = Lay<DOF>;
  const uwvk_pose_parameter& P = sh.p;
  pc.vpart = s < 3 ? L::s_vel + s : ((s >= L::s_vel && s < L::s_vel + 3) ? L::s_acc + s - L::s_vel : -1);
  pc.nt_lane = 0.0;
  pc.off_lane = 0.0;
  int k = -1;
  if (s >= L::s_bg && s < L::s_bg + 3) { pc.nt_lane = sh.ntau[0]; pc.off_lane = P.gyro_bias_offset[s - L::s_bg]; }
  if (s >= L::s_ba && s < L::s_ba + 3) { pc.nt_lane = sh.ntau[1]; pc.off_lane = P.acc_bias_offset[s - L::s_ba]; }
  if constexpr (L::has_params) {
    if (s >= L::s_inertia && s < L::s_inertia + 9) { k = s - L::s_inertia; pc.nt_lane = sh.ntau[2]; }
    if (s >= L::s_lin && s < L::s_lin + 9) { k = 9 + s - L::s_lin; pc.nt_lane = sh.ntau[3]; }
    if (s >= L::s_quad && s < L::s_quad + 9) { k = 18 + s - L::s_quad; pc.nt_lane = sh.ntau[4]; }
  }
  if (s >= L::s_wv && s < L::s_wv + 4) pc.nt_lane = sh.ntau[5];
  if (s >= L::s_badcp && s < L::s_badcp + 2) pc.nt_lane = sh.ntau[6];
  if (s == L::s_rho) { k = 27; pc.nt_lane = sh.ntau[7]; }
  if (k >= 0) pc.off_lane = b.off[inst * 28 + k];
  // tangent DOF `s` (the lane): its decay rate when it is time-scaled, so that
  // A_ll = 1 + dt nt_tan is one FMA per predict (0 keeps A_ll = 1 exactly)
  pc.nt_tan = 0.0;
  if (s < DOF && scaled_dof(s)) pc.nt_tan = tan_ntau_sel<DOF>(s, sh);
  if constexpr (PD) {
    // parameter t = s - 27 of the 53-DOF state (inertia, lin / quad damping,
    // 9 each, column-major): its mean's decay rate and offset, and the same
    // rate for its tangent DOF's time scale (the 53-DOF kernel's lanes 20 + t
    // and 19 + t hold the same values)
    if (s >= kPdLane0 && s < kPdLane0 + kPdN) {
      const int t = s - kPdLane0;
      const double nt = t < 9 ? sh.ntau[2] : (t < 18 ? sh.ntau[3] : sh.ntau[4]);
      pc.vpart = -1;
      pc.nt_lane = nt;
      pc.off_lane = b.off[inst * 28 + t];
      pc.nt_tan = nt;
    }
  }
}

// PD: the 53-DOF instance's HBM state through the 26-DOF layout.  Packed
// 26-layout entry e = (i, j) -> the 53-layout packed index (row / column DOF
// maps pd_dof); a float row estimate corrected by one step either way.
UWVK_DEV int pd_pidx(int e) {
  int i = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);
  if (((i + 1) * (i + 2)) / 2 <= e) i++;
  if ((i * (i + 1)) / 2 > e) i--;
  const int j = e - (i * (i + 1)) / 2;
  const int I = pd_dof(i), J = pd_dof(j);
  return (I * (I + 1)) / 2 + J;
}
UWVK_DEV constexpr int pd_diag53(int t) { return ((19 + t) * (20 + t)) / 2 + 19 + t; }  // parameter t's (i, i)

// the PD kernel's load: Sigma~'s 26-DOF subset, the mean's 27 stored values,
// the parameters' diagonal and means (lanes 27..53) into LDS
UWVK_DEV void load_psp_pd(PspSmem<26>& sm, double* px, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  const double* gs = b.sigma + inst * (int64_t)PG<53>::NP;
  const double* gm = b.mu + inst * (int64_t)Lay<53>::store;
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + 64 * t;
    v[t] = e < G::NP ? gs[pd_pidx(e)] : 0.0;
  }
  const double m = l < Lay<26>::store ? gm[pd_store(l)] : 0.0;
  const bool pl = l >= kPdLane0 && l < kPdLane0 + kPdN;
  const int tp = pl ? l - kPdLane0 : 0;
  const double ps = pl ? gs[pd_diag53(tp)] : 0.0, pm = pl ? gm[20 + tp] : 0.0;
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + 64 * t;
    if (e < G::NP) sm.S[e] = v[t];
  }
  if (l < Lay<26>::store) sm.mu[l] = m;
  if (pl) {
    px[tp] = ps;
    px[32 + tp] = pm;
  }
  psync();
}

// the PD kernel's store: the same entries back (the parameters' off-diagonal
// zeros are never written)
UWVK_DEV void store_psp_pd(const PspSmem<26>& sm, const double* px, const PoseBufs& b, int64_t inst, int l) {
  using G = PG<26>;
  double* gs = b.sigma + inst * (int64_t)PG<53>::NP;
  double* gm = b.mu + inst * (int64_t)Lay<53>::store;
  double v[G::NSLOT];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) v[t] = flat(sm)[l + 64 * t];  // S at offset 0 (over-reads stay in PspSmem)
  const double m = flat(sm)[kFlatMu<26> + (l & 63)];
  const bool pl = l >= kPdLane0 && l < kPdLane0 + kPdN;
  const int tp = (l - kPdLane0) & 31;
  const double ps = px[tp], pm = px[32 + tp];
#pragma unroll
  for (int t = 0; t < G::NSLOT; t++) {
    const int e = l + 64 * t;
    if (e < G::NP) gs[pd_pidx(e)] = v[t];
  }
  if (l < Lay<26>::store) gm[pd_store(l)] = m;
  if (pl) {
    gs[pd_diag53(tp)] = ps;
    gm[20 + tp] = pm;
  }
}

template <int DOF>
UWVK_DEV void store_psp(const PspSmem<DOF>& sm, const PoseBufs& b, int64_t inst, int l = lane_id()) {
  using G = PG<DOF>;
  double* gs = b.sigma + inst * (int64_t)G::NP;
  // (r04) every slot's LDS read first (the last, partial slot's lanes past the
  // triangle read the mean / staging area behind it, never stored), then the
  // coalesced stores: the masked form waited for each read inside its branch
  // in groups of SG slots (all of them at once held 30 more VGPRs at the
  // epilogue: 178, 2 waves per SIMD)
  static_assert(G::NSLOT * 64 <= G::NP + Lay<DOF>::store + PG<DOF>::STG, "slot over-read stays in PspSmem");
  constexpr int SG = 6;
#pragma unroll
  for (int t0 = 0; t0 < G::NSLOT; t0 += SG) {
    double v[SG];
#pragma unroll
    for (int u = 0; u < SG; u++)
      if (t0 + u < G::NSLOT) v[u] = flat(sm)[l + 64 * (t0 + u)];  // S at offset 0
#pragma unroll
    for (int u = 0; u < SG; u++) {
      const int t = t0 + u, e = l + 64 * t;
      if (t < G::NSLOT && (t + 1 < G::NSLOT || e < G::NP)) gs[e] = v[u];
    }
  }
  const double m = flat(sm)[kFlatMu<DOF> + (l & 63)];
  if (l < Lay<DOF>::store) b.mu[inst * Lay<DOF>::store + l] = m;
}

template <int M>
UWVK_DEV void copy_zr(const double* zin, const double* Rin, double (&z)[M], double (&R)[M * M]) {
#pragma unroll
  for (int k = 0; k < M; k++) z[k] = zin[k];
#pragma unroll
  for (int k = 0; k < M * M; k++) R[k] = Rin[k];
}

// one measurement update of kind KIND on instance inst (PSP form, SO3 side SR)
// NW: the filter's n for the sigma-point weights (psp_update)
template <int DOF, int KIND, int SR, int NW = DOF>
UWVK_DEV bool do_update(PspSmem<DOF>& sm, const PoseShared& sh, int64_t inst, const double* zin, const double* Rin,
                        const MeasArgs& ma, bool* ok, double ds, double ids, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  if constexpr (KIND == MK_ACC) {
    double z[3], R[9];
    copy_zr<3>(zin, Rin, z, R);
    return psp_update<DOF, SR, PAcc<DOF>, NW>(sm, z, R, 0, PAcc<DOF>{}, ok, ds, ids, st);
  } else if constexpr (KIND == MK_VEL) {
    double z[3], R[9];
    copy_zr<3>(zin, Rin, z, R);
    return psp_update<DOF, SR, PVel<DOF>, NW>(sm, z, R, 0, PVel<DOF>{}, ok, ds, ids, st);
  } else if constexpr (KIND == MK_PRESSURE) {
    double z[1], R[1];
    copy_zr<1>(zin, Rin, z, R);
    PPressure<DOF> h;
    h.h.s[0] = ma.v3[0]; h.h.s[1] = ma.v3[1]; h.h.s[2] = ma.v3[2];
    h.h.patm = sh.p.atmospheric_pressure;
    return psp_update<DOF, SR, PPressure<DOF>, NW>(sm, z, R, 0, h, ok, ds, ids, st);
  } else if constexpr (KIND == MK_WATER) {
    double z[2], R[4];
    copy_zr<2>(zin, Rin, z, R);
    PWater<DOF> h;
    h.cw = ma.extra ? ma.extra[inst] : 0.0;
    return psp_update<DOF, SR, PWater<DOF>, NW>(sm, z, R, 1, h, ok, ds, ids, st);
  } else if constexpr (KIND == MK_XY || KIND == MK_GEO || KIND == MK_DELAYED) {
    double z[2], R[4];
    copy_zr<2>(zin, Rin, z, R);
    int gate = 0;
    if constexpr (KIND == MK_GEO) {  // PoseUKF.cpp:571-578
      double r[3];
      const double x = (zin[0] - sh.lat0) * sh.rm;
      const double y = -(zin[1] - sh.lon0) * sh.rn_cos;
      qrot(sm.mu + L::s_quat, ma.v3, r);
      z[0] = x - r[0];
      z[1] = y - r[1];
      gate = 1;
    }
    if constexpr (KIND == MK_DELAYED) {  // PoseUKF.cpp:516-521
      z[0] = zin[0] + (sm.mu[L::s_pos] - ma.extra[2 * inst]);
      z[1] = zin[1] + (sm.mu[L::s_pos + 1] - ma.extra[2 * inst + 1]);
    }
    return psp_update<DOF, SR, PXY<DOF>, NW>(sm, z, R, gate, PXY<DOF>{}, ok, ds, ids, st);
  } else {
    static_assert(KIND == MK_Z, "PSP update kind");
    double z[1], R[1];
    copy_zr<1>(zin, Rin, z, R);
    return psp_update<DOF, SR, PZ<DOF>, NW>(sm, z, R, 0, PZ<DOF>{}, ok, ds, ids, st);
  }
}

// constrainVelocity (PoseUKF.cpp:199-219, the only_affect_velocity branch of
// :581-602) in PSP form (PEffVO, k = 9): the frozen inputs at mu exactly as the
// literal kernel's do_update_efforts<DOF, 1> builds them
template <int DOF, int SR>
UWVK_DEV bool do_update_vo(PspSmem<DOF>& sm, const PoseShared& sh, const PoseBufs& b, int64_t inst,
                           const double* zin, const double* Rin, bool* ok, double ds, double ids) {
  using L = Lay<DOF>;
  double z[6], R[36];
  copy_zr<6>(zin, Rin, z, R);
  PEffVO<DOF> hm;
  HConstrain<DOF>& h = hm.h;
  h.ef.base = b.uwv;
  h.ef.weight = sh.uwv_weight;
  h.ef.buoyancy = sh.uwv_buoyancy;
  for (int k = 0; k < 3; k++) { h.ef.cog[k] = sh.cog[k]; h.ef.cob[k] = sh.cob[k]; }
  const double w[3] = {b.rot[inst * 3], b.rot[inst * 3 + 1], b.rot[inst * 3 + 2]};
  double wb[3];
  rotation_rate_body_mu<DOF>(sm.mu, sh, w, wb);  // getRotationRate() at mu (PoseUKF.cpp:588)
  h.blk.has = true;
  h.blk.v = b.model + inst * 27;  // the shared model's current blocks (A9)
  for (int k = 0; k < 3; k++) { h.wb[k] = wb[k]; h.imu[k] = sh.p.imu_in_body[k]; }
  h.w3[0] = sm.mu[L::s_wv]; h.w3[1] = sm.mu[L::s_wv + 1]; h.w3[2] = 0.0;
  for (int k = 0; k < 4; k++) h.q[k] = sm.mu[L::s_quat + k];
  double ra[3], cr[3], cc[3];
  qrot_inv(h.q, sm.mu + L::s_acc, ra);
  cross3(wb, h.imu, cr);
  cross3(wb, cr, cc);
  for (int k = 0; k < 3; k++) h.ab[k] = ra[k] - cc[k];
  return psp_update<DOF, SR>(sm, z, R, 0, hm, ok, ds, ids);
}

// measurementEfforts (PoseUKF.cpp:153-196, the full model) in PSP form
// (psp_update_eff): the inputs frozen at mu as the literal kernel's
// do_update_efforts<DOF, 0> builds them, including its side effect on the
// shared model (PoseUKF.cpp:173: the pre-update mean's parameter blocks)
template <int DOF, int SR>
UWVK_DEV bool do_update_eff(PspSmem<DOF>& sm, const PoseShared& sh, const PoseBufs& b, int64_t inst,
                            const double* zin, const double* Rin, bool* ok) {
  using L = Lay<DOF>;
  HEfforts<DOF> h;
  h.ef.base = b.uwv;
  h.ef.weight = sh.uwv_weight;
  h.ef.buoyancy = sh.uwv_buoyancy;
  for (int k = 0; k < 3; k++) { h.ef.cog[k] = sh.cog[k]; h.ef.cob[k] = sh.cob[k]; }
  const double w[3] = {b.rot[inst * 3], b.rot[inst * 3 + 1], b.rot[inst * 3 + 2]};
  double wb[3];
  rotation_rate_body_mu<DOF>(sm.mu, sh, w, wb);
  for (int k = 0; k < 3; k++) { h.wb[k] = wb[k]; h.imu[k] = sh.p.imu_in_body[k]; }
  if constexpr (L::has_params) {
    double* model = b.model + inst * 27;
    const int l = lane_id();
    if (l < 9) {
      model[l] = sm.mu[L::s_inertia + l];
      model[9 + l] = sm.mu[L::s_lin + l];
      model[18 + l] = sm.mu[L::s_quad + l];
    }
  }
  return psp_update_eff<DOF, SR>(sm, b.sigma + inst * (int64_t)PG<DOF>::NP, h, zin, Rin, ok);
}

template <int DOF, int SR>
__global__ __launch_bounds__(64) void k_psp_predict(PoseBufs b, PoseShared sh, double dt) {
  __shared__ PspSmem<DOF> sm;
  const int64_t inst = xcd_instance(b.batch);
  load_psp<DOF>(sm, b, inst);
  ProcCtx pc;
  for (int k = 0; k < 3; k++) pc.w[k] = b.rot[inst * 3 + k];
  pc.dt = dt;
  pc.off = nullptr;
  lane_proc<DOF>(b, sh, inst, lane_id(), pc);
  double ds = 1.0, ids = 1.0;
  const LaneQ lq = lane_q<DOF>(b.Qp, lane_id());
  const bool ok = psp_predict<DOF, 0, SR>(sm, sh, pc, b.Q, b.Qp, ds, ids, lq);
  if (!ok && lane_id() == 0) b.status[inst] |= UWVK_ST_NOTPD;
  psp_fold<DOF>(sm, ds, ids);
  store_psp<DOF>(sm, b, inst);
}

template <int DOF, int KIND, int SR>
__global__ __launch_bounds__(64) void k_psp_update(PoseBufs b, PoseShared sh, MeasArgs ma, int m) {
  __shared__ PspSmem<DOF> sm;
  const int64_t inst = xcd_instance(b.batch);
  if (ma.mask && !ma.mask[inst]) {
    if (ma.accepted && lane_id() == 0) ma.accepted[inst] = 0;
    return;
  }
  const double* z = ma.mu + inst * m;
  const double* R = ma.cov ? ma.cov + inst * m * m : ma.shared_cov;
  if (!all_finite(z, m) || !all_finite(R, m * m)) {  // checkMeasurment [EXT]
    if (lane_id() == 0) {
      b.status[inst] |= UWVK_ST_NAN;
      if (ma.accepted) ma.accepted[inst] = 0;
    }
    return;
  }
  load_psp<DOF>(sm, b, inst);
  bool ok = true;
  bool acc;
  if constexpr (KIND == MK_EFFORTS)
    acc = ma.only_vel ? do_update_vo<DOF, SR>(sm, sh, b, inst, z, R, &ok, 1.0, 1.0)
                      : do_update_eff<DOF, SR>(sm, sh, b, inst, z, R, &ok);
  else acc = do_update<DOF, KIND, SR>(sm, sh, inst, z, R, ma, &ok, 1.0, 1.0);
  if (lane_id() == 0) {
    if (!ok) b.status[inst] |= UWVK_ST_NOTPD;
    if (ma.accepted) ma.accepted[inst] = acc ? 1 : 0;
  }
  store_psp<DOF>(sm, b, inst);
}

// batch-shared parameters read through a pointer laundered once per epoch:
// nothing derived from them is hoisted out of the epoch loop (VGPR pressure).
// The pointer is laundered in the constant address space: laundered as a
// generic pointer, every field read became a flat_load followed by
// s_waitcnt vmcnt(0) lgkmcnt(0) (a memory round trip on the epoch's critical
// path, which also drained the input prefetch); as a constant-space pointer
// the reads are scalar loads through the scalar cache.
UWVK_DEV const PoseShared& shared_for_epoch(const PoseBufs& b) {
  using CP = const __attribute__((address_space(4))) PoseShared*;
  CP p = (CP)b.shared;
  asm volatile("" : "+s"(p));
  return *(const PoseShared*)p;
}

// Needs <= 168 VGPRs (3 waves per SIMD: with 12 instances per CU from the LDS
// budget every wave slot is used; 156 now, tools/timeline.py shows 3,072
// resident waves).  amdgpu_waves_per_eu(3) also gives 156 but schedules the
// epoch loop worse: 145.0M against 148.5M steps/s (r02 A/B), so it is not set;
// a fully unrolled Sigma store once took the kernel to 188 (2 waves per SIMD).
UWVK_DEV TailUnit ticket_unit(const EpochArgs& ea, uint32_t u) {
  TailUnit t{(int64_t)u, ea.first, ea.first + ea.count, 0, -1};
  if (ea.chunks > 1 && (int64_t)u >= ea.tail0) {
    const uint32_t q = u - (uint32_t)ea.tail0, m = (uint32_t)ea.r_x;
    const uint32_t k = q / m, r = q - k * m;
    t.inst = ea.tail0 + r;
    t.chunk = (int)k;
    t.tslot = r;
    t.e0 = ea.first + ea.count * k / ea.chunks;
    t.e1 = ea.first + ea.count * (k + 1) / ea.chunks;
  }
  return t;
}
UWVK_DEV uint32_t ticket_issue(const EpochArgs& ea) {  // lane 0's atomic; the value is read by ticket_value
  uint32_t v = 0;
  if (lane_id() == 0) v = __hip_atomic_fetch_add(ea.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return v;
}
UWVK_DEV uint32_t ticket_value(const EpochArgs& ea, uint32_t v) {
  return __builtin_amdgcn_readfirstlane(v) - ea.ticket_base;
}

// One work unit of the epoch kernel: instance tu.inst over epochs
// [tu.e0, tu.e1), Sigma~ loaded from HBM into LDS, every epoch run, stored
// back (folded, or unfolded for the next chunk of a tail instance).  `again`
// re-derives the unit at the end (from the block index or the uniform ticket),
// so that the unit is not kept live through the epochs.  tlw: the timeline
// key of the diagnostic build.
// the next unit's Sigma~ and mean, loaded into registers before this unit's
// stores (persistent kernel): gfx950's vmcnt counts loads and stores in one
// ordered counter, so a load issued after the stores waits for them as well
template <int DOF>
struct PspPre {
  double v[PG<DOF>::NSLOT];
  double m;
  double ps, pm;  // PD: the lane's parameter diagonal entry and mean
  bool have;
};

// PD: the parameter-decoupled kernel (PspSmemPD): the 26-DOF layout of a
// 53-DOF instance, px its parameters' LDS
template <int DOF, bool PERSIST, int QM, int EVS, int SR, int PD, class Again>
UWVK_DEV void psp_unit(PspSmem<DOF>& sm, double* px, const PoseBufs& b, const EpochArgs& ea, const TailUnit& tu0,
                       const LaneQ& lq, Again again, int64_t tlw, int lp, uint32_t* next = nullptr,
                       PspPre<DOF>* pre = nullptr) {
  constexpr int NW = PD ? 53 : DOF;  // the filter's n (sigma-point weights)
  const int64_t B = b.batch;
  const int64_t inst = tu0.inst, e_begin = tu0.e0, e_end = tu0.e1;
#ifdef UWVK_STAMPS
  Stamper stamper;
  Stamper* st = &stamper;
#else
  Stamper* st = nullptr;
#endif
#ifdef UWVK_TIMELINE
  tl_mark(tlw, 0);
  if (lane_id() == 0 && tlw < 131072) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    uwvk_timeline[tlw * 8 + 4] = ((unsigned long long)xcc << 32) | (unsigned)__smid();
    uwvk_timeline[tlw * 8 + 5] = (unsigned long long)inst;
  }
#else
  (void)tlw;
#endif
  // (r04) the unit's independent input loads (rotation rate, per-lane process
  // constants, the first epoch's IMU) issued before Sigma~'s load is waited
  // for: one HBM round trip at the unit's start instead of three in a row
  bool ok = true, nan = false;
  uint32_t cnt[4] = {0, 0, 0, 0};
  MeasArgs ma{};
  ma.v3[0] = ea.p_sens[0]; ma.v3[1] = ea.p_sens[1]; ma.v3[2] = ea.p_sens[2];
  // the stored rotation rate (PoseUKF.cpp:492-496) lives in pc.w only (a
  // second copy for the final store was a second set of loop-carried VGPRs)
  ProcCtx pc;
  for (int k = 0; k < 3; k++) pc.w[k] = b.rot[inst * 3 + k];
  // dt as a VGPR: a uniform kernel argument is an SGPR pair live across the
  // whole epoch loop, which the allocator spilled to a VGPR lane and reloaded
  // (four v_readlane, the whole 16-byte kernarg group) at each of its ~23
  // uses per epoch (tools/isa_hot.py); as a VGPR each use is an operand
  {
    double dtv = ea.dt;
    asm volatile("" : "+v"(dtv));
    pc.dt = dtv;
  }
  pc.off = nullptr;
  lane_proc<DOF, PD>(b, *b.shared, inst, lp, pc);
  // the next epoch's IMU inputs are prefetched one epoch ahead (their load
  // latency overlaps this epoch's arithmetic)
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
  if (PERSIST && pre->have) {
    using G = PG<DOF>;
    const int l = olane();
#pragma unroll
    for (int t = 0; t < G::NSLOT; t++) {
      const int e = l + 64 * t;
      if (e < G::NP) sm.S[e] = pre->v[t];
    }
    if (l < Lay<DOF>::store) sm.mu[l] = pre->m;
    if constexpr (PD) {
      if (l >= kPdLane0 && l < kPdLane0 + kPdN) {
        px[l - kPdLane0] = pre->ps;
        px[32 + l - kPdLane0] = pre->pm;
      }
    }
    psync();
  } else if constexpr (PD) {
    load_psp_pd(sm, px, b, inst, PERSIST ? olane() : lane_id());
  } else {
    load_psp<DOF>(sm, b, inst, PERSIST ? olane() : lane_id());
  }
#ifdef UWVK_TIMELINE
  tl_mark(tlw, 1);
#endif
  UWVK_STAMP(40);
  double ds = 1.0, ids = 1.0;  // time scale of the Markov DOFs (Sigma = D Sigma~ D)
  if (tu0.chunk > 0) {  // the previous chunk's, unfolded: bitwise the one-block run
    const double2 c = PERSIST ? reinterpret_cast<const double2*>(ea.tail_carry)[tu0.tslot * 64 + lane_id()]
                              : tail_carry_in(ea, tu0.tslot);
    ds = c.x;
    ids = c.y;
  }
  // persistent: the next unit's ticket, claimed behind the first inputs' loads
  // (a wait for those does not wait for the atomic; it has long returned when
  // the next epoch's loads are waited for)
  if constexpr (PERSIST) *next = ticket_issue(ea);
#pragma unroll 1
  for (int64_t e = e_begin; e < e_end; e++) {
    const uint32_t fl = fl_n;
    const double g[3] = {g_n[0], g_n[1], g_n[2]}, za[3] = {a_n[0], a_n[1], a_n[2]};
    if (e + 1 < e_end) fetch(e + 1);
    if (all_finite(g, 3)) {  // integrateMeasurement(RotationRate): checkMeasurment, then store
      for (int k = 0; k < 3; k++) pc.w[k] = g[k];
    } else {
      nan = true;
    }
    const PoseShared& sh = shared_for_epoch(b);
    UWVK_STAMP(41);
    if (((e - ea.first) & 1023) == 1023) psp_fold<DOF, PD>(sm, ds, ids, px);  // keep d in range
    bool sok = psp_predict<DOF, QM, SR, PD>(sm, sh, pc, b.Q, b.Qp, ds, ids, lq, st, px);
    ok = ok && sok;
    if (fl & UWVK_EV_ACC) {
      if (all_finite(za, 3)) {
        do_update<DOF, MK_ACC, SR, NW>(sm, sh, inst, za, sh.log_acc_cov, ma, &sok, ds, ids, st);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    if (fl & UWVK_EV_DVL) {
      const double* z = ea.dvl + ((int64_t)ea.dvl_index[e] * B + inst) * 3;
      if (all_finite(z, 3)) {
        cnt[0] += do_update<DOF, MK_VEL, SR, NW>(sm, sh, inst, z, sh.log_dvl_cov, ma, &sok, ds, ids, st);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    // EVS 1: the launch's epochs hold no pressure / ADCP event (host-checked),
    // so those updates are not compiled in (half the SGPR spills, 1% faster:
    // profiles/r03/evs/)
    if constexpr (EVS == 0) {
    if (fl & UWVK_EV_PRESSURE) {
      const double* z = ea.pressure + (int64_t)ea.p_index[e] * B + inst;
      if (all_finite(z, 1)) {
        cnt[1] += do_update<DOF, MK_PRESSURE, SR, NW>(sm, sh, inst, z, &ea.p_cov, ma, &sok, ds, ids);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    if (fl & UWVK_EV_ADCP) {
      for (int c = 0; c < ea.cells; c++) {
        const double* z = ea.adcp + (((int64_t)ea.a_index[e] * ea.cells + c) * B + inst) * 2;
        if (!all_finite(z, 2)) { nan = true; continue; }
        double zz[2] = {z[0], z[1]}, R[4] = {ea.adcp_cov[0], ea.adcp_cov[1], ea.adcp_cov[2], ea.adcp_cov[3]};
        PWater<DOF> h;
        h.cw = ea.cw[c];
        cnt[2] += psp_update<DOF, SR, PWater<DOF>, NW>(sm, zz, R, 1, h, &sok, ds, ids);
        ok = ok && sok;
      }
    }
    }
  }
  if constexpr (PERSIST) {
    // the next unit (its ticket has long returned); a whole instance or a
    // first chunk has no predecessor to wait for, so its Sigma~ and mean are
    // loaded now, ahead of this unit's stores
    const uint32_t un = gridDim.x + ticket_value(ea, *next);
    *next = un;
    const TailUnit tn = ticket_unit(ea, un < ea.units ? un : 0u);
    pre->have = un < ea.units && tn.chunk <= 0;
    // every path defines the registers here (zeros when nothing is
    // prefetched), so they are dead through the next unit's epochs
    using G = PG<DOF>;
    const int l = olane();
    if constexpr (PD) {  // through the 26-DOF layout (load_psp_pd)
      const int64_t in = pre->have ? tn.inst : 0;
      const double* gs = b.sigma + in * (int64_t)PG<53>::NP;
      const double* gm = b.mu + in * (int64_t)Lay<53>::store;
#pragma unroll
      for (int t = 0; t < G::NSLOT; t++) {
        const int e = l + 64 * t;
        pre->v[t] = (pre->have && e < G::NP) ? gs[pd_pidx(e)] : 0.0;
      }
      pre->m = (pre->have && l < Lay<DOF>::store) ? gm[pd_store(l)] : 0.0;
      const bool pl = pre->have && l >= kPdLane0 && l < kPdLane0 + kPdN;
      const int tp = pl ? l - kPdLane0 : 0;
      pre->ps = pl ? gs[pd_diag53(tp)] : 0.0;
      pre->pm = pl ? gm[20 + tp] : 0.0;
    } else {
      const double* gs = b.sigma + (pre->have ? tn.inst : 0) * (int64_t)G::NP;
#pragma unroll
      for (int t = 0; t < G::NSLOT; t++) {
        const int e = l + 64 * t;
        pre->v[t] = (pre->have && e < G::NP) ? gs[e] : 0.0;
      }
      pre->m = (pre->have && l < Lay<DOF>::store) ? b.mu[(pre->have ? tn.inst : 0) * Lay<DOF>::store + l] : 0.0;
    }
  }
  if (lane_id() == 0) {
    // atomic: a later chunk that timed out flags the same word
    const uint32_t bits = (ok ? 0u : UWVK_ST_NOTPD) | (nan ? UWVK_ST_NAN : 0u);
    if (bits) __hip_atomic_fetch_or(b.status + inst, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e_end > e_begin) {
      b.rot[inst * 3] = pc.w[0]; b.rot[inst * 3 + 1] = pc.w[1]; b.rot[inst * 3 + 2] = pc.w[2];
    }
    if (ea.accept_counts)
      for (int k = 0; k < 4; k++) ea.accept_counts[inst * 4 + k] += cnt[k];
  }
#ifdef UWVK_TIMELINE
  tl_mark(tlw, 2);
#endif
  const TailUnit tu = again();  // re-derived, not kept live through the epochs
  const bool hand = tu.chunk >= 0 && tu.chunk + 1 < ea.chunks;
  if (hand) {  // hand on: Sigma~ and d unfolded
    double* c = ea.tail_carry + (tu.tslot * 64 + lane_id()) * 2;
    c[0] = ds;
    c[1] = ids;
    psync();
  } else {
    psp_fold<DOF, PD>(sm, ds, ids, px);
  }
  if constexpr (PD) store_psp_pd(sm, px, b, inst, PERSIST ? olane() : lane_id());
  else store_psp<DOF>(sm, b, inst, PERSIST ? olane() : lane_id());
  if (hand) tail_signal(ea, tu.tslot, tu.chunk);
#ifdef UWVK_TIMELINE
  __builtin_amdgcn_s_waitcnt(0);
  tl_mark(tlw, 3);
#endif
}

// Occupancy of the epoch kernels.  The 53-DOF layout is LDS-bound at 12
// instances per CU (3 waves per SIMD, PspSmem<53> = 12.8 KB) and keeps the
// compiler's own register allocation (<= 168 VGPRs; an explicit
// amdgpu_waves_per_eu(3) scheduled its epoch loop worse, r02).  The 26-DOF
// layout (the kinematic handles and the parameter-decoupled kernel of 53-DOF
// handles) needs ~4.4 KB of LDS: it is capped at 4 waves per SIMD (16
// instances per CU, <= 128 VGPRs) at the cost of ~80-130 B/lane of scratch,
// ~17 reloads per epoch (r06 interleaved A/B, profiles/r06/r06d/: the PD
// kernel 223.6 -> 233.9 M steps/s over 200 epochs, 206.3-207.9 -> 211.6-212.7
// over 20; the plain 26-DOF kernel +5.4% / +4%, r06a).  The expression is
// template-dependent: the 53-DOF instantiations' ISA is unchanged by it.
// PSP_EPOCH_ATTR (make variant VFLAGS=...) overrides it for occupancy A/Bs.
#ifndef PSP_EPOCH_ATTR
#define PSP_EPOCH_ATTR __attribute__((amdgpu_waves_per_eu(DOF == 26 ? 4 : 1, DOF == 26 ? 4 : 8)))
#endif
template <int DOF, int QM, int EVS, int SR, int PD = 0>
__global__ __launch_bounds__(64) PSP_EPOCH_ATTR void k_psp_epoch(PoseBufs b, PoseShared sh0, EpochArgs ea) {
  __shared__ typename SmemT<DOF, PD>::type smx;
  PspSmem<DOF>& sm = smx;
  double* const px = pd_ptr<DOF>(smx);
  const int64_t B = b.batch;
  const TailUnit tu = tail_unit(ea, B);
  if (tu.chunk > 0 && !tail_wait(ea.tail_flag + tu.tslot, ea.tag * 16u + (uint32_t)tu.chunk, ea.wait_bound)) {
    if (lane_id() == 0) {  // atomic: the late predecessor may still flag the same word
      __hip_atomic_fetch_or(b.status + tu.inst, UWVK_ST_SCHEDULE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ea.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-mapped word
    }
    return;
  }
  const LaneQ lq = lane_q<DOF, PD>(b.Qp, lane_id());
  psp_unit<DOF, false, QM, EVS, SR, PD>(sm, px, b, ea, tu, lq, [&] { return tail_unit(ea, B); }, blockIdx.x,
                                        lane_id());
}

// Persistent form (UWVK_OPT_PERSIST): as many blocks as are resident, each
// taking work units from the launch's ticket counter until none is left.  A
// unit is claimed only by a running block, and chunk k of a tail instance is
// claimed after chunk k - 1 (r_x tickets earlier), so a hand-off wait is always
// on a unit that a resident block holds or has finished: no placement or
// dispatch-order assumption.  Faster XCDs / CUs take more units, and a slot
// moves to its next unit without a new workgroup dispatch.  The next ticket is
// taken while the current unit runs (its atomic latency hidden).
template <int DOF, int QM, int EVS, int SR, int PD = 0>
__global__ __launch_bounds__(64) PSP_EPOCH_ATTR void k_psp_epoch_p(PoseBufs b, PoseShared sh0, EpochArgs ea) {
  __shared__ typename SmemT<DOF, PD>::type smx;
  PspSmem<DOF>& sm = smx;
  double* const px = pd_ptr<DOF>(smx);
  const LaneQ lq = lane_q<DOF, PD>(b.Qp, lane_id());
  // the first unit is the block's own index (no atomic: 3,072 blocks claiming
  // one counter at once queue for ~50 us); tickets number the units from the grid on
  const uint32_t grid = gridDim.x;
  uint32_t u = blockIdx.x;
  PspPre<DOF> pre;
  pre.have = false;
#pragma unroll
  for (int t = 0; t < PG<DOF>::NSLOT; t++) pre.v[t] = 0.0;
  pre.m = 0.0;
  pre.ps = 0.0;
  pre.pm = 0.0;
#pragma unroll 1
  while (u < ea.units) {
    const TailUnit tu = ticket_unit(ea, u);
    uint32_t vn = 0;
    if (tu.chunk > 0 && !tail_wait_t<true>(ea.tail_flag + tu.tslot, ea.tag * 16u + (uint32_t)tu.chunk, ea.wait_bound)) {
      if (lane_id() == 0) {
        __hip_atomic_fetch_or(b.status + tu.inst, UWVK_ST_SCHEDULE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ea.fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-mapped word
      }
      u = grid + ticket_value(ea, ticket_issue(ea));
      pre.have = false;
#pragma unroll
      for (int t = 0; t < PG<DOF>::NSLOT; t++) pre.v[t] = 0.0;
      pre.m = 0.0;
      pre.ps = 0.0;
      pre.pm = 0.0;
    } else {
      // a laundered lane id: the unit's per-lane constants are recomputed per
      // unit, not hoisted out of the unit loop (held live across it)
      psp_unit<DOF, true, QM, EVS, SR, PD>(sm, px, b, ea, tu, lq, [&] { return ticket_unit(ea, u); }, u, olane(),
                                           &vn, &pre);
      u = vn;  // resolved by psp_unit
    }
    psync();  // the next unit's LDS writes after this unit's reads
  }
}

// run_log's BodyEfforts epoch: after the k_psp_epoch launch that ran the
// epoch's predict and other updates, the efforts update alone (the last update
// of the epoch), VO 1 its velocity-only form (UWVK_EV_EFFORTS_VELOCITY_ONLY,
// constrainVelocity), VO 0 the full model; the same bookkeeping as the literal
// k_pose_efforts_epoch
// (r05: capped at 3 waves per SIMD, 168 VGPRs and 12 B/lane of scratch, the
// full update ran 1.420 against 1.415 ms per call: the 2-wave allocation stays,
// profiles/r05/r05f/single_update*.txt)
template <int DOF, int VO, int SR>
__global__ __launch_bounds__(64) void k_psp_efforts(PoseBufs b, PoseShared sh, EpochArgs ea) {
  __shared__ PspSmem<DOF> sm;
  const int64_t B = b.batch, inst = xcd_instance(B), e = ea.first;
  if (!(ea.flags[e] & UWVK_EV_EFFORTS)) return;
  const double* z = ea.efforts + ((int64_t)ea.e_index[e] * B + inst) * 6;
  if (!all_finite(z, 6)) {
    if (lane_id() == 0) b.status[inst] |= UWVK_ST_NAN;
    return;
  }
  load_psp<DOF>(sm, b, inst);
  bool ok = true;
  bool acc;
  if constexpr (VO) acc = do_update_vo<DOF, SR>(sm, sh, b, inst, z, ea.e_cov, &ok, 1.0, 1.0);
  else acc = do_update_eff<DOF, SR>(sm, sh, b, inst, z, ea.e_cov, &ok);
  if (lane_id() == 0) {
    if (!ok) b.status[inst] |= UWVK_ST_NOTPD;
    if (ea.accept_counts) ea.accept_counts[inst * 4 + 3] += acc ? 1u : 0u;
  }
  store_psp<DOF>(sm, b, inst);
}

}  // namespace psp

template <int DOF, int SR>
static hipError_t psp_update_dof(int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const MeasArgs& ma, int m) {
  const dim3 g((unsigned)b.batch), t(64);
  switch (kind) {
    case MK_ACC: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_ACC, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_VEL: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_VEL, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_PRESSURE: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_PRESSURE, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_WATER: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_WATER, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_XY: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_XY, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_Z: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_Z, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_GEO: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_GEO, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_DELAYED: hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_DELAYED, SR>), g, t, 0, st, b, sh, ma, m); break;
    case MK_EFFORTS:  // the full model (psp_update_eff) or its velocity-only form (ma.only_vel)
      hipLaunchKernelGGL((psp::k_psp_update<DOF, MK_EFFORTS, SR>), g, t, 0, st, b, sh, ma, m);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int SR>
hipError_t launch_psp_predict_sr(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt) {
  if (dof == 53)
    hipLaunchKernelGGL((psp::k_psp_predict<53, SR>), dim3((unsigned)b.batch), dim3(64), 0, st, b, sh, dt);
  else
    hipLaunchKernelGGL((psp::k_psp_predict<26, SR>), dim3((unsigned)b.batch), dim3(64), 0, st, b, sh, dt);
  return hipGetLastError();
}

template <int SR>
hipError_t launch_psp_update_sr(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                const MeasArgs& ma, int m) {
  return dof == 53 ? psp_update_dof<53, SR>(kind, st, b, sh, ma, m) : psp_update_dof<26, SR>(kind, st, b, sh, ma, m);
}

template <int SR>
hipError_t launch_psp_efforts_sr(int dof, int vo, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const EpochArgs& ea) {
  const dim3 g((unsigned)b.batch), t(64);
  if (dof == 53) {
    if (vo) hipLaunchKernelGGL((psp::k_psp_efforts<53, 1, SR>), g, t, 0, st, b, sh, ea);
    else hipLaunchKernelGGL((psp::k_psp_efforts<53, 0, SR>), g, t, 0, st, b, sh, ea);
  } else {
    if (vo) hipLaunchKernelGGL((psp::k_psp_efforts<26, 1, SR>), g, t, 0, st, b, sh, ea);
    else hipLaunchKernelGGL((psp::k_psp_efforts<26, 0, SR>), g, t, 0, st, b, sh, ea);
  }
  return hipGetLastError();
}

template <int DOF, int QM, int EVS, int SR, int PD = 0>
static void launch_epoch_q(hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea, dim3 g,
                           uint32_t pad) {
  if (ea.ticket)
    hipLaunchKernelGGL((psp::k_psp_epoch_p<DOF, QM, EVS, SR, PD>), g, dim3(64), pad, st, b, sh, ea);
  else
    hipLaunchKernelGGL((psp::k_psp_epoch<DOF, QM, EVS, SR, PD>), g, dim3(64), pad, st, b, sh, ea);
}

template <int DOF, int SR>
static void launch_epoch_dof(hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea, dim3 g,
                             uint32_t ev_any, uint32_t pad) {
  // the kernel instantiated for the handle's process-noise shape (psp_predict
  // QM) and the launch's event kinds (EVS 1: no pressure / ADCP epoch in the
  // range, the C3 workload); a general Q runs the one kernel with everything
  const bool pa = (ev_any & (UWVK_EV_PRESSURE | UWVK_EV_ADCP)) != 0;
  if (!sh.q_simple) launch_epoch_q<DOF, 2, 0, SR>(st, b, sh, ea, g, pad);
  else if (pa) launch_epoch_q<DOF, 1, 0, SR>(st, b, sh, ea, g, pad);
  else launch_epoch_q<DOF, 1, 1, SR>(st, b, sh, ea, g, pad);
}

template <int SR>
hipError_t launch_psp_epoch_sr(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                               int64_t grid, uint32_t ev_any, uint32_t lds_pad, int pd) {
  const dim3 g((unsigned)(grid > 0 ? grid : b.batch));
  if (dof == 53 && pd) {  // the parameter-decoupled kernel (b.Qp: the host's PD table; q_simple)
    if (!sh.q_simple) return hipErrorInvalidValue;
    if (ev_any & (UWVK_EV_PRESSURE | UWVK_EV_ADCP)) launch_epoch_q<26, 1, 0, SR, 1>(st, b, sh, ea, g, lds_pad);
    else launch_epoch_q<26, 1, 1, SR, 1>(st, b, sh, ea, g, lds_pad);
  } else if (dof == 53) {
    launch_epoch_dof<53, SR>(st, b, sh, ea, g, ev_any, lds_pad);
  } else {
    launch_epoch_dof<26, SR>(st, b, sh, ea, g, ev_any, lds_pad);
  }
  return hipGetLastError();
}

// this translation unit's side (uwvk_psp_k.hip: 0, uwvk_psp_k_r.hip: 1)
template hipError_t launch_psp_predict_sr<PSP_SIDE>(int, hipStream_t, const PoseBufs&, const PoseShared&, double);
template hipError_t launch_psp_update_sr<PSP_SIDE>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                   const MeasArgs&, int);
template hipError_t launch_psp_epoch_sr<PSP_SIDE>(int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                  const EpochArgs&, int64_t, uint32_t, uint32_t, int);
template hipError_t launch_psp_efforts_sr<PSP_SIDE>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                    const EpochArgs&);

#if PSP_SIDE == 0
// the handle's side picks the instantiation set (a template parameter of every
// PSP kernel, not a run-time branch in the epoch loop)
hipError_t launch_psp_predict(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt) {
  return sh.so3_right ? launch_psp_predict_sr<1>(dof, st, b, sh, dt) : launch_psp_predict_sr<0>(dof, st, b, sh, dt);
}

hipError_t launch_psp_update(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                             const MeasArgs& ma, int m) {
  return sh.so3_right ? launch_psp_update_sr<1>(dof, kind, st, b, sh, ma, m)
                      : launch_psp_update_sr<0>(dof, kind, st, b, sh, ma, m);
}

hipError_t launch_psp_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                            int64_t grid, uint32_t ev_any, uint32_t lds_pad, int pd) {
  return sh.so3_right ? launch_psp_epoch_sr<1>(dof, st, b, sh, ea, grid, ev_any, lds_pad, pd)
                      : launch_psp_epoch_sr<0>(dof, st, b, sh, ea, grid, ev_any, lds_pad, pd);
}

hipError_t launch_psp_efforts(int dof, int vo, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                              const EpochArgs& ea) {
  return sh.so3_right ? launch_psp_efforts_sr<1>(dof, vo, st, b, sh, ea) : launch_psp_efforts_sr<0>(dof, vo, st, b, sh, ea);
}

// XCC placement probe: block b writes the XCC it runs on (hardware XCC_ID).
__global__ __launch_bounds__(64) void k_xcc_probe(uint32_t* out) {
  if (threadIdx.x == 0) {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    out[blockIdx.x] = x & 0xfu;
  }
}

// 1 when the blocks of a probe grid were placed round-robin over 8 distinct
// XCCs (block b on the XCC of block b % 8: the placement of a single-partition MI355X, which the tail
// plan and xcd_instance assume), else 0.  Measured once per device.
int xcd_round_robin(int device) {
  // per-device result, -1 until measured; atomic so that host threads driving
  // handles on several GPUs may probe concurrently (two first callers of one
  // device both probe and store the same answer)
  static std::atomic<int> cache[64] = {};
  static std::once_flag init;
  std::call_once(init, [] {
    for (auto& c : cache) c.store(-1, std::memory_order_relaxed);
  });
  if (device < 0 || device >= 64) return 0;
  const int known = cache[device].load(std::memory_order_acquire);
  if (known >= 0) return known;
  DeviceGuard g(device);
  constexpr int kBlocks = 8 * 1024;
  uint32_t* d = nullptr;
  std::vector<uint32_t> h(kBlocks, 0xffu);
  int ok = 0;
  if (hipMalloc(&d, kBlocks * 4) == hipSuccess) {
    hipLaunchKernelGGL(k_xcc_probe, dim3(kBlocks), dim3(64), 0, 0, d);
    if (hipGetLastError() == hipSuccess && hipMemcpy(h.data(), d, kBlocks * 4, hipMemcpyDeviceToHost) == hipSuccess) {
      // blocks b and b + 8 k share an XCC, and the 8 residues cover 8 XCCs
      ok = 1;
      bool seen[16] = {};
      for (int b = 0; b < kBlocks; b++) {
        if (h[b] >= 16 || h[b] != h[b % 8]) ok = 0;
        if (b < 8 && h[b] < 16) seen[h[b]] = true;
      }
      int distinct = 0;
      for (bool v : seen) distinct += v;
      if (distinct != 8) ok = 0;
    }
    (void)hipFree(d);
  }
  cache[device].store(ok, std::memory_order_release);
  return ok;
}

size_t psp_epoch_lds_bytes(int dof) { return dof == 53 ? sizeof(psp::PspSmem<53>) : sizeof(psp::PspSmem<26>); }

int64_t psp_epoch_slots_per_xcd(int dof, int device, int pd) { return psp_epoch_slots(dof, device, false, pd) / 8; }

int64_t psp_epoch_slots(int dof, int device, bool persist, int pd) {
  int per_cu = 0, cus = 0;
  // (the other instantiations of a layout have the same LDS and occupancy:
  // tests/test_kernel_resources.py holds every 53-DOF one to 3 waves per SIMD
  // and every 26-DOF-layout one to 4)
  const void* k;
  if (dof == 53 && pd)
    k = persist ? (const void*)psp::k_psp_epoch_p<26, 1, 0, 0, 1> : (const void*)psp::k_psp_epoch<26, 1, 0, 0, 1>;
  else
    k = persist ? (dof == 53 ? (const void*)psp::k_psp_epoch_p<53, 1, 0, 0> : (const void*)psp::k_psp_epoch_p<26, 1, 0, 0>)
                : (dof == 53 ? (const void*)psp::k_psp_epoch<53, 1, 0, 0> : (const void*)psp::k_psp_epoch<26, 1, 0, 0>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64, 0) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return 0;
  return (int64_t)per_cu * cus;
}

// Last-generation spreading.  Blocks of one XCD are dispatched in order to
// its s resident slots; wave speeds differ (the first generation's waves end
// anywhere between 0.8 and 1.25 of the mean), so after a few generations the
// slots free up at scattered times and a launch of whole-instance blocks of
// duration D ends with a ramp: the slots idle for D / 2 on average while the
// last blocks finish.  Spreading ends the launch on short blocks instead: the
// last m = C s instances of each XCD run as C epoch chunks, grouped by chunk
// (all chunk-0 blocks after the whole instances, then all chunk-1 blocks,
// ...), so each group keeps the XCD busy for about D and a chunk's
// predecessor, m blocks earlier, has long finished; the ramp shrinks to
// D / (2 C), for (C - 1) m extra block prologues and epilogues (Sigma~ and
// its time scale reloaded and stored, the IMU prefetch restarted: about 0.75
// epoch each, r02 timeline).  C minimises
// count / (2 C) + 0.3 C (C - 1) epochs; none below a 10 % gain or when the
// XCD has under (C + 1) s instances.
constexpr double kTailChunkOverhead = 0.75;  // epochs per extra chunk (r02 timeline)
int plan_tail(int64_t n, int64_t s, int64_t count) {
  if (s <= 0 || count < 4) return 1;
  const double base = 0.5 * (double)count;
  double best = 0.9 * base;
  int chunks = 1;
  for (int c = 2; c <= 8 && 2 * c <= count; c++) {
    if (n < (c + 1) * s) break;
    const double cost = (double)count / (2.0 * c) + kTailChunkOverhead * c * (c - 1);
    if (cost < best) {
      best = cost;
      chunks = c;
    }
  }
  return chunks;
}

#endif  // PSP_SIDE == 0

}  // namespace uwvk

// diagnostic builds only: each side's translation unit keeps its own device
// symbols, so each exports its own reader (the _r suffix: the right side, SR = 1)
#if PSP_SIDE == 0
#define UWVK_PSP_DBG(name) name
#else
#define UWVK_PSP_DBG(name) name##_r
#endif

#if defined(UWVK_TIMELINE)
extern "C" int UWVK_PSP_DBG(uwvk_debug_read_timeline)(unsigned long long* out, long long n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(uwvk::psp::uwvk_timeline), (size_t)n * 8) != hipSuccess;
}
#endif

#if defined(UWVK_STAMPS)
// per-phase cycle sums of this side's PSP kernels
extern "C" int UWVK_PSP_DBG(uwvk_debug_read_stamps_psp)(unsigned long long* sum, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(sum, HIP_SYMBOL(uwvk::uwvk_stamp_sum), 64 * 8) != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(uwvk::uwvk_stamp_cnt), 64 * 8) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(uwvk::uwvk_stamp_sum), z, 64 * 8) != hipSuccess) return 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(uwvk::uwvk_stamp_cnt), z, 64 * 8) != hipSuccess) return 1;
  }
  return 0;
}
#endif
