// uwvk_pose_kernels.hpp — PoseUKF kernel templates (one workgroup of
// Geo<DOF>::T threads per filter instance) and their launch declarations.
// Explicit instantiations live in the uwvk_pose_k_*.hip translation units so
// the build parallelises; the C ABI (uwvk_pose.hip) only sees the launchers.
#pragma once
#include "uwvk_pose_dev.hpp"

namespace uwvk {

enum MeasKind { MK_ACC = 0, MK_VEL, MK_PRESSURE, MK_WATER, MK_EFFORTS, MK_XY, MK_Z, MK_GEO, MK_DELAYED };

struct MeasArgs {
  const double* mu;    // [batch][m]
  const double* cov;   // [batch][m*m] or null -> shared_cov
  double shared_cov[36];
  const uint8_t* mask; // nullable
  uint8_t* accepted;   // nullable
  const double* extra; // cell_weighting [batch] / delayed_xy [batch][2]
  double v3[3];        // sensor_in_imu / gps_in_body
  int only_vel;
};

struct EpochArgs {
  const uint32_t* flags;
  const double* gyro;
  const double* acc;
  double acc_cov[9];
  const int32_t* dvl_index;
  const double* dvl;
  double dvl_cov[9];
  const int32_t* p_index;
  const double* pressure;
  double p_cov;
  double p_sens[3];
  const int32_t* a_index;
  const double* adcp;
  int cells;
  double cw[8];
  double adcp_cov[4];
  const int32_t* e_index;
  const double* efforts;
  double e_cov[36];
  double dt;
  int64_t first, count;
  uint32_t* accept_counts;  // [batch][4] nullable
  // literal epoch kernel only: run just the BodyEfforts update of each epoch
  // (the PSP launch before it has done the epoch's predict and other updates)
  int efforts_only;
  // PSP epoch kernel, last-generation spreading (uwvk_psp_k.hip, plan_tail):
  // chunks <= 1 = one block per instance over [first, first + count).
  // Otherwise (static k_psp_epoch) block b runs on XCD x = b & 7 at position i = b >> 3: whole
  // instance x n_x + i for i < tail0, else chunk k = (i - tail0) / r_x of tail
  // instance x n_x + tail0 + (i - tail0) % r_x, handed on through tail_flag /
  // tail_carry
  uint32_t* tail_flag;  // per tail instance: tag * 16 + chunks done
  double* tail_carry;   // per tail instance: the time scale (ds, ids) per lane
  int64_t n_x;          // instances per XCD
  int64_t tail0;        // first tail instance (XCD-local) = n_x - r_x
  int64_t r_x;          // tail instances per XCD (chunks x resident blocks)
  int chunks;
  uint32_t tag;         // per launch
  uint32_t wait_bound;  // tail_wait: sleeps before a hand-off counts as lost
  // persistent PSP epoch kernel (UWVK_OPT_PERSIST, k_psp_epoch_p): block b
  // runs unit b first, then takes units from a ticket counter, unit
  // gridDim.x + (*ticket - ticket_base) before the atomic; units [0, tail0)
  // whole instances, then chunk k of tail
  // instance tail0 + t at unit tail0 + k r_x + t (r_x tail instances)
  uint32_t* ticket;
  uint32_t ticket_base;
  // the handle's hand-off fault word (pinned host memory): set to 1 by any
  // chunk whose predecessor's hand-off timed out (UWVK_ESCHEDULE)
  uint32_t* fault;
  uint32_t units;       // tail0 + chunks * r_x
};

// host-callable launchers (grid = one workgroup per instance)
hipError_t launch_pose_predict(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt);
hipError_t launch_pose_update(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                              const MeasArgs& ma, int m);
hipError_t launch_pose_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea);
// vo: the epoch's flag word has UWVK_EV_EFFORTS_VELOCITY_ONLY (constrainVelocity);
// the apply_delta form is sh.literal_apply_delta
hipError_t launch_pose_efforts_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                     const EpochArgs& ea, int vo);
hipError_t launch_pose_rotation_rate(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double* out);
// the truth store-vector of the ensemble statistics, passed by value (kernarg)
struct StatTruth {
  double v[54];
  int right;  // the handle's SO3 side (UWVK_OPT_SO3_RIGHT): orientation error log(t^-1 q), else log(q t^-1)
};
// part: ceil(batch / 64) x (3 store + 2) doubles of device scratch
hipError_t launch_pose_stats(int dof, hipStream_t st, const PoseBufs& b, const StatTruth& truth, double* out,
                             double* part);

#ifdef UWVK_POSE_KERNEL_BODIES





template <int DOF>
UWVK_DEV void load_instance(Smem<DOF>& sm, const PoseBufs& b, int64_t i) {
  const int l = tid();
  constexpr int T = Geo<DOF>::T, NL = (DOF * DOF + T - 1) / T;
  const double* gs = b.sigma + i * (int64_t)tri_n<DOF>();  // packed lower triangle in HBM
  double v[NL];
#pragma unroll
  for (int u = 0; u < NL; u++) {  // all loads in flight before the first LDS store
    const int k = l + u * T;
    const int r = k / DOF, c = k - (k / DOF) * DOF;
    v[u] = (k < DOF * DOF) ? gs[pidx(r, c)] : 0.0;
  }
  const double m = (l < Lay<DOF>::store) ? b.mu[i * Lay<DOF>::store + l] : 0.0;
#pragma unroll
  for (int u = 0; u < NL; u++) {
    const int k = l + u * T;
    if (k < DOF * DOF) sm.S[k] = v[u];
  }
  if (l < Lay<DOF>::store) sm.mu[l] = m;
  __syncthreads();
}

template <int DOF>
UWVK_DEV void store_instance(const Smem<DOF>& sm, const PoseBufs& b, int64_t i) {
  const int l = tid();
  double* gs = b.sigma + i * (int64_t)tri_n<DOF>();
  for (int e = l; e < tri_n<DOF>(); e += Geo<DOF>::T) {
    int r, c;
    unpack(e, r, c);
    gs[e] = sm.S[r * DOF + c];
  }
  if (l < Lay<DOF>::store) b.mu[i * Lay<DOF>::store + l] = sm.mu[l];
}

UWVK_DEV bool all_finite(const double* a, int n) {
  bool f = true;
  for (int k = 0; k < n; k++) f = f && isfinite(a[k]);
  return f;
}

// The BodyEfforts update (VO = 0, measurementEfforts, PoseUKF.cpp:581-602) or its
// velocity-only form (VO = 1, constrainVelocity, PoseUKF.cpp:585-591); LAD as in
// pose_update.  k_pose_efforts_epoch instantiates each (VO, LAD = 0) pair alone:
// with both models and the literal re-spread in one kernel the register peak was
// the re-spread's (512 B/lane of scratch; 24 B/lane without it).
template <int DOF, int VO, int LAD = -1>
UWVK_DEV bool do_update_efforts(Smem<DOF>& sm, const PoseShared& sh, const PoseBufs& b, int64_t i, const double* zin,
                                const double* Rin, const MeasArgs& ma, double wrot[3], bool* ok, Stamper* st) {
  using L = Lay<DOF>;
  double z[6], R[36];
  for (int k = 0; k < 6; k++) z[k] = zin[k];
  for (int k = 0; k < 36; k++) R[k] = Rin[k];
  Efforts6 ef;
  ef.base = b.uwv;
  ef.weight = sh.uwv_weight;
  ef.buoyancy = sh.uwv_buoyancy;
  for (int k = 0; k < 3; k++) { ef.cog[k] = sh.cog[k]; ef.cob[k] = sh.cob[k]; }
  double wb[3];
  rotation_rate_body<DOF>(sm, sh, wrot, wb);
  double* model = b.model + i * 27;
  if constexpr (VO) {
    HConstrain<DOF> h;
    h.ef = ef;
    h.blk.has = true;
    h.blk.v = model;
    for (int k = 0; k < 3; k++) { h.wb[k] = wb[k]; h.imu[k] = sh.p.imu_in_body[k]; }
    h.w3[0] = sm.mu[L::s_wv]; h.w3[1] = sm.mu[L::s_wv + 1]; h.w3[2] = 0.0;
    for (int k = 0; k < 4; k++) h.q[k] = sm.mu[L::s_quat + k];
    double ra[3], cr[3], cc[3];
    qrot_inv(h.q, sm.mu + L::s_acc, ra);
    cross3(wb, h.imu, cr);
    cross3(wb, cr, cc);
    for (int k = 0; k < 3; k++) h.ab[k] = ra[k] - cc[k];
    return pose_update<DOF, 6, HConstrain<DOF>, LAD>(sm, z, R, 0, 0, h, ok, st, sh.literal_apply_delta != 0,
                                                     sh.so3_right);
  } else {
    HEfforts<DOF> h;
    h.ef = ef;
    for (int k = 0; k < 3; k++) { h.wb[k] = wb[k]; h.imu[k] = sh.p.imu_in_body[k]; }
    // side effect of PoseUKF.cpp:173: the shared model ends with the last sigma
    // point's blocks, X_2n = mu [+] -L_{:,n-1}, i.e. the pre-update mean's.
    if constexpr (L::has_params) {
      const int l = tid();
      if (l < 9) {
        model[l] = sm.mu[L::s_inertia + l];
        model[9 + l] = sm.mu[L::s_lin + l];
        model[18 + l] = sm.mu[L::s_quad + l];
      }
    }
    return pose_update<DOF, 6, HEfforts<DOF>, LAD>(sm, z, R, 0, 0, h, ok, st, sh.literal_apply_delta != 0,
                                                   sh.so3_right);
  }
}

// one measurement update of kind K on instance i (Sigma in LDS)
template <int DOF, int K>
UWVK_DEV bool do_update(Smem<DOF>& sm, const PoseShared& sh, const PoseBufs& b, int64_t i, const double* zin,
                        const double* Rin, const MeasArgs& ma, double wrot[3], bool* ok, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  if constexpr (K == MK_ACC) {
    double z[3], R[9];
    for (int k = 0; k < 3; k++) z[k] = zin[k];
    for (int k = 0; k < 9; k++) R[k] = Rin[k];
    return pose_update<DOF, 3>(sm, z, R, 1, 0, HAcc<DOF>{}, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else if constexpr (K == MK_VEL) {
    double z[3], R[9];
    for (int k = 0; k < 3; k++) z[k] = zin[k];
    for (int k = 0; k < 9; k++) R[k] = Rin[k];
    return pose_update<DOF, 3>(sm, z, R, 1, 0, HVel<DOF>{}, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else if constexpr (K == MK_PRESSURE) {
    double z[1] = {zin[0]}, R[1] = {Rin[0]};
    HPressure<DOF> h;
    h.s[0] = ma.v3[0]; h.s[1] = ma.v3[1]; h.s[2] = ma.v3[2];
    h.patm = sh.p.atmospheric_pressure;
    return pose_update<DOF, 1>(sm, z, R, 0, 0, h, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else if constexpr (K == MK_WATER) {
    double z[2] = {zin[0], zin[1]}, R[4] = {Rin[0], Rin[1], Rin[2], Rin[3]};
    HWater<DOF> h;
    h.cw = ma.extra ? ma.extra[i] : 0.0;
    return pose_update<DOF, 2>(sm, z, R, 1, 1, h, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else if constexpr (K == MK_XY || K == MK_GEO || K == MK_DELAYED) {
    double z[2] = {zin[0], zin[1]}, R[4] = {Rin[0], Rin[1], Rin[2], Rin[3]};
    int gate = 0;
    if constexpr (K == MK_GEO) {  // PoseUKF.cpp:571-578
      double r[3];
      const double x = (zin[0] - sh.lat0) * sh.rm;
      const double y = -(zin[1] - sh.lon0) * sh.rn_cos;
      qrot(sm.mu + L::s_quat, ma.v3, r);
      z[0] = x - r[0];
      z[1] = y - r[1];
      gate = 1;
    }
    if constexpr (K == MK_DELAYED) {  // PoseUKF.cpp:516-521
      z[0] = zin[0] + (sm.mu[L::s_pos] - ma.extra[2 * i]);
      z[1] = zin[1] + (sm.mu[L::s_pos + 1] - ma.extra[2 * i + 1]);
    }
    return pose_update<DOF, 2>(sm, z, R, 0, gate, HXY<DOF>{}, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else if constexpr (K == MK_Z) {
    double z[1] = {zin[0]}, R[1] = {Rin[0]};
    return pose_update<DOF, 1>(sm, z, R, 0, 0, HZ<DOF>{}, ok, st, sh.literal_apply_delta != 0, sh.so3_right);
  } else {  // MK_EFFORTS, PoseUKF.cpp:581-602
    return ma.only_vel ? do_update_efforts<DOF, 1>(sm, sh, b, i, zin, Rin, ma, wrot, ok, st)
                       : do_update_efforts<DOF, 0>(sm, sh, b, i, zin, Rin, ma, wrot, ok, st);
  }
}

template <int DOF>
__global__ __launch_bounds__(Geo<DOF>::T) void k_pose_predict(PoseBufs b, PoseShared sh, double dt) {
  __shared__ Smem<DOF> sm;
  const int64_t i = xcd_instance(b.batch);
  load_instance<DOF>(sm, b, i);
  ProcCtx pc;
  for (int k = 0; k < 3; k++) pc.w[k] = b.rot[i * 3 + k];
  pc.dt = dt;
  pc.off = b.off + i * 28;
  const bool ok = pose_predict<DOF>(sm, sh, pc, b.Q);
  if (!ok && tid() == 0) b.status[i] |= UWVK_ST_NOTPD;
  store_instance<DOF>(sm, b, i);
}

// single-call literal updates at 2 waves/SIMD (scratch spills accepted), batch
// 65,536, tools/time_single_update.py: efforts 7.0 -> 5.3 ms, dense acceleration 5.2 -> 3.2 ms
#ifndef UWVK_UPD_ATTR
#define UWVK_UPD_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))
#endif
// VO / LAD (MK_EFFORTS only): >= 0 the efforts / velocity-only model and the
// apply_delta form fixed at compile time (do_update_efforts), picked by the host
template <int DOF, int K, int VO = -1, int LAD = -1>
__global__ __launch_bounds__(Geo<DOF>::T) UWVK_UPD_ATTR void k_pose_update(PoseBufs b, PoseShared sh, MeasArgs ma, int m) {
  __shared__ Smem<DOF> sm;
  const int64_t i = xcd_instance(b.batch);
  if (ma.mask && !ma.mask[i]) {
    if (ma.accepted && tid() == 0) ma.accepted[i] = 0;
    return;
  }
  const double* z = ma.mu + i * m;
  const double* R = ma.cov ? ma.cov + i * m * m : ma.shared_cov;
  if (!all_finite(z, m) || !all_finite(R, m * m)) {  // checkMeasurment [EXT]
    if (tid() == 0) {
      b.status[i] |= UWVK_ST_NAN;
      if (ma.accepted) ma.accepted[i] = 0;
    }
    return;
  }
  load_instance<DOF>(sm, b, i);
  double w[3] = {b.rot[i * 3], b.rot[i * 3 + 1], b.rot[i * 3 + 2]};
  bool ok = true;
  bool acc;
  if constexpr (K == MK_EFFORTS && VO >= 0)
    acc = do_update_efforts<DOF, VO, LAD>(sm, sh, b, i, z, R, ma, w, &ok, nullptr);
  else
    acc = do_update<DOF, K>(sm, sh, b, i, z, R, ma, w, &ok);
  if (tid() == 0) {
    if (!ok) b.status[i] |= UWVK_ST_NOTPD;
    if (ma.accepted) ma.accepted[i] = acc ? 1 : 0;
  }
  store_instance<DOF>(sm, b, i);
}

// The BodyEfforts update of epoch ea.first alone (run_log's PSP split: the PSP
// launch has done that epoch's predict and other updates).  Same effect as
// k_pose_epoch with efforts_only, but only this update is instantiated, so the
// kernel has the single-update register footprint instead of the fused
// kernel's (576 B/lane scratch, VGPR spills).
// 2 waves/SIMD (4 instances per CU, LDS-bound): 6.41 -> 4.10 ms per update at
// batch 65,536 when introduced (688 B/lane of scratch then; 24 B/lane since the
// per-model / per-apply_delta instantiation, 2.44 ms per update)
#ifndef UWVK_EFF_ATTR
#define UWVK_EFF_ATTR __attribute__((amdgpu_waves_per_eu(2, 2)))
#endif
// VO: 0 / 1 the efforts / velocity-only instantiation picked by the host from the
// epoch's flag word, LAD 0 (the default exact apply_delta); VO = -1 with LAD = -1
// decides both at run time (the UWVK_OPT_LITERAL_APPLY_DELTA option)
template <int DOF, int VO, int LAD>
__global__ __launch_bounds__(Geo<DOF>::T) UWVK_EFF_ATTR void k_pose_efforts_epoch(PoseBufs b, PoseShared sh, EpochArgs ea) {
  __shared__ Smem<DOF> sm;
  const int64_t B = b.batch, i = xcd_instance(B), e = ea.first;
  const uint32_t fl = ea.flags[e];
  if (!(fl & UWVK_EV_EFFORTS)) return;
#ifdef UWVK_STAMPS
  Stamper stamper;
  Stamper* st = &stamper;
#else
  Stamper* st = nullptr;
#endif
  load_instance<DOF>(sm, b, i);
  UWVK_STAMP(11);
  MeasArgs me{};
  me.only_vel = VO >= 0 ? VO : ((fl & UWVK_EV_EFFORTS_VELOCITY_ONLY) ? 1 : 0);
  me.v3[0] = ea.p_sens[0]; me.v3[1] = ea.p_sens[1]; me.v3[2] = ea.p_sens[2];
  double w[3] = {b.rot[i * 3], b.rot[i * 3 + 1], b.rot[i * 3 + 2]};
  const double* z = ea.efforts + ((int64_t)ea.e_index[e] * B + i) * 6;
  bool sok = true, nan = false;
  uint32_t acc = 0;
  if (all_finite(z, 6)) acc = (VO > 0 || (VO < 0 && me.only_vel) ? do_update_efforts<DOF, 1, LAD>(sm, sh, b, i, z, ea.e_cov, me, w, &sok, st)
                                                    : do_update_efforts<DOF, 0, LAD>(sm, sh, b, i, z, ea.e_cov, me, w, &sok, st))
              ? 1u : 0u;
  else nan = true;
  UWVK_STAMP(12);
  if (tid() == 0) {
    if (!sok) b.status[i] |= UWVK_ST_NOTPD;
    if (nan) b.status[i] |= UWVK_ST_NAN;
    if (ea.accept_counts) ea.accept_counts[i * 4 + 3] += acc;
  }
  store_instance<DOF>(sm, b, i);
  UWVK_STAMP(13);
}

template <int DOF>
__global__ __launch_bounds__(Geo<DOF>::T) void k_pose_epoch(PoseBufs b, PoseShared sh, EpochArgs ea) {
  __shared__ Smem<DOF> sm;
  const int64_t B = b.batch, i = xcd_instance(B);
#ifdef UWVK_STAMPS
  Stamper stamper;
  Stamper* st = &stamper;
#else
  Stamper* st = nullptr;
#endif
  load_instance<DOF>(sm, b, i);
  UWVK_STAMP(11);
  bool ok = true, nan = false;
  uint32_t cnt[4] = {0, 0, 0, 0};
  MeasArgs ma;
  ma.mask = nullptr; ma.accepted = nullptr; ma.cov = nullptr; ma.only_vel = 0;
  ma.v3[0] = ea.p_sens[0]; ma.v3[1] = ea.p_sens[1]; ma.v3[2] = ea.p_sens[2];
  double w[3] = {b.rot[i * 3], b.rot[i * 3 + 1], b.rot[i * 3 + 2]};
  ProcCtx pc;
  for (int k = 0; k < 3; k++) pc.w[k] = w[k];
  pc.dt = ea.dt;
  pc.off = b.off + i * 28;
  for (int64_t e = ea.first; e < ea.first + ea.count; e++) {
    const uint32_t fl = ea.flags[e];
    bool sok = true;
    if (!ea.efforts_only) {
    const double* g = ea.gyro + (e * B + i) * 3;
    if (all_finite(g, 3)) {  // integrateMeasurement(RotationRate): checkMeasurment, then store
      for (int k = 0; k < 3; k++) { w[k] = g[k]; pc.w[k] = g[k]; }
    } else {
      nan = true;
    }
    sok = pose_predict<DOF>(sm, sh, pc, b.Q, st);
    ok = ok && sok;
    if (fl & UWVK_EV_ACC) {
      const double* z = ea.acc + (e * B + i) * 3;
      if (all_finite(z, 3)) {
        do_update<DOF, MK_ACC>(sm, sh, b, i, z, ea.acc_cov, ma, w, &sok, st);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    if (fl & UWVK_EV_DVL) {
      const double* z = ea.dvl + ((int64_t)ea.dvl_index[e] * B + i) * 3;
      if (all_finite(z, 3)) {
        cnt[0] += do_update<DOF, MK_VEL>(sm, sh, b, i, z, ea.dvl_cov, ma, w, &sok, st);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    if (fl & UWVK_EV_PRESSURE) {
      const double* z = ea.pressure + (int64_t)ea.p_index[e] * B + i;
      if (all_finite(z, 1)) {
        cnt[1] += do_update<DOF, MK_PRESSURE>(sm, sh, b, i, z, &ea.p_cov, ma, w, &sok);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
    if (fl & UWVK_EV_ADCP) {
      for (int c = 0; c < ea.cells; c++) {
        const double* z = ea.adcp + (((int64_t)ea.a_index[e] * ea.cells + c) * B + i) * 2;
        if (!all_finite(z, 2)) { nan = true; continue; }
        double zz[2] = {z[0], z[1]}, R[4] = {ea.adcp_cov[0], ea.adcp_cov[1], ea.adcp_cov[2], ea.adcp_cov[3]};
        HWater<DOF> h;
        h.cw = ea.cw[c];
        cnt[2] += pose_update<DOF, 2>(sm, zz, R, 1, 1, h, &sok, st, sh.literal_apply_delta != 0, sh.so3_right);
        ok = ok && sok;
      }
    }
    }  // !efforts_only
    if (fl & UWVK_EV_EFFORTS) {
      MeasArgs me = ma;
      me.only_vel = (fl & UWVK_EV_EFFORTS_VELOCITY_ONLY) ? 1 : 0;
      const double* z = ea.efforts + ((int64_t)ea.e_index[e] * B + i) * 6;
      if (all_finite(z, 6)) {
        cnt[3] += do_update<DOF, MK_EFFORTS>(sm, sh, b, i, z, ea.e_cov, me, w, &sok);
        ok = ok && sok;
      } else {
        nan = true;
      }
    }
  }
  if (tid() == 0) {
    if (!ok) b.status[i] |= UWVK_ST_NOTPD;
    if (nan) b.status[i] |= UWVK_ST_NAN;
    if (ea.count > 0) {
      b.rot[i * 3] = w[0]; b.rot[i * 3 + 1] = w[1]; b.rot[i * 3 + 2] = w[2];
    }
    if (ea.accept_counts)
      for (int k = 0; k < 4; k++) ea.accept_counts[i * 4 + k] += cnt[k];
  }
  UWVK_STAMP(12);
  store_instance<DOF>(sm, b, i);
  UWVK_STAMP(13);
}

template <int DOF>
__global__ __launch_bounds__(64) void k_pose_rotation_rate(PoseBufs b, PoseShared sh, double* out) {
  __shared__ Smem<DOF> sm;
  const int64_t i = blockIdx.x;
  if (lane_id() < Lay<DOF>::store) sm.mu[lane_id()] = b.mu[i * Lay<DOF>::store + lane_id()];
  __syncthreads();
  double w[3] = {b.rot[i * 3], b.rot[i * 3 + 1], b.rot[i * 3 + 2]}, o[3];
  rotation_rate_body<DOF>(sm, sh, w, o);
  if (lane_id() < 3) out[i * 3 + lane_id()] = o[lane_id()];
}

// Ensemble statistics, deterministic two-stage reduction (no atomics): one wave
// per 64 instances writes one partial row, then k_pose_stats_sum adds the rows
// in a fixed order.  The 64 instances' mu rows are contiguous in HBM, so the
// wave copies them into LDS in one coalesced sweep; lane l then works on
// instance l (SO3 log error, 9x9 NEES solve) and lane s sums column s over the
// instances in order, so no cross-lane reduction tree is needed.
// Layout of out (nout = 3 store + 2): sum mu, sum mu^2, sum err^2 (orientation
// slots 3..5 hold the squared SO3 log error, slot 6 is 0), NEES over
// (position, orientation, velocity) summed over the instances whose 9x9 block
// is positive definite, and the number of instances left out of that sum.
template <int DOF>
__global__ __launch_bounds__(64) void k_pose_stats(PoseBufs b, StatTruth truth, double* part) {
  using L = Lay<DOF>;
  constexpr int S = L::store, NOUT = 3 * S + 2;
  static_assert(S + 2 <= 64, "one lane per output column");
  __shared__ double xs[64 * S];  // the block's mu rows, as stored
  __shared__ double pe[64 * 5];  // per instance: squared rotation-vector error (3), NEES, excluded
  const int l = threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.x * 64;
  const int nl = (int)(b.batch - i0 < 64 ? b.batch - i0 : 64);
  const double* tv = truth.v;
  const double* xg = b.mu + i0 * S;
#pragma unroll 6
  for (int k = l; k < nl * S; k += 64) xs[k] = xg[k];
  __syncthreads();
  if (l < nl) {
    const double* x = xs + l * S;
    const double* P = b.sigma + (i0 + l) * (int64_t)tri_n<DOF>();
    double r[3];
    qboxminus_side(x + 3, tv + 3, r, truth.right);  // the error in the covariance's frame
    // NEES over (position, orientation, velocity): e^T P_sub^-1 e via a 9x9 Cholesky solve
    double err[9];
    for (int k = 0; k < 3; k++) { err[k] = x[k] - tv[k]; err[3 + k] = r[k]; err[6 + k] = x[7 + k] - tv[7 + k]; }
    double A[45], id[9];  // packed lower triangle (Sigma's first 45 entries); reciprocal pivots
#pragma unroll
    for (int k = 0; k < 45; k++) A[k] = P[k];
    bool pd = true;  // a non-positive pivot (or a NaN) leaves the instance out of the NEES sum
#pragma unroll
    for (int c = 0; c < 9; c++) {
      double s = A[pidx(c, c)];
#pragma unroll
      for (int k = 0; k < c; k++) s -= A[pidx(c, k)] * A[pidx(c, k)];
      pd = pd && (s > 0.0);
      const double dg = sqrt(s > 0.0 ? s : 1.0);
      A[pidx(c, c)] = dg;
      id[c] = 1.0 / dg;
#pragma unroll
      for (int a = c + 1; a < 9; a++) {
        double t = A[pidx(a, c)];
#pragma unroll
        for (int k = 0; k < c; k++) t -= A[pidx(a, k)] * A[pidx(c, k)];
        A[pidx(a, c)] = t * id[c];
      }
    }
    double y[9], nees = 0;
#pragma unroll
    for (int a = 0; a < 9; a++) {
      double s = err[a];
#pragma unroll
      for (int k = 0; k < a; k++) s -= A[pidx(a, k)] * y[k];
      y[a] = s * id[a];
      nees += y[a] * y[a];
    }
    pd = pd && isfinite(nees);
    pe[l * 5 + 0] = r[0] * r[0];
    pe[l * 5 + 1] = r[1] * r[1];
    pe[l * 5 + 2] = r[2] * r[2];
    pe[l * 5 + 3] = pd ? nees : 0.0;
    pe[l * 5 + 4] = pd ? 0.0 : 1.0;
  }
  __syncthreads();
  double* o = part + (int64_t)blockIdx.x * NOUT;
  if (l < S) {
    const double t = tv[l];
    double sx = 0.0, sxx = 0.0, see = 0.0;
    for (int k = 0; k < nl; k++) {
      const double v = xs[k * S + l], e = v - t;
      sx += v;
      sxx += v * v;
      see += e * e;
    }
    if (l >= 3 && l < 7) {
      see = 0.0;  // orientation: the rotation-vector error (slot 6 stays 0)
      if (l < 6)
        for (int k = 0; k < nl; k++) see += pe[k * 5 + (l - 3)];
    }
    o[l] = sx;
    o[S + l] = sxx;
    o[2 * S + l] = see;
  } else if (l < S + 2) {
    double a = 0.0;
    for (int k = 0; k < nl; k++) a += pe[k * 5 + 3 + (l - S)];
    o[3 * S + (l - S)] = a;
  }
}

// out[s] = sum over the nblk partial rows, block s: thread t takes rows t, t + 256, ...
// then a fixed LDS tree; the result does not depend on timing
template <int DOF>
__global__ __launch_bounds__(256) void k_pose_stats_sum(const double* part, int64_t nblk, int nout, double* out) {
  __shared__ double red[256];
  const int s = blockIdx.x, t = threadIdx.x;
  double acc = 0.0;
  for (int64_t k = t; k < nblk; k += 256) acc += part[k * nout + s];
  red[t] = acc;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) out[s] = red[0];
}


#endif  // UWVK_POSE_KERNEL_BODIES

}  // namespace uwvk
