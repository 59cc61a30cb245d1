// uwvk_psp2_dev.hpp — the PSP PoseUKF epoch with TWO instances per wavefront
// (VERDICT r04 next #3).  The one-instance kernel (uwvk_psp_dev.hpp) keeps a
// 64-lane wave on one filter: its row phases use 53 of 64 lanes, but its
// sigma-point phases use 31 (predict) or 13 (update) and its wave-uniform
// chains (the mean's exp / product, the points' SO3 algebra) occupy all 64
// lanes for one instance's scalar work.  Here a wave owns instances A and B
// (Sigma~ of each in its own PspSmem, 25.6 KB per wave):
//   - row phases (partial Cholesky, L_a Delta, the A-coupled rows, the Q band,
//     H / P / G, the gain, Sigma~ -= C~ K~^T, apply_delta, the mean update) run
//     for A on all 64 lanes, then for B, with the one-instance code unchanged;
//   - point phases (sigma points and the process / measurement models, the
//     manifold mean, the sums over the points, Delta / Dz staging) run once
//     for both: lanes 0..31 hold A's points, lanes 32..63 B's (the predict's 31
//     and the update's 13 points fit a half), and per-instance uniform values
//     come from the half's own lanes (two readlanes per value).
// The arithmetic per instance is the one-instance kernel's, term by term (the
// same expressions in the same order), so results are bitwise those of
// k_psp_epoch on every instance (tests/test_gpu_pair.py).  Occupancy: LDS
// holds 6 waves per CU (12 instances, as before), i.e. 1.5 waves per SIMD
// instead of 3.
#pragma once
#include "uwvk_psp_dev.hpp"

namespace uwvk {
namespace psp2 {
using namespace psp;

// the half a lane belongs to (lanes 32..63: instance B), as a lane mask
UWVK_DEV bool hi_half(int l) { return LANE_IF(l, l >= 32); }

// value of lane j of each half, in every lane of that half (j compile-time)
UWVK_DEV double hb_d(double v, int j, bool hi) {
  const double a = readlane_d(v, j), b = readlane_d(v, 32 + j);
  return hi ? b : a;
}

// sums over lanes [0, NL) of each half (the other lanes must pass 0): DPP row
// sums, row_bcast:15 joining rows 0/1 and 2/3; sA / sB are uniform (SGPR) values
template <int NL>
UWVK_DEV void half_sum_dpp(double v, double& sA, double& sB) {
  static_assert(NL <= 32, "half");
  double s = v + dpp_d<0x111, 0xf, 0xf>(v);   // row_shr:1
  s = s + dpp_d<0x112, 0xf, 0xf>(v);          // row_shr:2
  s = s + dpp_d<0x113, 0xf, 0xf>(v);          // row_shr:3
  s = s + dpp_d<0x114, 0xf, 0xe>(s);          // row_shr:4, banks 1-3
  s = s + dpp_d<0x118, 0xf, 0xc>(s);          // row_shr:8, banks 2-3
  if constexpr (NL <= 16) {
    sA = readlane_d(s, 15);
    sB = readlane_d(s, 47);
  } else {
    s = s + dpp_d<0x142, 0xa, 0xf>(s);        // row_bcast:15, rows 1,3: lanes 31 / 63 hold the half totals
    sA = readlane_d(s, 31);
    sB = readlane_d(s, 63);
  }
}

// lds_sums per half: lane 32 h + STRIDE c (c < NL) writes v[i] to its
// instance's buf_h[i NL + c]; lane 32 h + i (i < R) adds row i; outA / outB
// uniform.  The per-instance sums are bitwise lds_sums' (same tree).
template <int R, int NL, int STRIDE>
UWVK_DEV void lds_sums2(const double (&v)[R], double* buf, int p, double (&outA)[R], double (&outB)[R]) {
  static_assert(NL % 2 == 0 && R * NL <= 115 && R <= 32, "transpose buffer (PG::STG)");
  const int c = p / STRIDE;
  if (p % STRIDE == 0 && c < NL) {
#pragma unroll
    for (int i = 0; i < R; i++) buf[i * NL + c] = v[i];
  }
  wsync();
  const double* row = buf + (p < R ? p : 0) * NL;
  double q[NL / 2];
#pragma unroll
  for (int k = 0; k < NL / 2; k++) q[k] = row[2 * k] + row[2 * k + 1];
#pragma unroll
  for (int w = 1; w < NL / 2; w *= 2)
#pragma unroll
    for (int k = 0; k + w < NL / 2; k += 2 * w) q[k] += q[k + w];
#pragma unroll
  for (int i = 0; i < R; i++) {
    outA[i] = readlane_d(q[0], i);
    outB[i] = readlane_d(q[0], 32 + i);
  }
}

// gen_rows for half-local point index p = l & 31 (the lane masks over l & 31)
template <class RL, int DOF, int K, int SR>
UWVK_DEV void gen_rows2(const double* mu, const double* stg, int p, double x[Lay<DOF>::store]) {
  using L = Lay<DOF>;
#pragma unroll
  for (int s = 0; s < L::store; s++) x[s] = mu[s];
  if constexpr (K > 0) {
    const bool in = LANE_IF(i, (i & 31) < 2 * K);
    const int j = in ? (p >> 1) : 0;
    const double sg = in ? (LANE_IF(i, (i & 1) != 0) ? -1.0 : 1.0) : 0.0;
    double v[3] = {0.0, 0.0, 0.0};
    gen_rows_q<RL, DOF, K, 0>(mu, stg, j, sg, v, x);
    if constexpr (has_rot<RL>()) {
      double e[4];
      so3_exp_psp(v, e);
      qplus_psp<SR>(e, mu + L::s_quat, x + L::s_quat);
    }
  }
}

// ---------------------------------------------------------------------------
// predict: per-instance front (noise shaping from the mean, partial Cholesky)
// ---------------------------------------------------------------------------
template <int DOF>
struct PredFront {
  double a[PG<DOF>::KP];  // row l's L_a
  double qo;              // lane a*3+b (< 9): (R Q_ori R^T)[a][b]
  double wv_add;
  bool ok;
};

template <int DOF>
UWVK_DEV void predict_front(PspSmem<DOF>& sm, const PoseShared& sh, double dt, double ds, PredFront<DOF>& f) {
  using L = Lay<DOF>;
  constexpr int K = PG<DOF>::KP;
  const int l = olane();
  f.qo = 0.0;
  if (LANE_IF(l, l < 9)) {
    double R[9];
    qmatrix(sm.mu + L::s_quat, R);
    const int r = l / 3, c = l % 3;
    double Rr[3], Rc[3];
#pragma unroll
    for (int m = 0; m < 3; m++) {
      Rr[m] = sel3(R[m], R[3 + m], R[6 + m], r);
      Rc[m] = sel3(R[m], R[3 + m], R[6 + m], c);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      double u = 0.0;
#pragma unroll
      for (int m = 0; m < 3; m++) u += Rr[m] * sh.q_ori[m * 3 + k];
      s += u * Rc[k];
    }
    f.qo = s;
  }
  const double vs0 = sm.mu[L::s_vel], vs1 = sm.mu[L::s_vel + 1], vs2 = 10 * sm.mu[L::s_vel + 2];
  f.wv_add = sh.p.water_velocity_scale * (vs0 * vs0 + vs1 * vs1 + vs2 * vs2) * dt;
  f.ok = pchol<DOF, K, PredRows>(sm.S, l, f.a, ds, sm.stg);
}

// the paired point phases' per-instance results (uniform values)
struct PredMid {
  double mq[4];  // manifold mean of the predicted orientation
  double oo[6];  // 1/2 sum of the weighted deviation products (ori x ori)
};

// the point phases for both instances: sigma points (lanes 32 h + p, p <= 2K),
// orientation through the process model, manifold mean, deviations, the
// ori x ori sums and Delta_j staged in each instance's stg
template <int DOF, int SR>
UWVK_DEV void predict_points2(PspSmem<DOF>& smA, PspSmem<DOF>& smB, const PoseShared& sh, const ProcCtx& pcA,
                              const ProcCtx& pcB, PredMid& mA, PredMid& mB) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int K = G::KP;
  const int l = olane();
  const bool hi = hi_half(l);
  const int p = l & 31;
  PspSmem<DOF>* sp = hi ? &smB : &smA;
  ProcCtx pc;  // the point lane's inputs: its instance's rotation rate, dt
#pragma unroll
  for (int k = 0; k < 3; k++) pc.w[k] = hi ? pcB.w[k] : pcA.w[k];
  pc.dt = pcA.dt;
  const bool pt = LANE_IF(i, (i & 31) < 2 * K), ctr = LANE_IF(i, (i & 31) == 2 * K);
  double o[4];
  {
    double x[L::store];
    gen_rows2<PredRows, DOF, K, SR>(sp->mu, sp->stg + STG_ROWS, p, x);
    proc_orientation<DOF, SR>(x, sh, pc, o);
  }
  constexpr double wc = 1.0 + 2.0 * (DOF - K);
  double mq[4];
#pragma unroll
  for (int i = 0; i < 4; i++) mq[i] = hb_d(o[i], 2 * K, hi);
  {
    // each instance iterates until its own |delta| <= 1e-6 (ukfom); the wave
    // runs until both have, a finished half keeping its mean
    bool runA = true, runB = true;
    int itA = 0, itB = 0;
    do {
      double d[3];
      qboxminus_psp<SR>(o, mq, d);
      const double w = pt ? 1.0 : (ctr ? wc : 0.0);
      double nA = 0.0, nB = 0.0, dh[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        double sA, sB;
        half_sum_dpp<2 * K + 1>(w * d[i], sA, sB);
        sA = sA * (1.0 / (double)G::N);
        sB = sB * (1.0 / (double)G::N);
        nA += sA * sA;
        nB += sB * sB;
        dh[i] = hi ? sB : sA;
      }
      double e[4], q[4];
      so3_exp_psp(dh, e);
      qplus_psp<SR>(e, mq, q);
      const bool upd = hi ? runB : runA;
#pragma unroll
      for (int i = 0; i < 4; i++) mq[i] = upd ? q[i] : mq[i];
      runA = runA && nA > 1e-12 && ++itA < 10000;
      runB = runB && nB > 1e-12 && ++itB < 10000;
    } while (runA || runB);
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    mA.mq[i] = readlane_d(mq[i], 0);
    mB.mq[i] = readlane_d(mq[i], 32);
  }
  double d[3];
  qboxminus_psp<SR>(o, mq, d);
  {
    const double w = pt ? 1.0 : (ctr ? wc : 0.0);
    double v[6];
    int k = 0;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) {
        const double t = w * d[i] * d[j];
        v[k++] = t + swap_pair_d(t);
      }
    lds_sums2<6, 16, 2>(v, sp->stg, p, mA.oo, mB.oo);
#pragma unroll
    for (int i = 0; i < 6; i++) {
      mA.oo[i] = 0.5 * mA.oo[i];
      mB.oo[i] = 0.5 * mB.oo[i];
    }
  }
  double dd[3];
#pragma unroll
  for (int i = 0; i < 3; i++) dd[i] = d[i] - swap_pair_d(d[i]);
  constexpr int DS = 4, D0 = 1;
  static_assert(D0 + DS * K <= PG<DOF>::STG, "Delta (PG::STG)");
  wsync();  // the sums' reads of stg before Delta is written over them
  if (LANE_IF(i, (i & 1) == 0 && (i & 31) < 2 * K)) {
#pragma unroll
    for (int i = 0; i < 3; i++) sp->stg[D0 + (p >> 1) * DS + i] = dd[i];
  }
  wsync();
}

// the row phases of one instance after the paired points: X = 1/2 A L_a Delta,
// the A-coupled rows, the time scale, rows < 9, ori x ori, the Q band, the new
// mean.  The code of psp_predict from its Delta phase on, with QM = 1.
template <int DOF, int SR>
UWVK_DEV void predict_back(PspSmem<DOF>& sm, const PoseShared& sh, const ProcCtx& pc, double& ds, double& ids,
                           const LaneQ& lq, const PredFront<DOF>& f, const PredMid& m) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int K = G::KP;
  const int l = olane();
  const double dt = pc.dt, dt2 = dt * dt;
  double X[3];
  {
    double Y[3] = {0.0, 0.0, 0.0};
    constexpr int DS = 4, D0 = 1;
    double dn[3];
#pragma unroll
    for (int i = 0; i < 3; i++) dn[i] = sm.stg[D0 + i];
#pragma unroll
    for (int j = 0; j < K; j++) {
      double dj[3] = {dn[0], dn[1], dn[2]};
      if (j + 1 < K) {
#pragma unroll
        for (int i = 0; i < 3; i++) dn[i] = sm.stg[D0 + DS * (j + 1) + i];
      }
#pragma unroll
      for (int i = 0; i < 3; i++) Y[i] += f.a[j] * dj[i];
      asm volatile("" : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2])::"memory");
    }
    wsync();
    const int cp = proc_couple(l);
    const int src = cp >= 0 ? cp : l;
    const double ar = 1.0 + dt * pc.nt_tan;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const double yc = shfl_d(Y[i], src);
      X[i] = 0.5 * (LANE_IF(l, proc_couple(l) >= 0) ? (ar * Y[i] + dt * yc) : ar * Y[i]);
    }
  }
  constexpr int pv[6] = {0, 1, 2, 6, 7, 8};
  double nv[6];
  const int jl = l < DOF ? l : DOF - 1;
  const int jc = proc_couple(jl);
  const double aj = 1.0 + dt * pc.nt_tan;
  const int Tl = (jl * (jl + 1)) >> 1;
  const int jcc = jc >= 0 ? jc : jl;
  const int Tc = (jcc * (jcc + 1)) >> 1;
  const double cf = LANE_IF(l, proc_couple(l < DOF ? l : DOF - 1) >= 0) ? dt : 0.0;
  constexpr unsigned long long ml_r[6] = {col_ge_mask<DOF>(0, false), col_ge_mask<DOF>(1, false),
                                          col_ge_mask<DOF>(2, false), col_ge_mask<DOF>(6, false),
                                          col_ge_mask<DOF>(7, false), col_ge_mask<DOF>(8, false)};
  constexpr unsigned long long ml_rc[6] = {col_ge_mask<DOF>(6, false), col_ge_mask<DOF>(7, false),
                                           col_ge_mask<DOF>(8, false), col_ge_mask<DOF>(9, false),
                                           col_ge_mask<DOF>(10, false), col_ge_mask<DOF>(11, false)};
  constexpr unsigned long long mc_r[6] = {col_ge_mask<DOF>(0, true), col_ge_mask<DOF>(1, true),
                                          col_ge_mask<DOF>(2, true), col_ge_mask<DOF>(6, true),
                                          col_ge_mask<DOF>(7, true), col_ge_mask<DOF>(8, true)};
  constexpr unsigned long long mc_rc[6] = {col_ge_mask<DOF>(6, true), col_ge_mask<DOF>(7, true),
                                           col_ge_mask<DOF>(8, true), col_ge_mask<DOF>(9, true),
                                           col_ge_mask<DOF>(10, true), col_ge_mask<DOF>(11, true)};
#pragma unroll
  for (int q = 0; q < 6; q++) {
    const int r = pv[q], rc = proc_couple(r);
    const double t0 = fma(cf, sm.S[pidx_sel_b(r, jcc, Tc, LANE_IN(mc_r[q]))],
                          aj * (ds * sm.S[pidx_sel_b(r, jl, Tl, LANE_IN(ml_r[q]))]));
    const double t1 = fma(cf, sm.S[pidx_sel_b(rc, jcc, Tc, LANE_IN(mc_rc[q]))],
                          aj * (ds * sm.S[pidx_sel_b(rc, jl, Tl, LANE_IN(ml_rc[q]))]));
    nv[q] = t0 + dt * t1;
  }
  if (LANE_IF(l, l < DOF && scaled_dof(l))) {
    ds = aj * ds;
    double rc = __builtin_amdgcn_rcp(ds);
    rc = fma(rc, fma(-ds, rc, 1.0), rc);
    ids = fma(rc, fma(-ds, rc, 1.0), rc);
  }
  psync();
  // rows < 9 (lane-resident Q: sh.q_simple, the QM = 1 instantiation)
  if (LANE_IF(l, l < DOF && !(l >= 3 && l < 6))) {
    const bool jpv = LANE_IF(l, proc_couple(l < DOF ? l : DOF - 1) >= 0);
    constexpr unsigned long long smask[6] = {rows_store_mask<DOF>(0), rows_store_mask<DOF>(1),
                                             rows_store_mask<DOF>(2), rows_store_mask<DOF>(6),
                                             rows_store_mask<DOF>(7), rows_store_mask<DOF>(8)};
    constexpr unsigned long long gmask[6] = {col_ge_mask<DOF>(0, false), col_ge_mask<DOF>(1, false),
                                             col_ge_mask<DOF>(2, false), col_ge_mask<DOF>(6, false),
                                             col_ge_mask<DOF>(7, false), col_ge_mask<DOF>(8, false)};
#pragma unroll
    for (int q = 0; q < 6; q++)
      if (LANE_IN(smask[q])) {
        const int e = pidx_sel_b(pv[q], l, Tl, LANE_IN(gmask[q]));
        sm.S[e] = (nv[q] + 0.0) * ids;
      }
    if (jpv) sm.S[Tl + l] += lq.q0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      constexpr unsigned long long omask[3] = {col_ge_mask<DOF>(3, false), col_ge_mask<DOF>(4, false),
                                               col_ge_mask<DOF>(5, false)};
      const int e = pidx_sel_b(3 + i, l, Tl, LANE_IN(omask[i]));
      sm.S[e] = X[i] * ids;
    }
  }
  if (LANE_IF(l, l < 9 && (l / 3) >= (l % 3))) {
    const int a2 = l / 3, b2 = l % 3;
    sm.S[pidx(3 + a2, 3 + b2)] =
        sel6(m.oo[0], m.oo[1], m.oo[2], m.oo[3], m.oo[4], m.oo[5], a2 * (a2 + 1) / 2 + b2) + dt2 * f.qo;
  }
  {
    constexpr int R0 = 9;
    const int bw = sh.q_bw;
    double qw4[4] = {sh.q_wv[0], sh.q_wv[1], sh.q_wv[2], sh.q_wv[3]};
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+s"(qw4[i]));
    const int lc = l < DOF ? l : DOF - 1;
    const int T = (lc * (lc + 1)) >> 1;
    double v[3], fv[3];
    int e[3];
    bool w[3];
    double idk = ids;
    constexpr unsigned long long bandm[3] = {
        lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l >= R0; }),
        lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l - 1 >= R0; }),
        lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l - 2 >= R0; })};
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k > 0) idk = dpp_d<0x138, 0xf, 0xf>(idk);
      const int j = l - k;
      e[k] = T + (j >= 0 ? (j <= lc ? j : lc) : 0);
      v[k] = sm.S[e[k]];
      double q = k == 0 ? lq.q0 : (k == 1 ? lq.q1 : lq.q2);
      if (k == 0 && LANE_IF(l, l >= L::d_wv && l < L::d_wv + 4)) {
        const int iw = l - L::d_wv;
        const double qw = iw == 0 ? qw4[0] : (iw == 1 ? qw4[1] : (iw == 2 ? qw4[2] : qw4[3]));
        q = dt2 * (qw + f.wv_add);
      }
      w[k] = LANE_IN(bandm[k]) && k <= bw && q != 0.0;
      fv[k] = q * (ids * idk);
    }
#pragma unroll
    for (int k = 0; k < 3; k++)
      if (w[k]) sm.S[e[k]] = v[k] + fv[k];
  }
  double mv = proc_vect_lane(l & 63, flat(sm) + kFlatMu<DOF>, pc);
  asm volatile("" : "+v"(mv));
  psync();
  if (LANE_IF(l, l < L::store && !(l >= 3 && l < 7))) sm.mu[l] = mv;
  if (LANE_IF(l, l < 4)) sm.mu[3 + l] = l == 0 ? m.mq[0] : (l == 1 ? m.mq[1] : (l == 2 ? m.mq[2] : m.mq[3]));
  psync();
}

// ---------------------------------------------------------------------------
// update: paired point phases, then the per-instance algebra
// ---------------------------------------------------------------------------
template <int M, int NC>
struct UpdMid {
  double zc[M];                  // z at the centre point (mu)
  double sums[M + M * (M + 1) / 2];
  double Hs[M][NC > 0 ? NC : 1];  // the affine part's Jacobian at mu
};

template <int DOF, int SR, class HM>
UWVK_DEV void update_points2(PspSmem<DOF>& smA, PspSmem<DOF>& smB, const HM& hm, UpdMid<HM::M, HM::NC>& uA,
                             UpdMid<HM::M, HM::NC>& uB) {
  using L = Lay<DOF>;
  constexpr int M = HM::M, K = HM::K, NC = HM::NC, NCA = NC > 0 ? NC : 1;
  static_assert(K > 0 && 2 * K + 1 <= 32, "points in a half");
  const int l = olane();
  const bool hi = hi_half(l);
  const int p = l & 31;
  PspSmem<DOF>* sp = hi ? &smB : &smA;
  double zp[M];
  {
    double x[L::store];
    gen_rows2<HM, DOF, K, SR>(sp->mu, sp->stg + STG_ROWS, p, x);
    hm.eval(x, zp);
  }
  double zc[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    uA.zc[i] = readlane_d(zp[i], 2 * K);
    uB.zc[i] = readlane_d(zp[i], 32 + 2 * K);
    zc[i] = hi ? uB.zc[i] : uA.zc[i];
  }
  {
    double H[M][NCA];
    hm.jac(sp->mu, H);
#pragma unroll
    for (int i = 0; i < M; i++)
#pragma unroll
      for (int t = 0; t < NC; t++) {
        uA.Hs[i][t] = readlane_d(H[i][t], 0);
        uB.Hs[i][t] = readlane_d(H[i][t], 32);
      }
  }
  // P (lane 32 h + i K + j) and the sums over the 2K point lanes of each half
  double Pl = 0.0;
  {
    const int q = LANE_IF(i, (i & 31) < M * K) ? p : 0;
    const int i = q / K, j = q - (q / K) * K;
#pragma unroll
    for (int t = 0; t < NC; t++) {
      double hA = uA.Hs[0][t], hB = uB.Hs[0][t];
#pragma unroll
      for (int ii = 1; ii < M; ii++) {
        hA = (i == ii) ? uA.Hs[ii][t] : hA;
        hB = (i == ii) ? uB.Hs[ii][t] : hB;
      }
      Pl += (hi ? hB : hA) * sp->stg[STG_ROWS + row_pos(HM::rows, HM::cols[t]) * K + j];
    }
  }
  constexpr int R = M + M * (M + 1) / 2;
  {
    double v[R];
#pragma unroll
    for (int i2 = 0; i2 < M; i2++) v[i2] = zp[i2] - zc[i2];
    int k = M;
#pragma unroll
    for (int i2 = 0; i2 < M; i2++)
#pragma unroll
      for (int j2 = 0; j2 <= i2; j2++) v[k++] = v[i2] * v[j2];
    lds_sums2<R, 2 * K, 1>(v, sp->stg, p, uA.sums, uB.sums);
  }
  double zd[M];
#pragma unroll
  for (int i = 0; i < M; i++) zd[i] = zp[i] - swap_pair_d(zp[i]);
  // P and Dz staged in each instance's stg (free after the sums), as psp_update
  constexpr int PS = M == 3 ? 4 : M, P0 = M >= 2 ? 1 : 0;
  static_assert(P0 + 2 * PS * K <= PG<DOF>::STG, "P and Dz (PG::STG)");
  wsync();
  if (LANE_IF(i, (i & 31) < M * K)) sp->stg[P0 + (p % K) * PS + p / K] = Pl;
  if (LANE_IF(i, (i & 1) == 0 && (i & 31) < 2 * K)) {
#pragma unroll
    for (int i = 0; i < M; i++) sp->stg[P0 + PS * K + (p >> 1) * PS + i] = zd[i];
  }
  wsync();
}

// psp_update after its point phases, for one instance: the row algebra, the
// gain, the gate, Sigma~ -= C~ K~^T and apply_delta (the one-instance code)
template <int DOF, int SR, class HM>
UWVK_DEV bool update_back(PspSmem<DOF>& sm, const double (&z)[HM::M], const double (&Rm)[HM::M * HM::M], int gate,
                          const UpdMid<HM::M, HM::NC>& u, const double (&a)[HM::K], bool cok, bool* ok, double ds,
                          double ids) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int M = HM::M, K = HM::K, NC = HM::NC;
  const int l = olane();
  constexpr double wc = 1.0 + 2.0 * (DOF - K);
  double S[M * M], zb[M], e[M];
  {
    double m[M];
#pragma unroll
    for (int i2 = 0; i2 < M; i2++) {
      m[i2] = u.sums[i2] * (1.0 / (double)G::N);
      zb[i2] = u.zc[i2] + m[i2];
      e[i2] = u.zc[i2] - zb[i2];
    }
    int k = M;
#pragma unroll
    for (int i2 = 0; i2 < M; i2++)
#pragma unroll
      for (int j2 = 0; j2 <= i2; j2++) {
        const double s = u.sums[k++] - m[i2] * u.sums[j2] - m[j2] * u.sums[i2] + (2.0 * K) * m[i2] * m[j2];
        S[i2 * M + j2] = 0.5 * (s + wc * e[i2] * e[j2]);
      }
  }
  const int rl = l < DOF ? l : DOF - 1;
  const int Trl = (rl * (rl + 1)) >> 1;
  double Gr[M];
#pragma unroll
  for (int i = 0; i < M; i++) Gr[i] = 0.0;
#pragma unroll
  for (int t = 0; t < NC; t++) {
    double s = sm.S[pidx_sel(HM::cols[t], rl, Trl)];
    if (scaled_dof(HM::cols[t])) s = s * readlane_d(ds, HM::cols[t]);
#pragma unroll
    for (int i = 0; i < M; i++) Gr[i] = hfma(u.Hs[i][t], s, Gr[i]);
  }
#pragma unroll
  for (int i = 0; i < M; i++) Gr[i] = Gr[i] * ds;
  double Gl[M], C[M];
  {
    constexpr int PS = M == 3 ? 4 : M, P0 = M >= 2 ? 1 : 0;
    double g[M], c[M];
#pragma unroll
    for (int i = 0; i < M; i++) {
      g[i] = Gr[i];
      c[i] = 0.0;
    }
#pragma unroll
    for (int j = 0; j < K; j++) {
      double pj[M], zj[M];
#pragma unroll
      for (int i = 0; i < M; i++) {
        pj[i] = sm.stg[P0 + j * PS + i];
        zj[i] = sm.stg[P0 + PS * K + j * PS + i];
      }
#pragma unroll
      for (int i = 0; i < M; i++) {
        g[i] -= a[j] * pj[i];
        c[i] += a[j] * zj[i];
        asm volatile("" : "+v"(g[i]), "+v"(c[i])::"memory");
      }
    }
    wsync();
#pragma unroll
    for (int i = 0; i < M; i++) {
      Gl[i] = g[i];
      C[i] = g[i] + 0.5 * c[i];
    }
  }
#pragma unroll
  for (int i = 0; i < M; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      double hg = 0.0;
#pragma unroll
      for (int t = 0; t < NC; t++) hg = hfma(u.Hs[i][t], readlane_d(Gl[j], HM::cols[t]), hg);
      const double s = S[i * M + j] + hg;
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
    double uu = 0.0;
#pragma unroll
    for (int i = 0; i < M; i++) uu += nu[i] * Si[i * M + j];
    d2 += uu * nu[j];
  }
  *ok = cok;
  const bool accept = gate == 0 ? true : !(d2 > kD2P95);
  if (!accept) return false;
  psync();
  double dl = 0.0;
#pragma unroll
  for (int i = 0; i < M; i++) dl += Kg[i] * nu[i];
  double Ct[M], Kt[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    Ct[i] = C[i] * ids;
    Kt[i] = Kg[i] * ids;
  }
  psync();
  rankm_mfma_o<DOF, M>(sm.S, sm.stg, Ct, Kt, l);
  psync();
  {
    const double dv[3] = {readlane_d(dl, 3), readlane_d(dl, 4), readlane_d(dl, 5)};
    double R[9], eq[4];
    so3_exp_psp(dv, eq);
    {
      const double tq[4] = {eq[0], SR ? -eq[1] : eq[1], SR ? -eq[2] : eq[2], SR ? -eq[3] : eq[3]};
      qmatrix(tq, R);
    }
    double nb;
    {
      const int lc = l < DOF ? l : DOF - 1;
      const int Tl = (lc * (lc + 1)) >> 1;
      const int e0 = pidx_sel_b(3, lc, Tl, LANE_IN(col_ge_mask<DOF>(3, false))),
                e1 = pidx_sel_b(4, lc, Tl, LANE_IN(col_ge_mask<DOF>(4, false))),
                e2 = pidx_sel_b(5, lc, Tl, LANE_IN(col_ge_mask<DOF>(5, false)));
      double s0 = sm.S[e0], s1 = sm.S[e1], s2 = sm.S[e2];
      asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2));
      double B[9];
#pragma unroll
      for (int uu = 0; uu < 3; uu++)
#pragma unroll
        for (int v = 0; v < 3; v++) B[uu * 3 + v] = sm.S[pidx(3 + uu, 3 + v)];
      const int r = l / 3, c = l % 3;
      double sb = 0.0;
#pragma unroll
      for (int uu = 0; uu < 3; uu++) {
        double t = 0.0;
#pragma unroll
        for (int v = 0; v < 3; v++) t += B[uu * 3 + v] * sel3(R[v], R[3 + v], R[6 + v], c);
        sb += sel3(R[uu], R[3 + uu], R[6 + uu], r) * t;
      }
      nb = sb;
      double n3[3];
#pragma unroll
      for (int i = 0; i < 3; i++) n3[i] = R[i * 3] * s0 + R[i * 3 + 1] * s1 + R[i * 3 + 2] * s2;
      if (LANE_IF(l, l < DOF && !(l >= 3 && l < 6))) {
        sm.S[e0] = n3[0];
        sm.S[e1] = n3[1];
        sm.S[e2] = n3[2];
      }
    }
    const double dsh = dpp_d<0x138, 0xf, 0xf>(dl);
    double mnew = flat(sm)[kFlatMu<DOF> + (l & 63)] + 1.0 * (LANE_IF(l, l < 3) ? dl : dsh);
    asm volatile("" : "+v"(mnew));
    double qn[4];
    qplus_psp<SR>(eq, sm.mu + L::s_quat, qn);
    psync();
    if (LANE_IF(l, l < 9 && (l / 3) >= (l % 3))) sm.S[pidx(3 + l / 3, 3 + l % 3)] = nb;
    if (LANE_IF(l, l < L::store && !(l >= 3 && l < 7))) sm.mu[l] = mnew;
    if (LANE_IF(l, l < 4)) sm.mu[3 + l] = qn[l];
    psync();
  }
  return true;
}

// one measurement update of kind HM on both instances (accept-any or d2p95):
// returns the two gate decisions in accA / accB
template <int DOF, int SR, class HM>
UWVK_DEV void psp2_update(PspSmem<DOF>& smA, PspSmem<DOF>& smB, const double (&zA)[HM::M],
                          const double (&zB)[HM::M], const double (&Rm)[HM::M * HM::M], int gate, const HM& hm,
                          bool* okA, bool* okB, bool* accA, bool* accB, double dsA, double idsA, double dsB,
                          double idsB) {
  constexpr int K = HM::K;
  const int l = olane();
  double aA[K], aB[K];
  const bool cA = pchol<DOF, K, HM>(smA.S, l, aA, dsA, smA.stg);
  const bool cB = pchol<DOF, K, HM>(smB.S, l, aB, dsB, smB.stg);
  UpdMid<HM::M, HM::NC> uA, uB;
  update_points2<DOF, SR, HM>(smA, smB, hm, uA, uB);
  *accA = update_back<DOF, SR, HM>(smA, zA, Rm, gate, uA, aA, cA, okA, dsA, idsA);
  *accB = update_back<DOF, SR, HM>(smB, zB, Rm, gate, uB, aB, cB, okB, dsB, idsB);
}

template <int DOF, int SR>
UWVK_DEV void psp2_predict(PspSmem<DOF>& smA, PspSmem<DOF>& smB, const PoseShared& sh, const ProcCtx& pcA,
                           const ProcCtx& pcB, double& dsA, double& idsA, double& dsB, double& idsB,
                           const LaneQ& lq, bool* okA, bool* okB) {
  PredFront<DOF> fA, fB;
  predict_front<DOF>(smA, sh, pcA.dt, dsA, fA);
  predict_front<DOF>(smB, sh, pcB.dt, dsB, fB);
  PredMid mA, mB;
  predict_points2<DOF, SR>(smA, smB, sh, pcA, pcB, mA, mB);
  predict_back<DOF, SR>(smA, sh, pcA, dsA, idsA, lq, fA, mA);
  predict_back<DOF, SR>(smB, sh, pcB, dsB, idsB, lq, fB, mB);
  *okA = fA.ok;
  *okB = fB.ok;
}

}  // namespace psp2
}  // namespace uwvk
