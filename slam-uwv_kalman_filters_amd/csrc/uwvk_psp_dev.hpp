// uwvk_psp_dev.hpp — partitioned sigma-point (PSP) PoseUKF: the same unscented
// transform as ukfom's (frozen spec), evaluated in O(n^2) per step.
//
// Why this is exact.  ukfom spreads X_0 = mu, X_{2j+1,2j+2} = mu [+] +-L_j with
// L the lower Cholesky factor of Sigma.  Let a model g (process model or
// measurement function) depend NON-affinely only on tangent DOFs < k (for fixed
// values of those, g is affine in the rest).  Column j >= k of a lower
// triangular L is zero in rows < k, so X_{j,+-} agrees with mu bitwise on every
// DOF g is non-affine in, and g(X_{j,+-}) = g(mu) +- J L_j with J the constant
// Jacobian of the affine part.  Substituting into ukfom's mean (weights 1/N) and
// covariances (weight 1/2, all 2n+1 points) gives, in exact arithmetic:
//   predict (k = 15: orientation depends on pos.x, q, gyro bias):
//     lin x lin = A Sigma A^T          (A: I + dt couplings + decays)
//     ori x lin = 1/2 A L_a Delta       (Delta_j = d_{j+} - d_{j-}, j < k)
//     ori x ori = 1/2 [sum_{2k pts} d d^T + (1 + 2(n-k)) c c^T]
//   update (k per model, H = Jacobian of the affine part at mu):
//     zbar = z_0 + (1/N) sum_{2k pts} (z_p - z_0)
//     S = 1/2 [sum_{2k} dz dz^T + (1 + 2(n-k)) e e^T] + H (Sigma - L_a L_a^T) H^T + R
//     C = 1/2 sum_{j<k} L_j (z_{j+} - z_{j-})^T + (Sigma - L_a L_a^T) H^T
// with L_a the first k columns of L (a k-step partial Cholesky).  Only 2k+1
// model evaluations and O(n^2) covariance algebra remain; results equal the
// literal spread to rounding (parity tests run both paths against the oracle).
// The literal path (uwvk_pose_dev.hpp) stays selectable: UWVK_OPT_DENSE_SIGMA.
//
// Both SO3 sides (template parameter SR, UWVK_OPT_SO3_RIGHT).  Nothing above
// depends on which side the orientation [+] multiplies: a point with a zero
// orientation component is mu on that block under q exp(0) and exp(0) q alike,
// so the points j >= k still agree with mu on every non-affine DOF, and the
// models' affine Jacobians do not involve the orientation.  The side enters
// only where a quaternion is combined: the 2k points' orientation, the process
// model's orientation step, the manifold mean and the deviations (qplus_psp /
// qboxminus_psp), and apply_delta's T (R(exp d) on the left, R(exp d)^T on the
// right; see psp_update).
//
// Execution: one wavefront (64 lanes) per filter instance, Sigma packed
// (lower triangle, row i at i(i+1)/2) in LDS for the whole multi-epoch run.
#pragma once
#include <cstddef>

#include "uwvk_pose_dev.hpp"

// r05: the compile-time A/B knobs of rounds 1-4 (PSP_*: lane-limited wave
// sums, LDS broadcasts, the three rank-M MFMA forms, lane masks, SGPR series
// constants, ...) are resolved to the measured winners; the ablation and
// hot-path-only diagnostics are gone from the product source.  The rejected
// arms, their measurements and the last commit that still builds them are
// listed in profiles/EXPERIMENTS.md ("r05: knob pruning").

// PSP_PAIR (r06, the pair translation unit uwvk_psp_pair.hip): TWO instances
// per wave, instance h = lane >> 5 on the 32 lanes [32 h, 32 h + 32), each with
// its own PspSmem; every routine below then works on the instance-local lane
// l & 31 (olane), builds its lane masks for the 32 local lanes of both halves
// (lane_mask / LANE_IN), reads a value of local lane j of its own half with
// hread (two readlanes and a select instead of one readlane), sums within a
// half (wave_sum_dpp), and runs Sigma~ -= C~ K~^T as a lane-per-row FMA sweep
// (rankm_rows: one MFMA tile spans all 64 lanes).  The code is compiled there
// under PSP_NS = psp2; the single-instance kernels (uwvk_psp_k.hip) are
// PSP_PAIR 0, namespace psp.
#ifndef PSP_PAIR
#define PSP_PAIR 0
#endif
#ifndef PSP_NS
#define PSP_NS psp
#endif

namespace uwvk {
namespace PSP_NS {

constexpr int kLanes = PSP_PAIR ? 32 : 64;  // lanes per instance

// (r05) a partial Cholesky is one serial chain (pivot readlane -> rsqrt ->
// scale -> column broadcast -> update, per column): the wave in it runs at
// raised issue priority (s_setprio 1) so that its next step issues ahead of the
// SIMD's other waves; interleaved A/B, six rounds: 200 epochs 62.21-62.43 ->
// 61.86-62.04 ms, 20 epochs 6.56-6.63 -> 6.53-6.60 ms (profiles/r05/ab_prio/).
// The predict's X = 1/2 A L_a Delta loop (one LDS broadcast and FMA per j)
// likewise: 200 epochs 61.52-61.90 -> 61.27-61.66 ms, ten rounds, 20 epochs
// within noise (profiles/r05/ab_prio/round3-4.txt).  Raising it over the
// manifold mean, the update's points, the gain, apply_delta or the BodyEfforts
// factor did not help (same runs).
UWVK_DEV void chain_prio_hi() { __builtin_amdgcn_s_setprio(1); }
UWVK_DEV void chain_prio_lo() { __builtin_amdgcn_s_setprio(0); }

template <int DOF>
struct PG {
  static constexpr int NP = DOF * (DOF + 1) / 2;     // packed entries
  static constexpr int NSLOT = (NP + kLanes - 1) / kLanes;  // flat slots per lane
  static constexpr int N = 2 * DOF + 1;              // ukfom sigma points
  static constexpr int KP = 15;                      // predict: nonlinear prefix (pos.x .. gyro bias)
  // staging area (L_a rows for the point lanes, the Cholesky column, C~ halves,
  // LDS transposes): 115 doubles puts PspSmem<53> at 12,800 B, the most that
  // fits 12 one-wave workgroups on a gfx950 CU (tools/probe_lds_occupancy.hip:
  // 12,800 B -> 12 per CU, 13,056 B -> 11); the r01 layout (160) ran at 11
  static constexpr int STG = 115;
};

template <int DOF>
struct alignas(16) PspSmem {
  double S[PG<DOF>::NP];          // Sigma, packed lower triangle
  double mu[Lay<DOF>::store];     // mean (store layout)
  double stg[PG<DOF>::STG];       // staging (see PG::STG)
  // everything else (Delta, Dz, H, P, delta, offsets, the Q band) lives in
  // lane registers or uniform SGPRs
};
static_assert(sizeof(PspSmem<53>) <= 12800, "12 instances per CU");
// S, mu and stg are contiguous: every-lane loads that run past one member (the
// epilogue's slot loop, the mean's lanes >= store) land in the next one and are
// never stored.  Such reads go through flat(), a view of the whole PspSmem as
// one double array, not through an out-of-range index of a member array.
static_assert(offsetof(PspSmem<53>, mu) == sizeof(double) * PG<53>::NP, "mu follows S");
static_assert(offsetof(PspSmem<53>, stg) == sizeof(double) * (PG<53>::NP + Lay<53>::store), "stg follows mu");
static_assert(offsetof(PspSmem<26>, mu) == sizeof(double) * PG<26>::NP, "mu follows S");
static_assert(offsetof(PspSmem<26>, stg) == sizeof(double) * (PG<26>::NP + Lay<26>::store), "stg follows mu");
// (r06) the parameter-decoupled epoch kernel (PD).  A
// 53-DOF instance whose 27 model-parameter DOFs (inertia, linear and quadratic
// damping: tangent 19..45, store 20..46) are uncoupled from every other DOF and
// from each other -- their rows of Sigma are zero off the diagonal, as the
// reference's P0 and Q make them (PoseUKF.cpp:333-335, :417-422) and as the
// IMU / DVL / pressure / ADCP / position updates keep them -- evolves exactly
// as follows: the other 26 DOFs run the unscented transform of the 53-DOF
// filter (sigma-point weights of n = 53), and each parameter DOF alone decays
// toward its offset (PoseUKF.cpp:50-72) with A_ii^2 Sigma_ii + dt^2 Q_ii.  The
// PD kernel runs the 26-DOF layout (Lay<26>: the same DOFs in the same order)
// with the 53-DOF weights; parameter t lives in lane 27 + t: its time scale in
// the lane's ds / ids (the tail hand-off carries all 64 lanes), its Sigma~_ii
// and mean in LDS (PspSmemPD).  The zeros are never touched, so the results
// are those of the 53-DOF kernel up to the sign of zero entries.
constexpr int kPdLane0 = 27, kPdN = 27;  // parameter t in lane kPdLane0 + t
template <int DOF>
struct alignas(16) PspSmemPD : PspSmem<DOF> {
  double pS[32];  // Sigma~_ii of parameter t (time-scaled like Sigma~)
  double pm[32];  // its mean (store 20 + t of the 53-DOF layout)
};
template <int DOF, int PD>
struct SmemT {
  using type = PspSmem<DOF>;
};
template <int DOF>
struct SmemT<DOF, 1> {
  using type = PspSmemPD<DOF>;
};
template <int DOF>
UWVK_DEV double* pd_ptr(PspSmem<DOF>&) {
  return nullptr;
}
template <int DOF>
UWVK_DEV double* pd_ptr(PspSmemPD<DOF>& s) {
  return s.pS;  // pm at +32
}
// 26-layout tangent DOF / store index -> the 53-layout one (parameters removed)
UWVK_DEV constexpr int pd_dof(int d) { return d < 19 ? d : d + 27; }
UWVK_DEV constexpr int pd_store(int s) { return s < 20 ? s : s + 27; }

template <int DOF>
UWVK_DEV double* flat(PspSmem<DOF>& sm) {
  return reinterpret_cast<double*>(&sm);
}
template <int DOF>
UWVK_DEV const double* flat(const PspSmem<DOF>& sm) {
  return reinterpret_cast<const double*>(&sm);
}
template <int DOF>
constexpr int kFlatMu = PG<DOF>::NP;  // mu's offset in flat()

// pidx / unpack: uwvk_dev.hpp (the HBM layout is the same packed triangle)

// lane id that the optimiser cannot treat as loop-invariant: phases inside the
// multi-epoch loop recompute their lane-derived addresses instead of having
// LICM hoist hundreds of them out of the epoch loop (register blow-up)
UWVK_DEV int olane() {
  int l = PSP_PAIR ? ((int)threadIdx.x & 31) : (int)threadIdx.x;
  asm volatile("" : "+v"(l));
  return l;  // (restoring the range with l & 63 measured 1% slower)
}

// (r04) A condition on the lane id alone as a compile-time lane
// mask (one wave per instance: lane l is bit l of EXEC).  LANE_IF(l, expr)
// folds expr over the 64 lanes into a constant and hands it to
// inverse_ballot: an s_mov of the mask into an SGPR pair, instead of a v_cmp
// (plus the integer arithmetic on the laundered lane id) per use.  Every PSP
// kernel is one 64-lane wave per workgroup (__launch_bounds__(64)).
template <class F>
UWVK_DEV constexpr unsigned long long lane_mask(F f) {
  unsigned long long m = 0;
  for (int i = 0; i < 64; i++)
    if (f(PSP_PAIR ? (i & 31) : i)) m |= 1ull << i;  // pair: the local lane of either half
  return m;
}
// a mask built for local lanes 0..63 as the mask of both halves' local lanes
// 0..31 (PSP_PAIR; the identity otherwise)
UWVK_DEV constexpr unsigned long long rep_mask(unsigned long long m) {
  return PSP_PAIR ? ((m & 0xFFFFFFFFull) | ((m & 0xFFFFFFFFull) << 32)) : m;
}
// A 64-bit mask whose value is a sign-extended 32-bit number but not an
// inline constant (e.g. lanes >= 5: 0xffffffffffffffe0) was emitted by the
// compiler as s_mov_b64 with a 32-bit literal, which gfx950 ZERO-extends:
// lanes 32..63 came out clear (tools/probe_lmask.hip, profiles/r04/lmask/).
// Such masks are built from their two 32-bit halves through an opaque SGPR
// pair instead; every other mask is a plain constant.
UWVK_DEV constexpr bool mask_needs_split(unsigned long long m) {
  return m >= 0xFFFFFFFF80000000ull && m < 0xFFFFFFFFFFFFFFF0ull;
}
UWVK_DEV bool lane_in_split(unsigned long long m) {
  unsigned lo = (unsigned)m, hi = (unsigned)(m >> 32);
  asm volatile("" : "+s"(lo), "+s"(hi));
  return __builtin_amdgcn_inverse_ballot_w64(((unsigned long long)hi << 32) | lo);
}
template <unsigned long long M>
UWVK_DEV bool lane_const() {
  if constexpr (mask_needs_split(M)) return lane_in_split(M);
  else return __builtin_amdgcn_inverse_ballot_w64(M);
}
#define LANE_IF(l, expr)                                                                                        \
  ({                                                                                                            \
    constexpr unsigned long long m_ = ::uwvk::PSP_NS::lane_mask([](int l) constexpr { return (bool)(expr); }); \
    ::uwvk::PSP_NS::lane_const<m_>();                                                                           \
  })
#define LANE_IN(m)                                                                     \
  (::uwvk::PSP_NS::mask_needs_split(::uwvk::PSP_NS::rep_mask(m))                       \
       ? ::uwvk::PSP_NS::lane_in_split(::uwvk::PSP_NS::rep_mask(m))                    \
       : __builtin_amdgcn_inverse_ballot_w64(::uwvk::PSP_NS::rep_mask(m)))
// the upper half of the wave (PSP_PAIR: instance 1)
UWVK_DEV bool upper_half() { return lane_const<0xFFFFFFFF00000000ull>(); }
// local lane j's value of the lane's own instance: readlane (a uniform SGPR
// pair) with one instance per wave; PSP_PAIR: lane j or 32 + j by half
#if PSP_PAIR
// (r06) local lane J < 16 of each half by two DPP moves per dword:
// row_newbcast:J (every 16-lane row takes its lane J), then row_bcast:15 into
// rows 1 and 3 from rows 0 and 2 (row_mask 0xa; rows 0 and 2 keep their
// value): 4 VALU per double instead of four v_readlane and two selects
template <int J>
UWVK_DEV double hbc(double v) {
  static_assert(J >= 0 && J < 16, "row_newbcast lane");
  int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x150 + J, 0xf, 0xf, false);
  int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x150 + J, 0xf, 0xf, false);
  lo = __builtin_amdgcn_update_dpp(lo, lo, 0x142, 0xa, 0xf, false);
  hi = __builtin_amdgcn_update_dpp(hi, hi, 0x142, 0xa, 0xf, false);
  return __hiloint2double(hi, lo);
}
#endif
UWVK_DEV double hread(double v, int j) {
#if PSP_PAIR
  if (__builtin_constant_p(j) && j >= 0 && j < 16) {  // (r06: +12% / +8% at 20 / 200 epochs, profiles/r06/r06o/)
    switch (j) {
      case 0: return hbc<0>(v);
      case 1: return hbc<1>(v);
      case 2: return hbc<2>(v);
      case 3: return hbc<3>(v);
      case 4: return hbc<4>(v);
      case 5: return hbc<5>(v);
      case 6: return hbc<6>(v);
      case 7: return hbc<7>(v);
      case 8: return hbc<8>(v);
      case 9: return hbc<9>(v);
      case 10: return hbc<10>(v);
      case 11: return hbc<11>(v);
      case 12: return hbc<12>(v);
      case 13: return hbc<13>(v);
      case 14: return hbc<14>(v);
      default: return hbc<15>(v);
    }
  }
  const double a = readlane_d(v, j), b = readlane_d(v, 32 + j);
  return upper_half() ? b : a;
#else
  return readlane_d(v, j);
#endif
}
// global lane of local lane j of the lane's own instance (shuffles)
UWVK_DEV int hlane(int j) { return PSP_PAIR ? j + ((int)threadIdx.x & 32) : j; }
// lanes whose column j >= p, with j the lane clamped to the last DOF (jl) or its
// A-coupled column (jcc: pos -> vel, vel -> acc, else jl), for pidx_sel_b
UWVK_DEV constexpr int couple_c(int d) { return d < 3 ? d + 6 : (d >= 6 && d < 9 ? d + 3 : -1); }
template <int DOF>
UWVK_DEV constexpr unsigned long long col_ge_mask(int p, bool coupled) {
  unsigned long long m = 0;
  for (int l = 0; l < 64; l++) {
    const int jl = l < DOF ? l : DOF - 1, jc = couple_c(jl);
    const int j = coupled ? (jc >= 0 ? jc : jl) : jl;
    if (j >= p) m |= 1ull << l;
  }
  return m;
}
// rows_lt9: lanes storing entry (p, l): uncoupled lanes, or coupled ones at l <= p
template <int DOF>
UWVK_DEV constexpr unsigned long long rows_store_mask(int p) {
  unsigned long long m = 0;
  for (int l = 0; l < 64; l++) {
    const int jl = l < DOF ? l : DOF - 1;
    if (!(couple_c(jl) >= 0) || l <= p) m |= 1ull << l;
  }
  return m;
}
// lanes of a compile-time row list
template <class RL>
UWVK_DEV constexpr unsigned long long rows_mask() {
  unsigned long long m = 0;
  for (int k = 0; k < RL::NR; k++) m |= 1ull << RL::rows[k];
  return m;
}
// lanes of a measurement model's affine Jacobian columns (HM::cols, ascending)
template <class HM>
UWVK_DEV constexpr unsigned long long cols_mask() {
  unsigned long long m = 0;
  for (int k = 0; k < HM::NC; k++) m |= 1ull << HM::cols[k];
  for (int k = 1; k < HM::NC; k++)
    if (HM::cols[k] <= HM::cols[k - 1]) return 0;  // (not ascending: unusable, see the static_assert)
  return m;
}
template <class RL>
UWVK_DEV constexpr bool rows_ascending() {
  for (int k = 1; k < RL::NR; k++)
    if (RL::rows[k] <= RL::rows[k - 1]) return false;
  return true;
}

// ---------------------------------------------------------------------------
// DPP wave reductions (no LDS crossbar): row_shr 1/2/3 -> 4-lane sums,
// row_shr 4/8 with bank masks -> row sums in lane 15 of each row, row_bcast
// 15/31 -> the total in lane 63, read back as a uniform (SGPR) value.
// ---------------------------------------------------------------------------
template <int CTRL, int ROW, int BANK>
UWVK_DEV double dpp_d(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW, BANK, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW, BANK, true);
  return __hiloint2double(hi, lo);
}
// NL: lanes that may hold a non-zero term (the others must pass 0).  Sums over
// <= 16 lanes stop at the row total (lane 15), <= 32 lanes after row_bcast:15.
template <int NL = 64>
UWVK_DEV double wave_sum_dpp(double v) {
  double s = v + dpp_d<0x111, 0xf, 0xf>(v);   // row_shr:1
  s = s + dpp_d<0x112, 0xf, 0xf>(v);          // row_shr:2
  s = s + dpp_d<0x113, 0xf, 0xf>(v);          // row_shr:3
  s = s + dpp_d<0x114, 0xf, 0xe>(s);          // row_shr:4, banks 1-3
  s = s + dpp_d<0x118, 0xf, 0xc>(s);          // row_shr:8, banks 2-3
#if PSP_PAIR
  // within each 32-lane half: rows 0 / 2 end in lanes 15 / 47, rows 0+1 / 2+3 in 31 / 63
  static_assert(NL <= 32, "pair: one instance per 32-lane half");
  if constexpr (NL <= 16) return hread(s, 15);
  s = s + dpp_d<0x142, 0xa, 0xf>(s);          // row_bcast:15, rows 1,3
  return hread(s, 31);
#else
  if constexpr (NL <= 16) return readlane_d(s, 15);
  s = s + dpp_d<0x142, 0xa, 0xf>(s);          // row_bcast:15, rows 1,3
  if constexpr (NL <= 32) return readlane_d(s, 31);
  s = s + dpp_d<0x143, 0xc, 0xf>(s);          // row_bcast:31, rows 2,3
  return readlane_d(s, 63);
#endif
}
// ---------------------------------------------------------------------------
// Small-angle SO3 exp / log (the same maps as so3_exp / so3_log, evaluated by
// their Taylor series in the squared angle: no sqrt, sincos, atan2 or division
// in the common case; truncation < 1e-20 relative inside the thresholds; the
// library forms are the fallback).
// ---------------------------------------------------------------------------
// (r04) PSP_SCONST: a series coefficient as a uniform (SGPR) operand of its FMA.
// Without it every coefficient was rebuilt in a VGPR pair by two v_mov_b32 per
// use (~150 VALU per instance-epoch, on the kernel's bound unit); an empty asm
// pins the value to an SGPR pair, made by two s_mov_b32 on the scalar unit.
UWVK_DEV double sk(double c) {
  asm volatile("" : "+s"(c));
  return c;
}
UWVK_DEV void so3_exp_psp(const double v[3], double o[4]) {
  const double t2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
  if (t2 < 0.0625) {  // |v| < 0.25: h = |v|/2 < 0.125, u = h^2
    const double u = 0.25 * t2;
    // sin(h) / (2h) and cos(h), Horner in u; the next terms, u^6 / 13! and
    // u^6 / 12!, are < 3e-20 relative for u < 1/64 (r04: dropped)
    double s = u * sk(-1.0 / 39916800.0);
    s = s + sk(1.0 / 362880.0);
    s = fma(s, u, sk(-1.0 / 5040.0));
    s = fma(s, u, sk(1.0 / 120.0));
    s = fma(s, u, sk(-1.0 / 6.0));
    s = fma(s, u, 1.0);
    s = 0.5 * s;
    double c = u * sk(-1.0 / 3628800.0);
    c = c + sk(1.0 / 40320.0);
    c = fma(c, u, sk(-1.0 / 720.0));
    c = fma(c, u, sk(1.0 / 24.0));
    c = fma(c, u, -0.5);
    c = fma(c, u, 1.0);
    o[0] = c; o[1] = s * v[0]; o[2] = s * v[1]; o[3] = s * v[2];
  } else {
    so3_exp(v, o);
  }
}
UWVK_DEV void so3_log_psp(const double q[4], double o[3]) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  if (w < 0) { w = -w; x = -x; y = -y; z = -z; }
  const double n2 = x * x + y * y + z * z, w2 = w * w;
  if (n2 < 0.0025 * w2) {  // r = |v|/w < 0.05 (rotation < 0.1 rad)
    double iw = __builtin_amdgcn_rcp(w);  // w in (0.99, 1]: two Newton steps -> correctly rounded to ~1 ulp
    iw = fma(iw, fma(-w, iw, 1.0), iw);
    iw = fma(iw, fma(-w, iw, 1.0), iw);
    const double r2 = n2 * (iw * iw);
    // atan(r)/r = sum (-r^2)^k / (2k+1), k <= 6 (k = 7: < 5e-20 for r^2 < 0.0025)
    double a = r2 * sk(-1.0 / 13.0);
    a = fma(a, -r2, sk(1.0 / 11.0));
    a = fma(a, -r2, sk(1.0 / 9.0));
    a = fma(a, -r2, sk(1.0 / 7.0));
    a = fma(a, -r2, sk(1.0 / 5.0));
    a = fma(a, -r2, sk(1.0 / 3.0));
    a = fma(a, -r2, 1.0);
    const double k = 2.0 * a * iw;  // 2 atan2(|v|, w) / |v|
    o[0] = k * x; o[1] = k * y; o[2] = k * z;
  } else {
    so3_log(q, o);
  }
}
// SO3 [+] / [-] of side SR (a template parameter of every PSP kernel, DESIGN.md
// section 4.3): SR = 0 nav-frame (left), q [+] v = exp(v) q, a [-] b = log(a b^-1);
// SR = 1 body-frame (right, classic MTK SO3::boxplus), q [+] v = q exp(v),
// a [-] b = log(b^-1 a).  e = exp(v) is passed in.  The oracle's or_set_so3_right.
template <int SR>
UWVK_DEV void qplus_psp(const double e[4], const double q[4], double o[4]) {
  if constexpr (SR) qmul(q, e, o);
  else qmul(e, q, o);
}
template <int SR>
UWVK_DEV void qboxminus_psp(const double a[4], const double b[4], double o[3]) {
  double bc[4] = {b[0], -b[1], -b[2], -b[3]}, r[4];
  if constexpr (SR) qmul(bc, a, r);
  else qmul(a, bc, r);
  so3_log_psp(r, o);
}

// value of lane l ^ 1 (quad_perm [1,0,3,2])
UWVK_DEV double swap_pair_d(double v) { return dpp_d<0xb1, 0xf, 0xf>(v); }

// v_i for a lane-varying i as a select chain on scalars (a dynamically
// indexed private array would be placed in scratch memory, and a select
// chain over array elements is folded back into such an indexed load)
UWVK_DEV double sel3(double v0, double v1, double v2, int i) { return i == 0 ? v0 : (i == 1 ? v1 : v2); }
UWVK_DEV double sel6(double v0, double v1, double v2, double v3, double v4, double v5, int i) {
  return i < 3 ? sel3(v0, v1, v2, i) : sel3(v3, v4, v5, i - 3);
}

// pidx(p, j) for a compile-time p and lane-varying j, given Tj = j (j + 1) / 2
UWVK_DEV int pidx_sel(int p, int j, int Tj) { return j >= p ? Tj + p : p * (p + 1) / 2 + j; }
// the same with the branch given (a lane mask)
UWVK_DEV int pidx_sel_b(int p, int j, int Tj, bool ge) { return ge ? Tj + p : p * (p + 1) / 2 + j; }

UWVK_DEV void wsync() {  // LDS ordering point between the lanes of one wave
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// R sums over NL contributors at once (instead of R DPP reductions): lane
// l = STRIDE * c (c < NL) writes v[i] to buf[i * NL + c]; lane i < R adds row
// i by a pairwise tree; out[i] is read back as a uniform value.
template <int R, int NL, int STRIDE>
UWVK_DEV void lds_sums(const double (&v)[R], double* buf, int l, double (&out)[R]) {
  static_assert(NL % 2 == 0 && R * NL <= 115, "transpose buffer (PG::STG)");
  const int c = l / STRIDE;
  if (l % STRIDE == 0 && c < NL) {
#pragma unroll
    for (int i = 0; i < R; i++) buf[i * NL + c] = v[i];
  }
  wsync();
  const double* row = buf + (l < R ? l : 0) * NL;  // 8-B aligned only (ds_read2_b64 pairs)
  double p[NL / 2];
#pragma unroll
  for (int k = 0; k < NL / 2; k++) p[k] = row[2 * k] + row[2 * k + 1];
#pragma unroll
  for (int w = 1; w < NL / 2; w *= 2)
#pragma unroll
    for (int k = 0; k + w < NL / 2; k += 2 * w) p[k] += p[k + w];
#pragma unroll
  for (int i = 0; i < R; i++) out[i] = hread(p[0], i);
}

// phase boundary: the stamp of the diagnostic build, and (PSP_FAST & 4096) a
// fresh laundered lane id, so that lane masks are recomputed per phase (one
// v_cmp each) instead of being kept as SGPR pairs across the epoch, where they
// were spilled to VGPR lanes and reloaded (two v_readlane each) in every phase
#define PSP_PHASE(ph) \
  do {                \
    UWVK_STAMP(ph);   \
    l = olane();      \
  } while (0)

UWVK_DEV void psync() {  // LDS ordering point for the single wave of the block
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------------
// k-column partial Cholesky, lane r owns row r: a[c] = L[r][c] (0 above the
// diagonal).  Right-looking; L[c][J] is broadcast from lane c's registers.
// ---------------------------------------------------------------------------
// DOFs whose first-order Markov decay is carried by the time scale
// (Sigma = D Sigma~ D, D = diag(d)): gyro/acc bias, model parameters, water
// velocities, ADCP bias, density.  Position, orientation, velocity,
// acceleration and gravity keep d = 1.
UWVK_DEV constexpr bool scaled_dof(int d) { return d >= 12 && d != 18; }

// r04: broadcast reads from the staging area 16-byte aligned, so that pairs of
// doubles are one ds_read_b128 (4 LDS-array cycles, one address) instead of a
// ds_read2_b64 (8 cycles) with a per-pair address.  sm.stg starts 8 bytes past a
// 16-byte boundary (PspSmem: 11,448 + 432 B), so an odd stg index is aligned.
// The Cholesky column of step J is shifted by one slot when J + 1 is even; the
// predict's Delta_j and the update's P / Dz rows are padded to 4 per j.
// (LDS-array cycles per instance-epoch: 1,987 measured before, r04b lds pass.)
// column J broadcast through an LDS column (no readlanes); the rows the
// sigma-point lanes need (RL::rows) are staged in the same step: lane r with
// q = row_pos(r) writes L[r][J] to rows[q*K + J] (one write per column).
// piv: this step's pivot (an SGPR pair from the look-ahead readlane); with
// PSP_PIV_EARLY the look-ahead also takes the next pivot's rsqrt at once, so
// only the VGPR result crosses the step: the SGPR pair, held across the
// column update, was spilled to a VGPR lane and read back (2 v_writelane + 2
// v_readlane per column step, tools/spill_report.py).  The sign test rides on
// the rsqrt: rsqrt of a pivot <= 0 or NaN is NaN or +-inf, so chk += inv * 0
// is NaN exactly when some pivot failed piv > 0 (pchol tests chk once).
template <int K, int J>
UWVK_DEV void pchol_step_lds(double (&a)[K], int r, bool& ok, double* col, double* rows, int q, double piv,
                             double inv_in, double& chk) {
  if constexpr (J < K) {
    ok = ok && (piv > 0.0);
    const double inv = rsqrt_f64(piv);
    // lane J's own a[J] is the pivot (the look-ahead below evaluates the same
    // fma as the column update), so one product serves the diagonal too
    a[J] = LANE_IF(r, r >= J) ? a[J] * inv : 0.0;
    // look-ahead: the next pivot is lane J+1's a[J+1] - L[J+1][J]^2 (its own
    // registers), so its rsqrt need not wait for the column broadcast
    double pnext = 0.0, invn = 0.0;
    if constexpr (J + 1 < K) {
      pnext = hread(a[J + 1] - a[J] * a[J], J + 1);
    }
    if constexpr (J + 1 < K) {
      // col aliases the LAST staged row's not-yet-written slots J+1 .. K-1:
      // only L[c][J] for c > J is read, and that row's own L[.][c] lands in
      // slot c at step c, after this step's reads (one wave: LDS in order)
      // (PSP_LDS_ALIGN with PSP_STAGE_LATE: slot c + 1 when J + 1 is even, so
      // that the reads start on a 16-byte boundary; col is odd-aligned)
      // (PSP_CHOL_RL1: the next column's entry L[J+1][J] by readlane, the
      // LDS reads start at J + 2 and are aligned from there)
      constexpr int C0 = J + 1;
      double* const cj = col + (((C0 & 1) == 0) ? 1 : 0);
      // r04: every lane stores its a[J] to slot r: the slots read this step
      // are (J, K), which only the lanes r in (J, K) write; the others land in
      // slots that are not read now and that nothing else holds while the
      // factor runs (the rows area is written only after the last step).  The
      // address is one per-lane constant plus the step's immediate offset,
      // instead of a select per step (4 VALU)
      static_assert(64 + 1 <= 115, "column slots (PG::STG)");
      cj[r & 63] = a[J];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int c = C0; c < K; c++) a[c] -= a[J] * cj[c];
#pragma unroll
      for (int c = J + 1; c < K; c++) asm volatile("" : "+v"(a[c]));
    }
    pchol_step_lds<K, J + 1>(a, r, ok, col, rows, q, pnext, invn, chk);
  }
}

// staged rows of L_a start here inside sm.stg; the Cholesky column buffer is
// folded into the last staged row (pchol_step_lds)
constexpr int STG_ROWS = 0;

// panel Sigma[r][0..K) = d_r d_c Sigma~[r][c] (dl: this lane's d); stg: the
// staging area (the rows of RL::rows, the column buffer inside the last one)
template <int DOF, int K, class RL>
UWVK_DEV bool pchol(const double* S, int r, double (&a)[K], double dl, double* stg) {
  const int rr = r < DOF ? r : DOF - 1;
  // row rr from its packed start with immediate offsets: for c > rr this reads
  // a later (finite) entry of Sigma~, which the column steps never use (they
  // zero L[r][c] for r < c before it is read)
  const double* Sr = S + rr * (rr + 1) / 2;
#pragma unroll
  for (int c = 0; c < K; c++) a[c] = Sr[c] * (scaled_dof(c) ? dl * hread(dl, c) : dl);
  bool ok = true;
  // the staged-row slot of lane r is its rank among the staged rows (the row
  // list is ascending): the set bits of the constant row mask below the lane,
  // two v_mbcnt instead of a select per staged row
  static_assert(rows_ascending<RL>(), "RL::rows ascending");
  constexpr unsigned long long rm = rep_mask(rows_mask<RL>());
  int q = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(rm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)rm, 0u));
  if constexpr (PSP_PAIR) q -= upper_half() ? __builtin_popcount((unsigned)rm) : 0;  // the lower half's rows
  static_assert(RL::NR >= 1 && STG_ROWS + RL::NR * K <= 115, "staging area (PG::STG)");
  const double p0 = hread(a[0], 0);
  const double inv0 = rsqrt_f64(p0);
  double chk = fma(inv0, 0.0, 0.0);
  // the column buffer anywhere in the (not yet written) rows area; the rows are
  // staged after the last step, one lane-addressed run of K stores per row
  // lane, instead of one masked store (and its address product) per step
  pchol_step_lds<K, 0>(a, r, ok, stg + STG_ROWS, stg + STG_ROWS, q, p0, inv0, chk);
  if (LANE_IN(rows_mask<RL>())) {  // q >= 0
    double* rp = stg + STG_ROWS + q * K;
#pragma unroll
    for (int J = 0; J < K; J++) rp[J] = a[J];
  }
  psync();  // the staged rows are read by the point lanes next
  return ok;
}

// row list helpers (compile-time lists of tangent DOFs)
template <int NR>
UWVK_DEV constexpr int row_pos(const int (&rows)[NR], int d) {
  for (int q = 0; q < NR; q++)
    if (rows[q] == d) return q;
  return -1;
}

// point p (< 2K: column p>>1, sign + for even p; p == 2K: centre) restricted to
// the DOFs in RL::rows (template recursion: every register index is constant);
// the other entries of x keep mu.
template <class RL, int DOF, int K, int Q>
UWVK_DEV void gen_rows_q(const double* mu, const double* stg, int j, double sg, double (&v)[3], double* x) {
  if constexpr (Q < RL::NR) {
    constexpr int d = RL::rows[Q];
    const double l = stg[Q * K + j];
    if constexpr (d >= 3 && d < 6) {
      v[d - 3] = sg * l;
    } else {
      x[d2s(d)] = mu[d2s(d)] + sg * l;
    }
    gen_rows_q<RL, DOF, K, Q + 1>(mu, stg, j, sg, v, x);
  }
}
template <class RL>
UWVK_DEV constexpr bool has_rot() {
  for (int q = 0; q < RL::NR; q++)
    if (RL::rows[q] >= 3 && RL::rows[q] < 6) return true;
  return false;
}
template <class RL, int DOF, int K, int SR>
UWVK_DEV void gen_rows(const double* mu, const double* stg, int p, double x[Lay<DOF>::store]) {
  using L = Lay<DOF>;
#pragma unroll
  for (int s = 0; s < L::store; s++) x[s] = mu[s];
  if constexpr (K > 0) {
    const bool in = LANE_IF(p, p < 2 * K);
    const int j = in ? (p >> 1) : 0;
    const double sg = in ? (LANE_IF(p, (p & 1) != 0) ? -1.0 : 1.0) : 0.0;  // the centre: mu + 0 (bitwise mu)
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
// Process model pieces (PoseUKF.cpp:12-84), bitwise the same expressions as
// process_point() in uwvk_pose_dev.hpp.
// ---------------------------------------------------------------------------
template <int DOF, int SR>
UWVK_DEV void proc_orientation(const double x[Lay<DOF>::store], const PoseShared& sh, const ProcCtx& c, double o[4]) {
  using L = Lay<DOF>;
  // sin / cos of lat = lat0 + x / R_M by angle addition from lat0 (Taylor in
  // d = x / R_M, < 1e-20 relative for |d| < 0.01 rad, i.e. |x| < 64 km)
  const double dl = x[L::s_pos] * sh.inv_rm;
  double sl, cl;
  if (fabs(dl) < 0.01) {
    const double u = dl * dl;
    double sd = fma(fma(fma(u * sk(1.0 / 362880.0) + sk(-1.0 / 5040.0), u, sk(1.0 / 120.0)), u, sk(-1.0 / 6.0)), u, 1.0) * dl;
    double cd = fma(fma(fma(u * sk(1.0 / 40320.0) + sk(-1.0 / 720.0), u, sk(1.0 / 24.0)), u, -0.5), u, 1.0);
    sl = sh.slat0 * cd + sh.clat0 * sd;
    cl = sh.clat0 * cd - sh.slat0 * sd;
  } else {
    sincos(sh.lat0 + dl, &sl, &cl);
  }
  const double er[3] = {kEarthW * cl, 0.0, kEarthW * sl};
  double wb[3], wn[3];
#pragma unroll
  for (int i = 0; i < 3; i++) wb[i] = c.w[i] - x[L::s_bg + i];
  qrot(x + L::s_quat, wb, wn);
#pragma unroll
  for (int i = 0; i < 3; i++) wn[i] = (wn[i] - er[i]) * c.dt;
  double e[4];
  so3_exp_psp(wn, e);
  qplus_psp<SR>(e, x + L::s_quat, o);  // new_state.orientation.boxplus (PoseUKF.cpp:32)
}

// the same, branch-free from the lane constants (psp::lane_proc, set once per
// launch): x + dt * mu[vpart] | x + dt * (nt (x - off)) | x
UWVK_DEV double proc_vect_lane(int s, const double* mu, const ProcCtx& c) {
  const double x = mu[s];
  const double y = mu[c.vpart >= 0 ? c.vpart : s];
  const double d = c.vpart >= 0 ? y : c.nt_lane * (x - c.off_lane);
  return (c.vpart >= 0 || c.nt_lane != 0.0) ? x + c.dt * d : x;
}

// the same per lane from the eight uniform decay rates by selects: a runtime
// index into sh.ntau was a per-lane global load whose s_waitcnt vmcnt(0) also
// drained the next epoch's IMU prefetch on the predict's critical path
template <int DOF>
UWVK_DEV double tan_ntau_sel(int d, const PoseShared& sh) {
  using L = Lay<DOF>;
  double nt = 0.0;
  nt = (d >= L::d_bg && d < L::d_bg + 3) ? sh.ntau[0] : nt;
  nt = (d >= L::d_ba && d < L::d_ba + 3) ? sh.ntau[1] : nt;
  if constexpr (L::has_params) {
    nt = (d >= L::d_inertia && d < L::d_inertia + 9) ? sh.ntau[2] : nt;
    nt = (d >= L::d_lin && d < L::d_lin + 9) ? sh.ntau[3] : nt;
    nt = (d >= L::d_quad && d < L::d_quad + 9) ? sh.ntau[4] : nt;
  }
  nt = (d >= L::d_wv && d < L::d_wv + 4) ? sh.ntau[5] : nt;
  nt = (d >= L::d_badcp && d < L::d_badcp + 2) ? sh.ntau[6] : nt;
  nt = (d == L::d_rho) ? sh.ntau[7] : nt;
  return nt;
}
// coupled column of row d (pos -> vel, vel -> acc) or -1
UWVK_DEV constexpr int proc_couple(int d) { return d < 3 ? d + 6 : (d >= 6 && d < 9 ? d + 3 : -1); }

// DOFs the orientation row of the process model reads (lat from pos.x, q, b_g)
struct PredRows {
  static constexpr int NR = 7;
  static constexpr int rows[NR] = {0, 3, 4, 5, 12, 13, 14};
};

// ---------------------------------------------------------------------------
// predictionStepImpl (PoseUKF.cpp:446-474) + ukf::predict, PSP form
// ---------------------------------------------------------------------------
// dt^2 Q entries a lane needs every predict, loaded once per launch (row l's
// band: (l,l), (l,l-1), (l,l-2)); used when sh.q_simple (Q block-diagonal with
// no coupling between the rewritten rows < 9 and the rest, band <= 2)
struct LaneQ {
  double q0, q1, q2;
};
// PD: fq is the 26-DOF subset's table followed by the parameters' diagonal
// entries (parameter t at NP + t), the host's PD table (uwvk_pose.hip)
template <int DOF, int PD = 0>
UWVK_DEV LaneQ lane_q(const double* fq, int l) {
  const double2* f2 = reinterpret_cast<const double2*>(fq);
  LaneQ q{0.0, 0.0, 0.0};
  if (l < DOF) {
    q.q0 = f2[pidx(l, l)].y;
    if (l >= 1) q.q1 = f2[pidx(l, l - 1)].y;
    if (l >= 2) q.q2 = f2[pidx(l, l - 2)].y;
  }
  if constexpr (PD && !PSP_PAIR) {
    if (l >= kPdLane0 && l < kPdLane0 + kPdN) q.q0 = f2[PG<DOF>::NP + (l - kPdLane0)].y;
  }
  return q;
}

// Q: process_noise_cov (DOF x DOF); fq: per packed entry {., dt^2 Q_ij} (host-made per dt)
// ds, ids: this lane's time scale d_l and 1/d_l (updated: d' = A_ll d)
// QM: the process-noise shape, 0 read from sh at run time, 1 known simple
// (sh.q_simple: lane-resident band <= 2), 2 known general.  The epoch kernel is
// instantiated for 1 and 2 and the host picks one: with both branches in one
// kernel the epoch loop ran 0.7-0.8% slower (profiles/r03/qm/).
// PD (the parameter-decoupled kernel, see PspSmemPD): DOF = 26 layout with the
// 53-DOF weights; px: the parameters' LDS (pS, pm at + 32)
template <int DOF, int QM = 0, int SR = 0, int PD = 0>
UWVK_DEV bool psp_predict(PspSmem<DOF>& sm, const PoseShared& sh, const ProcCtx& pc, const double* Q,
                          const double* fq, double& ds, double& ids, const LaneQ& lq,
                          Stamper* st = nullptr, double* px = nullptr) {
  using L = Lay<DOF>;
  using G = PG<DOF>;
  constexpr int K = G::KP;
  static_assert(!PD || (DOF == 26 && QM == 1), "PD: the 26-DOF layout, lane-resident Q");
  constexpr int NW = PD ? 53 : DOF;  // the filter's n (sigma-point weights)
  int l = olane();  // re-laundered per phase (PSP_PHASE)
  const double dt = pc.dt, dt2 = dt * dt;
  // process-noise shaping from the pre-predict mean (PoseUKF.cpp:448-460)
  double qo_lane = 0.0;  // lane a*3+b (< 9) keeps (R Q_ori R^T)[a][b]
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
    qo_lane = s;
  }
  const double vs0 = sm.mu[L::s_vel], vs1 = sm.mu[L::s_vel + 1], vs2 = 10 * sm.mu[L::s_vel + 2];
  const double wv_add = sh.p.water_velocity_scale * (vs0 * vs0 + vs1 * vs1 + vs2 * vs2) * dt;
  // partial Cholesky and row staging
  double a[K];
  chain_prio_hi();
  const bool ok = pchol<DOF, K, PredRows>(sm.S, l, a, ds, sm.stg);
  chain_prio_lo();
  PSP_PHASE(20);
  // sigma points: lanes < 2K plus the centre lane 2K; orientation output only
  const bool pt = LANE_IF(l, l < 2 * K), ctr = LANE_IF(l, l == 2 * K);
  double o[4];
  {
    double x[L::store];
    gen_rows<PredRows, DOF, K, SR>(sm.mu, sm.stg + STG_ROWS, l, x);
    proc_orientation<DOF, SR>(x, sh, pc, o);
  }
  PSP_PHASE(21);
  // manifold mean of the orientations (ukfom: ref = X_0, Gauss-Newton, |d| <= 1e-6)
  constexpr double wc = 1.0 + 2.0 * (NW - K);
  double mq[4];
#pragma unroll
  for (int i = 0; i < 4; i++) mq[i] = hread(o[i], 2 * K);
  {
    int it = 0;
    double nrm;
    do {
      double d[3];
      qboxminus_psp<SR>(o, mq, d);
      const double w = pt ? 1.0 : (ctr ? wc : 0.0);
      nrm = 0.0;
#pragma unroll
      for (int i = 0; i < 3; i++) {
        d[i] = wave_sum_dpp<2 * K + 1>(w * d[i]) * (1.0 / (double)(2 * NW + 1));
        nrm += d[i] * d[i];
      }
      double e[4], q[4];
      so3_exp_psp(d, e);
      qplus_psp<SR>(e, mq, q);
#pragma unroll
      for (int i = 0; i < 4; i++) mq[i] = q[i];
    } while (nrm > 1e-12 && ++it < 10000);  // |delta| > 1e-6
  }
  PSP_PHASE(22);
  // deviations; ori x ori block; Delta_j = d_{j+} - d_{j-}
  double d[3];
  qboxminus_psp<SR>(o, mq, d);
  double oo[6];
  {
    const double w = pt ? 1.0 : (ctr ? wc : 0.0);
    // six sums over lanes 0..2K: pair sums by one DPP swap, then the 16 even
    // lanes' values transposed through LDS (stg is free after the points)
    double v[6];
    int k = 0;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) {
        const double t = w * d[i] * d[j];
        v[k++] = t + swap_pair_d(t);
      }
    static_assert(2 * K + 1 <= 32, "pair sums over two DPP rows");
    lds_sums<6, 16, 2>(v, sm.stg, l, oo);
#pragma unroll
    for (int i = 0; i < 6; i++) oo[i] = 0.5 * oo[i];
  }
  // Delta_j = d_{j+} - d_{j-} lives in lane 2j; it is read back as a uniform
  // (SGPR) value below, no LDS staging
  double dd[3];
#pragma unroll
  for (int i = 0; i < 3; i++) dd[i] = d[i] - swap_pair_d(d[i]);
  // ori x lin: X_r = 1/2 (A (L_a Delta))_r, lane r
  double X[3];
  chain_prio_hi();  // the broadcast loop over Delta_j is a chain too (see chain_prio_hi)
  {
    double Y[3] = {0.0, 0.0, 0.0};
    // Delta_j staged in stg (free after the ori x ori sums) by lane 2j and read
    // back by every lane as a broadcast, one j at a time (a compiler memory
    // barrier per j keeps at most two j's loads in flight: hoisted all at once
    // they took 90 VGPRs); 45 LDS reads instead of 90 v_readlane
    // (PSP_LDS_ALIGN: 4 slots per j from slot 1, so each j's first pair is one
    // aligned ds_read_b128)
    constexpr int DS = 4, D0 = 1;
    static_assert(D0 + DS * K <= PG<DOF>::STG, "Delta (PG::STG)");
    if (LANE_IF(l, (l & 1) == 0 && l < 2 * K)) {
#pragma unroll
      for (int i = 0; i < 3; i++) sm.stg[D0 + (l >> 1) * DS + i] = dd[i];
    }
    wsync();
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
      for (int i = 0; i < 3; i++) Y[i] += a[j] * dj[i];
      // j's products before the barrier, j + 2's loads after it
      asm volatile("" : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2])::"memory");
    }
    wsync();  // stg is rewritten by the next phase's users
    chain_prio_lo();
    const int cp = proc_couple(l);
    const int src = cp >= 0 ? cp : l;
    const double ar = 1.0 + dt * pc.nt_tan;  // proc_diag_sel's value (nt_tan = 0 off the scaled DOFs)
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const double yc = shfl_d(Y[i], hlane(src));
      X[i] = 0.5 * (LANE_IF(l, proc_couple(l) >= 0) ? (ar * Y[i] + dt * yc) : ar * Y[i]);
    }
  }
  PSP_PHASE(23);
  // rows/cols coupled by A (pos, vel): new values into registers first.
  // Sigma[p][jl] = d_jl Sigma~[p][jl] (p, jc < 12 carry d = 1)
  constexpr int pv[6] = {0, 1, 2, 6, 7, 8};
  double nv[6];
  const int jl = l < DOF ? l : DOF - 1;
  const int jc = proc_couple(jl);
  const double aj = 1.0 + dt * pc.nt_tan;  // lanes >= DOF: 1 (their values are never stored)
  const int Tl = (jl * (jl + 1)) >> 1;  // (unused without PSP_PIDX_SEL)
  // packed (p, j) for a compile-time row p < 12 and a lane column j as a select
  // between two sums (tri(j) once per lane): pidx's max / min / product per
  // access were 7 integer instructions; the coupled column is clamped so its
  // loads need no exec branch (their products are selected away)
  const int jcc = jc >= 0 ? jc : jl;
  const int Tc = (jcc * (jcc + 1)) >> 1;
  [[maybe_unused]] const double cf = LANE_IF(l, proc_couple(l < DOF ? l : DOF - 1) >= 0) ? dt : 0.0;
  // (r04) pidx_sel's branch per row as lane masks: rows pv[q] and
  // proc_couple(pv[q]), against the lane column jl and the coupled one jcc
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
    // (r04) the coupled column's term as an FMA with cf = dt (coupled lanes) or
    // 0: the conditional form was compiled to 12 exec-masked branches, each
    // waiting for its own LDS load (lgkmcnt(0)); S~ is finite, so cf = 0 adds 0
    const double t0 = fma(cf, sm.S[pidx_sel_b(r, jcc, Tc, LANE_IN(mc_r[q]))],
                          aj * (ds * sm.S[pidx_sel_b(r, jl, Tl, LANE_IN(ml_r[q]))]));
    const double t1 = fma(cf, sm.S[pidx_sel_b(rc, jcc, Tc, LANE_IN(mc_rc[q]))],
                          aj * (ds * sm.S[pidx_sel_b(rc, jl, Tl, LANE_IN(ml_rc[q]))]));
    nv[q] = t0 + dt * t1;  // A_rr = 1 for pos/vel rows
  }
  // new time scale d' = A_ll d (A_ll = 1 on the unscaled DOFs)
  // (PD: the parameters' lanes too; pc.nt_tan holds their decay rate)
  // (PSP_PAIR: the parameters are the pair kernel's own, uwvk_psp_pair.hip)
  constexpr bool kPL = PD && !PSP_PAIR;
  if (LANE_IF(l, (l < DOF && scaled_dof(l)) || (kPL && l >= kPdLane0 && l < kPdLane0 + kPdN))) {
    ds = aj * ds;
    double rc = __builtin_amdgcn_rcp(ds);  // d in (0, 1]: two Newton steps
    rc = fma(rc, fma(-ds, rc, 1.0), rc);
    ids = fma(rc, fma(-ds, rc, 1.0), rc);
  }
  psync();
  PSP_PHASE(24);
  // rewrite rows/cols < 9 (stored as Sigma / d'_l): A-coupled rows (pos, vel),
  // orientation rows (cross terms), ori x ori
  const bool qs = QM == 1 ? true : (QM == 2 ? false : sh.q_simple != 0);
  // the lane-resident Q (qs, a uniform branch) needs no global load: the
  // dt^2 Q table is read only for a general Q (a load under a per-lane select
  // was issued anyway and waited for on the critical path)
  auto rows_lt9 = [&](auto QS) {
    constexpr bool kQS = decltype(QS)::value;
    if (LANE_IF(l, l < DOF && !(l >= 3 && l < 6))) {
      const bool jpv = LANE_IF(l, proc_couple(l < DOF ? l : DOF - 1) >= 0);
      const double2* f2 = reinterpret_cast<const double2*>(fq);
      constexpr unsigned long long smask[6] = {rows_store_mask<DOF>(0), rows_store_mask<DOF>(1),
                                               rows_store_mask<DOF>(2), rows_store_mask<DOF>(6),
                                               rows_store_mask<DOF>(7), rows_store_mask<DOF>(8)};
      constexpr unsigned long long gmask[6] = {col_ge_mask<DOF>(0, false), col_ge_mask<DOF>(1, false),
                                               col_ge_mask<DOF>(2, false), col_ge_mask<DOF>(6, false),
                                               col_ge_mask<DOF>(7, false), col_ge_mask<DOF>(8, false)};
#pragma unroll
      for (int q = 0; q < 6; q++)
        if (LANE_IN(smask[q])) {  // !jpv || l <= pv[q]
          const int e = pidx_sel_b(pv[q], l, Tl, LANE_IN(gmask[q]));  // l < DOF: jl == l
          double qq;
          if constexpr (kQS) qq = 0.0;
          else qq = f2[e].y;
          sm.S[e] = (nv[q] + qq) * ids;
        }
      // (r04) the lane-resident Q's diagonal on the pos / vel rows added by
      // their own lane afterwards, instead of a select per row: lane l in
      // {0, 1, 2, 6, 7, 8} (jpv) stored (l, l) above; d_l = 1 there (ids == 1),
      // so nv + q0 is bitwise the (nv + q0) * ids of the select form
      if (kQS && jpv) sm.S[Tl + l] += lq.q0;
#pragma unroll
      for (int i = 0; i < 3; i++) {
        constexpr unsigned long long omask[3] = {col_ge_mask<DOF>(3, false), col_ge_mask<DOF>(4, false),
                                                 col_ge_mask<DOF>(5, false)};
        const int e = pidx_sel_b(3 + i, l, Tl, LANE_IN(omask[i]));
        if constexpr (kQS) sm.S[e] = X[i] * ids;
        else sm.S[e] = (X[i] + f2[e].y) * ids;
      }
    }
  };
  if (qs)
    rows_lt9(std::true_type{});
  else
    rows_lt9(std::false_type{});
  if (LANE_IF(l, l < 9 && (l / 3) >= (l % 3))) {
    const int a2 = l / 3, b2 = l % 3;
    sm.S[pidx(3 + a2, 3 + b2)] = sel6(oo[0], oo[1], oo[2], oo[3], oo[4], oo[5], a2 * (a2 + 1) / 2 + b2) + dt2 * qo_lane;
  }
  // rows/cols >= 9: A Sigma A^T = D' Sigma~ D' leaves Sigma~ unchanged; only
  // dt^2 Q / (d'_i d'_j) is added on Q's band.  Lane l owns row l's band
  // entries (l, l - k); k <= 2 from registers, wider bands from global memory.
  {
    constexpr int R0 = 9;
    const double2* f2 = reinterpret_cast<const double2*>(fq);
    const int bw = sh.q_bw;
    // the lane-resident band (qs) and the table band are separate uniform
    // branches: a per-lane select between them made the compiler issue the
    // table load anyway and wait for it (and for the IMU prefetch) every epoch.
    // The water-velocity noise comes from four uniform values passed through an
    // empty asm, so that the select is not turned back into a per-lane load.
    double qw4[4] = {sh.q_wv[0], sh.q_wv[1], sh.q_wv[2], sh.q_wv[3]};
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" : "+s"(qw4[i]));
    auto band = [&](auto QS) {
      constexpr bool kQS = decltype(QS)::value;
      if constexpr (kQS) {
        // (r04) the three entries (l, l - k) loaded unconditionally (clamped
        // into the triangle), then stored under the lane's mask: the masked
        // read-modify-write per k waited for its own load (lgkmcnt(0)) inside
        // an exec branch, three times in a row
        const int lc = l < DOF ? l : DOF - 1;
        const int T = (lc * (lc + 1)) >> 1;
        double v[3], f[3];
        int e[3];
        bool w[3];
        double idk = ids;  // 1 / d'_{l-k}
        // (r04) the band's lane conditions per k as constant masks
        constexpr unsigned long long bandm[3] = {
            lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l >= R0; }),
            lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l - 1 >= R0; }),
            lane_mask([](int l) constexpr { return l >= R0 && l < DOF && l - 2 >= R0; })};
#pragma unroll
        for (int k = 0; k < 3; k++) {
          if (k > 0) idk = dpp_d<0x138, 0xf, 0xf>(idk);  // wave_shr:1 -> lane l - k
          const int j = l - k;
          e[k] = T + (j >= 0 ? (j <= lc ? j : lc) : 0);
          v[k] = sm.S[e[k]];
          double q = k == 0 ? lq.q0 : (k == 1 ? lq.q1 : lq.q2);
          if (k == 0 && LANE_IF(l, l >= L::d_wv && l < L::d_wv + 4)) {
            const int iw = l - L::d_wv;
            const double qw = iw == 0 ? qw4[0] : (iw == 1 ? qw4[1] : (iw == 2 ? qw4[2] : qw4[3]));
            q = dt2 * (qw + wv_add);
          }
          w[k] = LANE_IN(bandm[k]) && k <= bw && q != 0.0;
          f[k] = q * (ids * idk);
        }
#pragma unroll
        for (int k = 0; k < 3; k++)
          if (w[k]) sm.S[e[k]] = v[k] + f[k];
        return;
      }
      double idk = ids;  // 1 / d'_{l-k}
#pragma unroll
      for (int k = 0; k < 3; k++) {
        if (k > 0) idk = dpp_d<0x138, 0xf, 0xf>(idk);  // wave_shr:1 -> lane l - k
        const int j = l - k;
        if (l >= R0 && l < DOF && j >= R0 && k <= bw) {
          const int e = pidx(l, j);
          double q;
          if constexpr (kQS) q = k == 0 ? lq.q0 : (k == 1 ? lq.q1 : lq.q2);
          else q = f2[e].y;
          if (k == 0 && l >= L::d_wv && l < L::d_wv + 4) {
            const int iw = l - L::d_wv;
            const double qw = iw == 0 ? qw4[0] : (iw == 1 ? qw4[1] : (iw == 2 ? qw4[2] : qw4[3]));
            q = dt2 * (qw + wv_add);
          }
          if (q != 0.0) sm.S[e] += q * (ids * idk);
        }
      }
    };
    if (qs)
      band(std::true_type{});
    else
      band(std::false_type{});
    if constexpr (PD && !PSP_PAIR) {  // the parameters' diagonal: the band's k = 0 entry, as above
      if (LANE_IF(l, l >= kPdLane0 && l < kPdLane0 + kPdN)) {
        const int t = (l - kPdLane0) & 31;
        const double v = px[t];
        const double f = lq.q0 * (ids * ids);
        if (lq.q0 != 0.0) px[t] = v + f;
      }
    }
    for (int k = 3; k <= (QM == 1 ? 0 : bw); k++) {  // uniform bound: wide Q bands only
      const double idj = shfl_d(ids, hlane(l - k >= 0 ? l - k : 0));
      const int j = l - k;
      if (l >= R0 && l < DOF && j >= R0) {
        const int e = pidx(l, j);
        const double q = f2[e].y;
        if (q != 0.0) sm.S[e] += q * (ids * idj);
      }
    }
  }
  PSP_PHASE(25);
  // new mean: vect parts f(mu), orientation the manifold mean
  // every lane evaluates (reads past mu land in the staging area, never
  // stored): the loads need no exec branch and wait
  static_assert(Lay<DOF>::store + PG<DOF>::STG >= 64, "mu reads of lanes >= store stay in PspSmem");
  double mv = proc_vect_lane(l & 63, flat(sm) + kFlatMu<DOF>, pc);
  asm volatile("" : "+v"(mv));
  [[maybe_unused]] double mvp = 0.0;  // PD: the parameters' means (lane 27 + t, px + 32)
  if constexpr (PD && !PSP_PAIR) {
    mvp = proc_vect_lane((l - kPdLane0) & 31, px + 32, pc);
    asm volatile("" : "+v"(mvp));
  }
  psync();
  if (LANE_IF(l, l < L::store && !(l >= 3 && l < 7))) sm.mu[l] = mv;
  if (LANE_IF(l, l < 4)) sm.mu[3 + l] = mq[l];
  if constexpr (PD && !PSP_PAIR) {
    if (LANE_IF(l, l >= kPdLane0 && l < kPdLane0 + kPdN)) px[32 + ((l - kPdLane0) & 31)] = mvp;
  }
  psync();
  PSP_PHASE(26);
  return ok;
}

// Sigma~ -> Sigma (d folded in, d = 1 afterwards): row sweep, lane l owns
// column l of every row i >= l (uniform row offset, d_i a uniform read-back);
// d = 1 on the unscaled DOFs, so their entries are multiplied by 1 (bitwise kept)
template <int DOF, int PD = 0>
UWVK_DEV void psp_fold(PspSmem<DOF>& sm, double& ds, double& ids, double* px = nullptr) {
  const int l = olane();
  psync();
  const double dl = l < DOF ? ds : 1.0;
  // blocks of FB rows, branch-free: every lane loads (its column clamped to the
  // diagonal), then stores to its entry or, for l > i, to a throw-away slot of
  // the staging area (free between epochs): the loads of a block are in flight
  // together instead of one masked read-modify-write per row (r03)
  constexpr int R0 = 12, FB = 4;  // rows < 12 and columns < 12 of them are unscaled
#pragma unroll 1
  for (int i0 = R0; i0 < DOF; i0 += FB) {
    double v[FB];
    int e[FB];
#pragma unroll
    for (int r = 0; r < FB; r++) {
      const int i = i0 + r < DOF ? i0 + r : DOF - 1;
      e[r] = i * (i + 1) / 2 + (l <= i ? l : i);
      v[r] = sm.S[e[r]];
    }
#pragma unroll
    for (int r = 0; r < FB; r++) {
      const int i = i0 + r;
      const double di = hread(ds, i < DOF ? i : DOF - 1);
      double* dst = (i < DOF && l <= i) ? sm.S + e[r] : sm.stg + (l & 63);
      *dst = v[r] * (di * dl);
    }
  }
  if constexpr (PD && !PSP_PAIR) {  // the parameters' diagonal: d_i d_i as for any (i, i)
    if (LANE_IF(l, l >= kPdLane0 && l < kPdLane0 + kPdN)) {
      const int t = (l - kPdLane0) & 31;
      px[t] = px[t] * (ds * ds);
    }
  }
  psync();
  ds = 1.0;
  ids = 1.0;
}

// ---------------------------------------------------------------------------
// measurement models in PSP form: K = nonlinear prefix, ROWS = DOFs eval reads
// (beyond mu), COLS = columns of the affine Jacobian H (COLS within ROWS)
// ---------------------------------------------------------------------------
template <int DOF>
struct PAcc {  // measurementAcceleration, PoseUKF.cpp:125-131
  using L = Lay<DOF>;
  static constexpr int M = 3, K = 6, NR = 10, NC = 7, ZMODE = 1, GATE = 0;
  static constexpr int rows[NR] = {3, 4, 5, 9, 10, 11, 15, 16, 17, 18};
  static constexpr int cols[NC] = {9, 10, 11, 15, 16, 17, 18};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { HAcc<DOF>{}(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);  // z = R^T (a + g e_z) + ba
#pragma unroll
    for (int r = 0; r < 3; r++) {
#pragma unroll
      for (int i = 0; i < 3; i++) {
        H[r][i] = R[i * 3 + r];
        H[r][3 + i] = r == i ? 1.0 : 0.0;
      }
      H[r][6] = R[2 * 3 + r];
    }
  }
};
template <int DOF>
struct PVel {  // measurementVelocity, PoseUKF.cpp:117-123
  using L = Lay<DOF>;
  static constexpr int M = 3, K = 6, NR = 6, NC = 3, ZMODE = 1, GATE = 0;
  static constexpr int rows[NR] = {3, 4, 5, 6, 7, 8};
  static constexpr int cols[NC] = {6, 7, 8};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { HVel<DOF>{}(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int i = 0; i < 3; i++) H[r][i] = R[i * 3 + r];
  }
};
template <int DOF>
struct PPressure {  // measurementPressureSensor, PoseUKF.cpp:107-115 (p_z * g * rho: k = 19)
  using L = Lay<DOF>;
  static constexpr int M = 1, K = 19, NR = 6, NC = 1, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {2, 3, 4, 5, 18, L::d_rho};
  static constexpr int cols[NC] = {L::d_rho};
  HPressure<DOF> h;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { h(x, z); }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double r[3];
    qrot(mu + L::s_quat, h.s, r);
    const double pz = mu[L::s_pos + 2] + r[2];
    H[0][0] = -(pz * mu[L::s_grav]);
  }
};
template <int DOF>
struct PWater {  // measurementWaterCurrents, PoseUKF.cpp:133-151
  using L = Lay<DOF>;
  static constexpr int M = 2, K = 6, NR = 12, NC = 9, ZMODE = 1, GATE = 1;
  static constexpr int rows[NR] = {3, 4, 5, 6, 7, 8, L::d_wv, L::d_wv + 1, L::d_wvb, L::d_wvb + 1,
                                   L::d_badcp, L::d_badcp + 1};
  static constexpr int cols[NC] = {6, 7, 8, L::d_wv, L::d_wv + 1, L::d_wvb, L::d_wvb + 1, L::d_badcp, L::d_badcp + 1};
  double cw;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const {
    HWater<DOF> h;
    h.cw = cw;
    h(x, z);
  }
  UWVK_DEV void jac(const double* mu, double (&H)[M][NC]) const {
    double R[9];
    qmatrix(mu + L::s_quat, R);
#pragma unroll
    for (int r = 0; r < 2; r++) {
#pragma unroll
      for (int i = 0; i < 3; i++) H[r][i] = cw * R[i * 3 + r] + (1 - cw) * R[i * 3 + r];
#pragma unroll
      for (int i = 0; i < 2; i++) {
        H[r][3 + i] = -((1 - cw) * R[i * 3 + r]);
        H[r][5 + i] = -(cw * R[i * 3 + r]);
        H[r][7 + i] = r == i ? 1.0 : 0.0;
      }
    }
  }
};
template <int DOF>
struct PXY {  // measurementXYPosition, PoseUKF.cpp:87-92: linear (k = 0)
  static constexpr int M = 2, K = 0, NR = 2, NC = 2, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {0, 1};
  static constexpr int cols[NC] = {0, 1};
  int gate = 0;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { z[0] = x[0]; z[1] = x[1]; }
  UWVK_DEV void jac(const double*, double (&H)[M][NC]) const { H[0][0] = 1; H[0][1] = 0; H[1][0] = 0; H[1][1] = 1; }
};
template <int DOF>
struct PZ {  // measurementZPosition, PoseUKF.cpp:100-105: linear (k = 0)
  static constexpr int M = 1, K = 0, NR = 1, NC = 1, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {2};
  static constexpr int cols[NC] = {2};
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { z[0] = x[2]; }
  UWVK_DEV void jac(const double*, double (&H)[M][NC]) const { H[0][0] = 1; }
};

template <int DOF>
struct PEffVO {  // constrainVelocity, PoseUKF.cpp:199-219, 585-591 (only_affect_velocity)
  // The model reads the state's velocity only: orientation, water velocity and
  // body acceleration are frozen at mu (HConstrain), the dynamic model's
  // parameters are the shared model's (the handle's model blocks, A9).  It is
  // nonlinear in the velocity (Coriolis, quadratic damping) and independent of
  // every other DOF, so the nonlinear prefix is the velocity block's end, k = 9
  // (19 model evaluations), and there is no affine part (H = 0, NC = 0).
  static constexpr int M = 6, K = 9, NR = 3, NC = 0, ZMODE = 0, GATE = 0;
  static constexpr int rows[NR] = {6, 7, 8};
  static constexpr int cols[1] = {6};  // placeholder: NC = 0 columns are used
  HConstrain<DOF> h;
  UWVK_DEV void eval(const double* x, double (&z)[M]) const { h(x, z); }
  UWVK_DEV void jac(const double*, double (&)[M][1]) const {}
};

// R sums (R > what one staging round holds) over NL contributors: chunks of
// lds_sums, the staging area reused between rounds
template <int R, int NL, int STRIDE, int C0 = 0>
UWVK_DEV void lds_sums_chunked(const double (&v)[R], double* buf, int l, double (&out)[R]) {
  if constexpr (C0 < R) {
    constexpr int CH0 = 115 / NL, CH = (R - C0) < CH0 ? (R - C0) : CH0;
    double vc[CH], oc[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) vc[i] = v[C0 + i];
    lds_sums<CH, NL, STRIDE>(vc, buf, l, oc);
#pragma unroll
    for (int i = 0; i < CH; i++) out[C0 + i] = oc[i];
    wsync();  // every lane's reads of this round before the next round's writes
    lds_sums_chunked<R, NL, STRIDE, C0 + CH>(v, buf, l, out);
  }
}

#if !PSP_PAIR
// one row block I of rankm_mfma_o (tiles (I, J), J <= I), then block I + 1
template <int DOF, int I, int NT>
UWVK_DEV void rankm_block(double* S, const double (&Aop)[NT], const double (&Bop)[NT], int q, int c, int tq) {
  if constexpr (I < NT) {
    constexpr int O = DOF - 16 * NT;
    int base[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      // row R = x + q, x = O + 16 I + 4 i: packed offset T(x) + q x + T(q) + O + c
      // (tq = T(q) + O + c, once per phase) instead of R (R + 1) / 2 per row
      const int x = O + 16 * I + 4 * i;  // a constant after unrolling
      base[i] = q * x + (x * (x + 1) / 2) + tq;
    }
    d4_t acc[I + 1];
    // (r05) the tile loads are volatile LDS reads through one pointer per row
    // (tile J at the immediate offset 128 J): one ds_read_b64 per element
    // straight into its MFMA tuple.  Plain loads were paired across tiles J
    // and J + 1 (16 apart) into ds_read2_b64 and split again by v_mov_b32 (48
    // per rank-3 update), and the stores rematerialised their addresses (2
    // VALU each): -43 VALU per update, C3 +1% (profiles/r05/r05k/)
    using LdsV = const volatile __attribute__((address_space(3))) double*;
    LdsV rp[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      rp[i] = (LdsV)(S + base[i]);
      // opaque, so that the masked diagonal stores reuse the register rather
      // than rematerialise the address
      asm volatile("" : "+v"(rp[i]));
    }
#pragma unroll
    for (int J = 0; J <= I; J++)
#pragma unroll
      for (int i = 0; i < 4; i++) acc[J][i] = rp[i][16 * J];
#pragma unroll
    for (int J = 0; J <= I; J++) acc[J] = mfma_f64(Aop[I], Bop[J], acc[J]);
    // one empty asm over every accumulator: all MFMAs issue before the first
    // store waits for its result (otherwise: MFMA, s_nop 16, stores, MFMA ...)
    if constexpr (I == 0) asm volatile("" : "+v"(acc[0]));
    else if constexpr (I == 1) asm volatile("" : "+v"(acc[0]), "+v"(acc[1]));
    else if constexpr (I == 2) asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]));
    else asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]));
    // (r04) the diagonal tile's lower-triangle lanes per i as constant masks
    constexpr unsigned long long diagm[4] = {
        lane_mask([](int l) constexpr { return (l & 15) <= ((l >> 4) & 3) + 0; }),
        lane_mask([](int l) constexpr { return (l & 15) <= ((l >> 4) & 3) + 4; }),
        lane_mask([](int l) constexpr { return (l & 15) <= ((l >> 4) & 3) + 8; }),
        lane_mask([](int l) constexpr { return (l & 15) <= ((l >> 4) & 3) + 12; })};
    using LdsW = __attribute__((address_space(3))) double*;
#pragma unroll
    for (int J = 0; J <= I; J++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (J < I || LANE_IN(diagm[i])) ((LdsW)rp[i])[16 * J] = acc[J][i];
    rankm_block<DOF, I + 1, NT>(S, Aop, Bop, q, c, tq);
  }
}

// Sigma~ -= C~ K~^T on v_mfma_f64_16x16x4_f64.  Tile D = A B + acc with
// A[r][k] = -C~[row r][k], B[k][c] = K~[col c][k] (k < M, zero padded to K = 4)
// and acc the tile of Sigma~ (lane l holds rows (l >> 4) + 4 i, column l & 15:
// the f64 C/D map, uwvk_dev.hpp).  The frame is shifted by O = DOF mod 16: the
// NT = DOF / 16 full row blocks [O + 16 I, O + 16 I + 16) make NT (NT + 1) / 2
// tiles with every row inside the triangle (53: 6 tiles instead of the 10 of
// a 16-aligned frame, whose last row block held 5 rows of 16); in diagonal
// tiles only column <= row is stored.  The strip of columns < O (rows
// 0..DOF-1) is a lane-per-row FMA chain with K~ of those columns as uniform
// values.  The operands are transposed through stg one 16-row block at a time.
// Within a row block all tiles' loads are issued first, then the MFMAs back to
// back (independent accumulators), then the stores (the r03 16-aligned form
// ran load -> MFMA -> s_nop 16 -> store per tile, its latencies exposed; the
// r03 all-tiles-in-flight form tied: profiles/EXPERIMENTS.md).  The per-entry
// flops and their summation order differ from an FMA-chain row sweep only in
// rounding.
template <int DOF, int M>
UWVK_DEV void rankm_mfma_o(double* S, double* stg, const double (&Ct)[M], const double (&Kt)[M], int l) {
  static_assert(M <= 3, "rank <= 3 (K = 4 with zero padding)");
  constexpr int NT = DOF / 16, O = DOF - 16 * NT;
  static_assert(NT >= 1 && NT <= 4, "frame");
  static_assert(2 * 16 * M <= PG<DOF>::STG, "operand blocks (PG::STG)");
  constexpr bool kStripLds = 2 * 16 * M + O * M <= PG<DOF>::STG;  // else readlane (26 DOF: O = 10)
  const int q = (l >> 4) & 3, c = l & 15;
  double Aop[NT], Bop[NT];
#pragma unroll
  for (int T = 0; T < NT; T++) {
    // rows O + 16 T + c: their lanes stage C~ / K~, every lane reads component q
    const int src = l - O - 16 * T;
    if (src >= 0 && src < 16) {
#pragma unroll
      for (int k = 0; k < M; k++) {
        stg[src * M + k] = Ct[k];
        stg[16 * M + src * M + k] = Kt[k];
      }
    }
    if (kStripLds && T == 0 && LANE_IF(l, l < O)) {  // K~ of the strip columns, read back as broadcasts
#pragma unroll
      for (int k = 0; k < M; k++) stg[32 * M + l * M + k] = Kt[k];
    }
    wsync();
    const int qq = LANE_IF(l, ((l >> 4) & 3) < M) ? q : 0;
    const double a = stg[c * M + qq], b = stg[16 * M + c * M + qq];
    Aop[T] = LANE_IF(l, ((l >> 4) & 3) < M) ? -a : 0.0;
    Bop[T] = LANE_IF(l, ((l >> 4) & 3) < M) ? b : 0.0;
    wsync();  // the next block's writes after every lane's reads
  }
  // strip: lane i (row i) updates columns 0 .. min(i, O - 1).  Column j's
  // address is clamped to the diagonal (min(j, i)) and the columns are stored
  // in descending order, so a row i < O - 1 rewrites its diagonal with
  // throw-away values first and the j = i store lands last (LDS stores of one
  // wave are ordered): no exec-masked store per column
  if constexpr (O > 0) {
    double kc[O][M];
#pragma unroll
    for (int j = 0; j < O; j++)
#pragma unroll
      for (int k = 0; k < M; k++) kc[j][k] = kStripLds ? stg[32 * M + j * M + k] : readlane_d(Kt[k], j);
    {
      // (r04) every lane loads its row (clamped to the last one) outside any
      // branch; only the stores are masked to the rows of the triangle
      const int lc = l < DOF ? l : DOF - 1;
      const int b0 = (lc * (lc + 1)) >> 1;
      double sv[O];
#pragma unroll
      for (int j = 0; j < O; j++) sv[j] = S[b0 + (j <= lc ? j : lc)];
      double nv[O];
#pragma unroll
      for (int j = O - 1; j >= 0; j--) {
        double s2 = sv[j];
#pragma unroll
        for (int k = 0; k < M; k++) s2 = fma(-Ct[k], kc[j][k], s2);
        nv[j] = s2;
      }
      if (l < DOF) {
#pragma unroll
        for (int j = O - 1; j >= 0; j--) S[b0 + (j <= lc ? j : lc)] = nv[j];
      }
    }
  }
  rankm_block<DOF, 0, NT>(S, Aop, Bop, q, c, ((q * (q + 1)) >> 1) + O + c);
}

#else
// PSP_PAIR: Sigma~ -= C~ K~^T as a lane-per-row sweep (one v_mfma_f64_16x16x4
// tile spans all 64 lanes, i.e. both instances): lane r holds C~_r and K~_r;
// K~ of every row is staged in the instance's stg and read back as broadcasts;
// row r's entries go in blocks of RB columns, each block's loads before its
// stores; only the entries on or below the diagonal are stored (lane masks)
// the rows r of column j's entries: j <= r < DOF (local lanes of either half)
template <int DOF>
UWVK_DEV constexpr unsigned long long rankm_col_mask(int j) {
  unsigned long long m = 0;
  for (int l = 0; l < 64; l++)
    if (l >= j && l < DOF) m |= 1ull << l;
  return m;
}
template <int DOF, int M>
UWVK_DEV void rankm_rows(double* S, double* stg, const double (&Ct)[M], const double (&Kt)[M], int l) {
  static_assert(DOF * M <= PG<DOF>::STG, "K~ rows (PG::STG)");
  constexpr int RB = 4;
  if (l < DOF) {
#pragma unroll
    for (int k = 0; k < M; k++) stg[l * M + k] = Kt[k];
  }
  wsync();
  const int lc = l < DOF ? l : DOF - 1;
  const int b0 = (lc * (lc + 1)) >> 1;
  // (r06) entry (r, j) loaded from S[T(r) + j] for every lane (j > r reads a
  // later entry of the triangle: T(r) + j <= T(DOF - 1) + DOF - 1 < NP) and
  // stored under the constant lane mask {l : j <= l < DOF} (an EXEC mask by
  // scalar instructions), instead of two address selects per entry to a
  // throw-away slot: +1.5% at 200 epochs (profiles/r06/r06q/)
#pragma unroll
  for (int j0 = 0; j0 < DOF; j0 += RB) {
    double sv[RB];
#pragma unroll
    for (int u = 0; u < RB; u++)
      if (j0 + u < DOF) sv[u] = S[b0 + j0 + u];
#pragma unroll
    for (int u = 0; u < RB; u++) {
      if (j0 + u >= DOF) continue;
      double s2 = sv[u];
#pragma unroll
      for (int k = 0; k < M; k++) s2 = fma(-Ct[k], stg[(j0 + u) * M + k], s2);
      if (LANE_IN(rankm_col_mask<DOF>(j0 + u))) S[b0 + j0 + u] = s2;
    }
  }
  wsync();  // stg is rewritten next
}
#endif  // !PSP_PAIR

// acc + h x for an entry h of a measurement Jacobian: the structural zeros of
// H (e.g. the identity block of the acceleration model's bias columns) are
// compile-time constants after inlining, and their terms are dropped.  For
// finite x the sum is bitwise the same (fma(0, x, acc) == acc); the
// multiply-by-zero FMAs were issued, since IEEE fma(0, x, acc) is not acc for x
// inf / NaN.
UWVK_DEV double hfma(double h, double x, double acc) {
  if (__builtin_constant_p(h) && h == 0.0) return acc;
  return acc + h * x;
}

// apply_delta, exact form (psp_update, psp_update_eff; delta_r in lane r):
// mu <- mu [+] delta, Sigma <- T Sigma T^T with T
// the identity except on the orientation block.  ukfom re-spreads X_p =
// mu [+] +-L_j, shifts every point by delta and takes the deviations from
// mu [+] delta; on the orientation block that deviation is, for the left
// side, log(exp(d) exp(l) q q^-1 exp(-d)) = R(exp d) l, and for the right
// side log(exp(-d) q^-1 q exp(l) exp(d)) = R(exp d)^T l (conjugation), so
// T = R(exp d) (SR = 0) or R(exp d)^T = R(exp(d)^-1) (SR = 1); the vector
// deviations are L_j unchanged.  The weights (1/2 over the 2n points) give
// T L L^T T^T exactly.
template <int DOF, int SR>
UWVK_DEV void psp_apply_delta(PspSmem<DOF>& sm, double dl, int l) {
  using L = Lay<DOF>;
  const double dv[3] = {hread(dl, 3), hread(dl, 4), hread(dl, 5)};
  double R[9], eq[4];  // exp(delta_ori) once: T's rotation and the mean's [+]
  so3_exp_psp(dv, eq);
  {
    const double tq[4] = {eq[0], SR ? -eq[1] : eq[1], SR ? -eq[2] : eq[2], SR ? -eq[3] : eq[3]};
    qmatrix(tq, R);
  }
  // (r04) rows 3..5 of every column j outside the block, and the ori x ori
  // block R B R^T: every lane loads and computes (its column clamped into
  // the triangle; the block's lanes 3..5 and lanes >= 9 compute values that
  // are not stored), only the stores are masked: no load waits in branches.
  // The block is disjoint from the rows' entries, so its loads go first too.
  double nb;
  {
    const int lc = l < DOF ? l : DOF - 1;
    const int Tl = (lc * (lc + 1)) >> 1;
    const int e0 = pidx_sel_b(3, lc, Tl, LANE_IN(col_ge_mask<DOF>(3, false))),
              e1 = pidx_sel_b(4, lc, Tl, LANE_IN(col_ge_mask<DOF>(4, false))),
              e2 = pidx_sel_b(5, lc, Tl, LANE_IN(col_ge_mask<DOF>(5, false)));
    double s0 = sm.S[e0], s1 = sm.S[e1], s2 = sm.S[e2];
    asm volatile("" : "+v"(s0), "+v"(s1), "+v"(s2));  // loaded here, not sunk into the store branch
    double B[9];
#pragma unroll
    for (int u = 0; u < 3; u++)
#pragma unroll
      for (int v = 0; v < 3; v++) B[u * 3 + v] = sm.S[pidx(3 + u, 3 + v)];
    const int r = l / 3, c = l % 3;  // (r >= 3 for lanes >= 9: not stored)
    double sb = 0.0;
#pragma unroll
    for (int u = 0; u < 3; u++) {
      double t = 0.0;
#pragma unroll
      for (int v = 0; v < 3; v++) t += B[u * 3 + v] * sel3(R[v], R[3 + v], R[6 + v], c);
      sb += sel3(R[u], R[3 + u], R[6 + u], r) * t;
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
  // storage s = l takes tangent delta_{l} (l < 3) or delta_{l-1} (l >= 7): DPP wave_shr:1
  const double dsh = dpp_d<0x138, 0xf, 0xf>(dl);
  double mnew = flat(sm)[kFlatMu<DOF> + (l & 63)] + 1.0 * (LANE_IF(l, l < 3) ? dl : dsh);  // stored for the vector lanes only
  asm volatile("" : "+v"(mnew));
  double qn[4];
  qplus_psp<SR>(eq, sm.mu + L::s_quat, qn);
  psync();
  if (LANE_IF(l, l < 9 && (l / 3) >= (l % 3))) sm.S[pidx(3 + l / 3, 3 + l % 3)] = nb;
  if (LANE_IF(l, l < L::store && !(l >= 3 && l < 7))) sm.mu[l] = mnew;
  if (LANE_IF(l, l < 4)) sm.mu[3 + l] = qn[l];
  psync();
}

// ---------------------------------------------------------------------------
// ukf::update [EXT], PSP form.  gate: 0 accept any, 1 d2p95.  Returns the gate
// decision; *ok = false on a non-positive pivot of the partial Cholesky.
// ---------------------------------------------------------------------------
// NW: the filter's n for the sigma-point weights (53 in the PD kernel's 26-DOF
// layout, else DOF)
template <int DOF, int SR, class HM, int NW = DOF>
UWVK_DEV bool psp_update(PspSmem<DOF>& sm, const double (&z)[HM::M], const double (&Rm)[HM::M * HM::M], int gate,
                         const HM& hm, bool* ok, double ds, double ids, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  constexpr int M = HM::M, K = HM::K, NC = HM::NC, KA = K > 0 ? K : 1, NCA = NC > 0 ? NC : 1;
  static_assert(!PSP_PAIR || 2 * K + 1 <= 32, "pair: the 2k + 1 sigma points of an update fit 32 lanes");
  int l = olane();  // re-laundered per phase (PSP_PHASE)
  double a[KA];
  bool cok = true;
  if constexpr (K > 0) {
    chain_prio_hi();
    cok = pchol<DOF, K, HM>(sm.S, l, a, ds, sm.stg);
    chain_prio_lo();
  }
  PSP_PHASE(30);
  [[maybe_unused]] const bool pt = LANE_IF(l, l < 2 * K);  // the non-lds_sums path (PSP_FAST & 256 off)
  double zp[M];
  {
    double x[L::store];
    gen_rows<HM, DOF, K, SR>(sm.mu, sm.stg + STG_ROWS, l, x);
    hm.eval(x, zp);
  }
  double zc[M], zb[M], e[M];
#pragma unroll
  for (int i = 0; i < M; i++) zc[i] = hread(zp[i], 2 * K);
  constexpr double wc = 1.0 + 2.0 * (NW - K);
  double S[M * M];
  // H and P first: P reads the staged rows, after which stg holds the
  // transposed sums.  One round of M + M(M+1)/2 sums over the 2K point lanes:
  // u = z_p - z_0, s = sum u, m = s / N; sum dz dz^T = sum u u^T - m s^T - s m^T + 2K m m^T
  // H as every lane computes it (the same values in VGPRs; r05: read back as
  // uniform SGPR pairs they were spilled to VGPR lanes and reloaded, 10
  // v_readlane per update, profiles/r05/r05m/); its structural zeros and ones
  // stay compile-time constants for hfma
  double Hs[M][NCA];
  hm.jac(sm.mu, Hs);
  double Pl = 0.0;
  if constexpr (K > 0) {
    const int q = LANE_IF(l, l < M * K) ? l : 0;
    const int i = q / K, j = q - (q / K) * K;
    // (r05) every row's sum with H's uniform entries as operands (structural
    // zeros dropped by hfma), then one select of the lane's row: selecting
    // H[i][t] per column first cost 2 (M - 1) v_cndmask and the SGPR-to-VGPR
    // moves for every t (the same products in the same order)
    double lv[NCA];
#pragma unroll
    for (int t = 0; t < NC; t++) lv[t] = sm.stg[STG_ROWS + row_pos(HM::rows, HM::cols[t]) * K + j];
#pragma unroll
    for (int ii = 0; ii < M; ii++) {
      double pr = 0.0;
#pragma unroll
      for (int t = 0; t < NC; t++) pr = hfma(Hs[ii][t], lv[t], pr);
      Pl = (ii == 0 || i == ii) ? pr : Pl;
    }
    constexpr int R = M + M * (M + 1) / 2;
    double v[R], sums[R];
#pragma unroll
    for (int i2 = 0; i2 < M; i2++) v[i2] = zp[i2] - zc[i2];
    int k = M;
#pragma unroll
    for (int i2 = 0; i2 < M; i2++)
#pragma unroll
      for (int j2 = 0; j2 <= i2; j2++) v[k++] = v[i2] * v[j2];
    if constexpr (R * 2 * K <= 115) lds_sums<R, 2 * K, 1>(v, sm.stg, l, sums);
    else lds_sums_chunked<R, 2 * K, 1>(v, sm.stg, l, sums);  // M = 6 (constrainVelocity)
    double m[M];
#pragma unroll
    for (int i2 = 0; i2 < M; i2++) {
      m[i2] = sums[i2] * (1.0 / (double)(2 * NW + 1));
      zb[i2] = zc[i2] + m[i2];
      e[i2] = zc[i2] - zb[i2];
    }
    k = M;
#pragma unroll
    for (int i2 = 0; i2 < M; i2++)
#pragma unroll
      for (int j2 = 0; j2 <= i2; j2++) {
        const double s = sums[k++] - m[i2] * sums[j2] - m[j2] * sums[i2] + (2.0 * K) * m[i2] * m[j2];
        S[i2 * M + j2] = 0.5 * (s + wc * e[i2] * e[j2]);
      }
  } else {
#pragma unroll
    for (int i2 = 0; i2 < M; i2++) {
      zb[i2] = zc[i2];
      e[i2] = 0.0;
#pragma unroll
      for (int j2 = 0; j2 <= i2; j2++) S[i2 * M + j2] = 0.0;
    }
  }
  double zd[M];
#pragma unroll
  for (int i = 0; i < M; i++) zd[i] = K > 0 ? zp[i] - swap_pair_d(zp[i]) : 0.0;
  PSP_PHASE(31);
  const int rl = l < DOF ? l : DOF - 1;
  const int Trl = (rl * (rl + 1)) >> 1;
  double Gr[M];
#pragma unroll
  for (int i = 0; i < M; i++) Gr[i] = 0.0;
#pragma unroll
  for (int t = 0; t < NC; t++) {
    double s = sm.S[pidx_sel_b(HM::cols[t], rl, Trl, LANE_IN(col_ge_mask<DOF>(HM::cols[t], false)))];
    if (scaled_dof(HM::cols[t])) s = s * hread(ds, HM::cols[t]);
#pragma unroll
    for (int i = 0; i < M; i++) Gr[i] = hfma(Hs[i][t], s, Gr[i]);
  }
#pragma unroll
  for (int i = 0; i < M; i++) Gr[i] = Gr[i] * ds;  // Sigma[r][c] = d_r d_c Sigma~[r][c]
  PSP_PHASE(32);
  // Glin_r = G_r - sum_j L[r][j] P[:, j]: row r of (Sigma - L_a L_a^T) H^T;
  // C_r = Glin_r + 1/2 sum_j L[r][j] Dz_j; S += H Glin + R  (H Glin = H Sigma H^T - P P^T)
  double Gl[M], C[M];
  if constexpr (K > 0) {
    // P (lane i K + j) and Dz_j (lane 2 j) staged in stg (free after the sums)
    // and read back as broadcasts one j at a time, as the predict's Delta
    // (PSP_DELTA_LDS): LDS reads instead of 4 M K v_readlane
    // (PSP_LDS_ALIGN: M = 3 rows padded to 4 from slot 1, so each j's first
    // pair is one aligned ds_read_b128)
    constexpr int PS = M == 3 ? 4 : M, P0 = M >= 2 ? 1 : 0;
    static_assert(P0 + 2 * PS * K <= PG<DOF>::STG, "P and Dz (PG::STG)");
    if (LANE_IF(l, l < M * K)) sm.stg[P0 + (l % K) * PS + l / K] = Pl;  // j-major: P[i][j] at j PS + i
    if (LANE_IF(l, (l & 1) == 0 && l < 2 * K)) {
#pragma unroll
      for (int i = 0; i < M; i++) sm.stg[P0 + PS * K + (l >> 1) * PS + i] = zd[i];
    }
    wsync();
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
        asm volatile("" : "+v"(g[i]), "+v"(c[i])::"memory");  // one j's loads in flight
      }
    }
    wsync();  // stg is rewritten by the rank-M staging
#pragma unroll
    for (int i = 0; i < M; i++) {
      Gl[i] = g[i];
      C[i] = g[i] + 0.5 * c[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < M; i++) {
      Gl[i] = Gr[i];
      C[i] = Gr[i];
    }
  }
#if PSP_PAIR
  // Gl of the Jacobian's columns through the staging area: lane c of column
  // rank t (HM::cols ascending) writes Gl[.] to stg[t M + .], every lane reads
  // them back as LDS broadcasts -- one hread per (t, j) costs a DPP pair or a
  // readlane + select per half (r06zf: -0.5 % kernel time at 20 epochs,
  // -0.8 % at 200)
  double glb[NCA][M];
  {
    static_assert(NC * M <= PG<DOF>::STG, "Gl staging (PG::STG)");
    constexpr unsigned long long cm = cols_mask<HM>();
    static_assert(NC == 0 || (cm != 0 && (cm >> 32) == 0), "HM::cols ascending, below 32");
    const int t = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(rep_mask(cm) >> 32),
                                                  __builtin_amdgcn_mbcnt_lo((unsigned)rep_mask(cm), 0u)) -
                  (upper_half() ? __builtin_popcount((unsigned)cm) : 0);
    if (LANE_IN(cm)) {
#pragma unroll
      for (int j = 0; j < M; j++) sm.stg[t * M + j] = Gl[j];
    }
    wsync();
#pragma unroll
    for (int tt = 0; tt < NC; tt++)
#pragma unroll
      for (int j = 0; j < M; j++) glb[tt][j] = sm.stg[tt * M + j];
    wsync();  // stg is rewritten by the rank-M staging
  }
#endif
#pragma unroll
  for (int i = 0; i < M; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) {
      double hg = 0.0;
#pragma unroll
#if PSP_PAIR
      for (int t = 0; t < NC; t++) hg = hfma(Hs[i][t], glb[t][j], hg);
#else
      for (int t = 0; t < NC; t++) hg = hfma(Hs[i][t], hread(Gl[j], HM::cols[t]), hg);
#endif
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
    double u = 0.0;
#pragma unroll
    for (int i = 0; i < M; i++) u += nu[i] * Si[i * M + j];
    d2 += u * nu[j];
  }
  *ok = cok;
  const bool accept = gate == 0 ? true : !(d2 > kD2P95);
  if (!accept) return false;
  PSP_PHASE(33);
  // Sigma -= C K^T: row sweep (rankm_rows), lane = column j holds K_j, C_i is
  // an LDS broadcast; each block's loads precede its stores.  delta = K nu (lane r).
  psync();
  double dl = 0.0;  // delta = K nu, lane r
#pragma unroll
  for (int i = 0; i < M; i++) dl += Kg[i] * nu[i];
  // Sigma~ -= (C / d)(K / d)^T
  double Ct[M], Kt[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    Ct[i] = C[i] * ids;
    Kt[i] = Kg[i] * ids;
  }
  psync();
#if PSP_PAIR
  rankm_rows<DOF, M>(sm.S, sm.stg, Ct, Kt, l);
#else
  if constexpr (M <= 3) {
    rankm_mfma_o<DOF, M>(sm.S, sm.stg, Ct, Kt, l);
  } else {  // rank M > 3 (constrainVelocity, M = 6): two passes of rank 3 and M - 3
    double c0[3], k0[3], c1[M - 3], k1[M - 3];
#pragma unroll
    for (int i = 0; i < 3; i++) { c0[i] = Ct[i]; k0[i] = Kt[i]; }
#pragma unroll
    for (int i = 0; i < M - 3; i++) { c1[i] = Ct[3 + i]; k1[i] = Kt[3 + i]; }
    rankm_mfma_o<DOF, 3>(sm.S, sm.stg, c0, k0, l);
    psync();
    rankm_mfma_o<DOF, M - 3>(sm.S, sm.stg, c1, k1, l);
  }
#endif
  psync();
  PSP_PHASE(34);
  psp_apply_delta<DOF, SR>(sm, dl, l);
  PSP_PHASE(35);
  return true;
}


#if !PSP_PAIR  // (the pair kernel runs no BodyEfforts update)
// ---------------------------------------------------------------------------
// measurementEfforts (PoseUKF.cpp:153-196), the full BodyEfforts update, in PSP
// form on one wave per instance (r05; the literal two-wave kernel stays on
// UWVK_OPT_DENSE_SIGMA).  The model is non-affine in K = HJmax DOFs (48 of 53:
// orientation, velocity, acceleration, the 27 model parameters, the water
// velocity; 21 of 26) and reads none after them, so PSP's prefix is k = K:
// 2K + 1 model evaluations and no affine part (H = 0), i.e. the literal
// update's algebra with the points j >= K folded into the centre.  LDS is the
// epoch kernel's PspSmem (12.8 KB):
//  - Sigma's Cholesky factor overwrites the packed triangle (all DOF columns,
//    so the positive-definiteness flag is the literal factor's), in panels of
//    16 columns: the panel's update by the columns before it on
//    v_mfma_f64_16x16x4 tiles (A = -L[rows][k], B = L[panel][k]^T, the
//    accumulator the panel's entries), then the panel's columns right-looking,
//    lane r holding row r of the panel in registers;
//  - lane j < K evaluates mu [+] L_j and mu [+] -L_j, lane K the centre;
//  - C = 1/2 L_a Dz^T with Dz staged 16 columns at a time in stg, the 27
//    sums of z through the factor's area (dead by then), Sigma re-read from
//    HBM, Sigma -= C K^T as two rank-3 MFMA passes, the exact apply_delta.
// ---------------------------------------------------------------------------
// S[rows >= P][P, P + W) -= L[rows][0, P) L[P, P + W)[0, P)^T.  Tile t holds
// rows P + 16 t + (l >> 4) + 4 i, column P + (l & 15) (the f64 C/D map); A
// lane l: row P + 16 t + (l & 15), k = 4 s + (l >> 4); B lane l: k = 4 s +
// (l >> 4), column P + (l & 15).  Entries outside the triangle are clamped
// into it for the load and not stored; only columns >= P are written, only
// columns < P are read as operands, so the tiles need no ordering.
template <int DOF, int P, int W>
UWVK_DEV void eff_chol_update(double* S, int l) {
  constexpr int NRT = (DOF - P + 15) / 16, NS = P / 4;
  const int q = (l >> 4) & 3, c = l & 15;
  const int bc = P + c < DOF ? P + c : DOF - 1;
  const double* Bp = S + ((bc * (bc + 1)) >> 1);
  const bool bv = c < W;  // P + c < DOF
  double Bop[NS];
#pragma unroll
  for (int s = 0; s < NS; s++) Bop[s] = bv ? Bp[4 * s + q] : 0.0;
#pragma unroll
  for (int t = 0; t < NRT; t++) {
    const int ar = P + 16 * t + c;
    const int arc = ar < DOF ? ar : DOF - 1;
    const double* Ap = S + ((arc * (arc + 1)) >> 1);
    const bool av = ar < DOF;
    int idx[4];
    bool st[4];
    d4_t acc;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int row = P + 16 * t + q + 4 * i, col = P + c;
      st[i] = row < DOF && bv && col <= row;
      const int rr = row < DOF ? row : DOF - 1;
      const int cc = col <= rr ? col : rr;
      idx[i] = ((rr * (rr + 1)) >> 1) + cc;
      acc[i] = S[idx[i]];
    }
#pragma unroll
    for (int s = 0; s < NS; s++) acc = mfma_f64(av ? -Ap[4 * s + q] : 0.0, Bop[s], acc);
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (st[i]) S[idx[i]] = acc[i];
  }
}

// column P + J of the panel: pivot from lane P + J's registers, the column
// broadcast through col (lane r writes slot r; one wave: LDS in order)
template <int P, int W, int J>
UWVK_DEV void eff_chol_step(double (&a)[W], int r, bool& ok, double* col) {
  if constexpr (J < W) {
    const double piv = readlane_d(a[J], P + J);
    ok = ok && (piv > 0.0);
    const double inv = rsqrt_f64(piv);
    a[J] = LANE_IF(r, r >= P + J) ? a[J] * inv : 0.0;  // lane P + J: piv / sqrt(piv)
    if constexpr (J + 1 < W) {
      col[r & 63] = a[J];
      wsync();
#pragma unroll
      for (int c = J + 1; c < W; c++) a[c] -= a[J] * col[P + c];
#pragma unroll
      for (int c = J + 1; c < W; c++) asm volatile("" : "+v"(a[c]));
    }
    eff_chol_step<P, W, J + 1>(a, r, ok, col);
  }
}

// lanes l in [P + c, LIM) for each panel column c, as constant masks
struct PanelMasks {
  unsigned long long m[16];
};
template <int P, int W, int LIM>
UWVK_DEV constexpr PanelMasks panel_masks() {
  PanelMasks g{};
  for (int c = 0; c < W; c++) {
    unsigned long long m = 0;
    for (int i = 0; i < 64; i++)
      if (i >= P + c && i < LIM) m |= 1ull << i;
    g.m[c] = m;
  }
  return g;
}

template <int DOF, int P>
UWVK_DEV void eff_chol(double* S, double* col, int l, bool& ok) {
  if constexpr (P < DOF) {
    constexpr int W = DOF - P < 16 ? DOF - P : 16;
    if constexpr (P > 0) {
      eff_chol_update<DOF, P, W>(S, l);
      psync();
    }
    // lanes >= DOF shadow the last row (never stored); a row above the panel
    // column reads a later entry of the triangle, selected away
    const int rr = l < DOF ? l : DOF - 1;
    double* Sr = S + ((rr * (rr + 1)) >> 1) + P;
    constexpr PanelMasks ld = panel_masks<P, W, 64>(), stm = panel_masks<P, W, DOF>();
    double a[W];
#pragma unroll
    for (int c = 0; c < W; c++) {
      const double v = Sr[c];
      a[c] = LANE_IN(ld.m[c]) ? v : 0.0;
    }
    eff_chol_step<P, W, 0>(a, l, ok, col);
#pragma unroll
    for (int c = 0; c < W; c++)
      if (LANE_IN(stm.m[c])) Sr[c] = a[c];
    psync();
    eff_chol<DOF, P + 16>(S, col, l, ok);
  }
}

// point mu [+] sg L_j over the first K DOFs (L in place in S; L[d][j] = 0 for
// j > d); sg = 0: the centre, bitwise mu.  The orientation first
// (eff_point_quat), for both signs before any model evaluation: so3_exp_psp's
// library fallback then runs with almost nothing else live (inside an
// evaluation it stacked ~90 VGPRs on the model's)
template <int DOF, int SR>
UWVK_DEV void eff_point_quat(const PspSmem<DOF>& sm, int j, double sg, double (&q)[4]) {
  using L = Lay<DOF>;
  double v[3];
#pragma unroll
  for (int d = 3; d < 6; d++) {
    const bool in = j <= d;
    const double ld = sm.S[d * (d + 1) / 2 + (in ? j : d)];
    v[d - 3] = sg * (in ? ld : 0.0);
  }
  double e[4];
  so3_exp_psp(v, e);
  qplus_psp<SR>(e, sm.mu + L::s_quat, q);
}
template <int DOF, int K, class HM>
UWVK_DEV void eff_point(const PspSmem<DOF>& sm, const HM& h, int j, double sg, const double (&q)[4],
                        double (&z)[6]) {
  using L = Lay<DOF>;
  double x[L::store];
#pragma unroll
  for (int s = 0; s < L::store; s++) x[s] = sm.mu[s];
#pragma unroll
  for (int i = 0; i < 4; i++) x[L::s_quat + i] = q[i];
#pragma unroll
  for (int d = 0; d < K; d++) {
    if (d >= 3 && d < 6) continue;
    const bool in = j <= d;
    const double ld = sm.S[d * (d + 1) / 2 + (in ? j : d)];
    x[d2s(d)] = sm.mu[d2s(d)] + sg * (in ? ld : 0.0);
  }
  h(x, z);
}

// R sums over NL lanes through a CAP-double buffer, in rounds of CAP / NL rows
template <int R, int NL, int CAP, int C0 = 0>
UWVK_DEV void lds_sums_cap(const double (&v)[R], double* buf, int l, double (&out)[R]) {
  if constexpr (C0 < R) {
    constexpr int CH0 = CAP / NL, CH = (R - C0) < CH0 ? (R - C0) : CH0;
    static_assert(NL % 2 == 0 && NL <= 64 && CH0 >= 1, "transpose buffer");
    if (l < NL) {
#pragma unroll
      for (int i = 0; i < CH; i++) buf[i * NL + l] = v[C0 + i];
    }
    wsync();
    const double* row = buf + (l < CH ? l : 0) * NL;
    double p[NL / 2];
#pragma unroll
    for (int k = 0; k < NL / 2; k++) p[k] = row[2 * k] + row[2 * k + 1];
#pragma unroll
    for (int w = 1; w < NL / 2; w *= 2)
#pragma unroll
      for (int k = 0; k + w < NL / 2; k += 2 * w) p[k] += p[k + w];
#pragma unroll
    for (int i = 0; i < CH; i++) out[C0 + i] = readlane_d(p[0], i);
    wsync();  // every lane's reads of this round before the next round's writes
    lds_sums_cap<R, NL, CAP, C0 + CH>(v, buf, l, out);
  }
}

// S x = b for a symmetric positive definite M x M S (lower triangle packed,
// row i at i (i + 1) / 2): S = L L^T (1 / L_ii kept), then two substitutions
template <int M>
UWVK_DEV void spd_factor(const double (&S)[M * (M + 1) / 2], double (&L)[M * (M + 1) / 2], double (&idg)[M]) {
#pragma unroll
  for (int j = 0; j < M; j++) {
    double d = S[j * (j + 1) / 2 + j];
#pragma unroll
    for (int k = 0; k < j; k++) d -= L[j * (j + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
    idg[j] = rsqrt_f64(d);
    L[j * (j + 1) / 2 + j] = d * idg[j];
#pragma unroll
    for (int i = j + 1; i < M; i++) {
      double t = S[i * (i + 1) / 2 + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= L[i * (i + 1) / 2 + k] * L[j * (j + 1) / 2 + k];
      L[i * (i + 1) / 2 + j] = t * idg[j];
    }
  }
}
template <int M>
UWVK_DEV void spd_solve(const double (&L)[M * (M + 1) / 2], const double (&idg)[M], const double (&b)[M],
                        double (&x)[M]) {
  double y[M];
#pragma unroll
  for (int i = 0; i < M; i++) {
    double t = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) t -= L[i * (i + 1) / 2 + k] * y[k];
    y[i] = t * idg[i];
  }
#pragma unroll
  for (int i = M - 1; i >= 0; i--) {
    double t = y[i];
#pragma unroll
    for (int k = i + 1; k < M; k++) t -= L[k * (k + 1) / 2 + i] * x[k];
    x[i] = t * idg[i];
  }
}

// the full BodyEfforts update (gate: accept any).  sig_hbm: the instance's
// Sigma in HBM (what sm.S held before the factor overwrote it).
// PRECONDITION: sm.S holds Sigma itself, not the epoch kernel's time-scaled
// Sigma~ = D^-1 Sigma D^-1 (ds = ids = 1: the state load_psp leaves), and
// sig_hbm holds the same Sigma.  Both callers (k_psp_efforts, k_psp_update)
// load the instance just before the call; fusing this update into
// k_psp_epoch's epoch loop needs psp_fold first (tests/test_gpu_efforts.py
// holds run_log's efforts epochs to the literal kernel at a full grid).  z and R are
// read where they are used (held in registers through the factor and the
// points they were 84 VGPRs of the kernel's peak)
template <int DOF, int SR, class HM>
UWVK_DEV bool psp_update_eff(PspSmem<DOF>& sm, const double* sig_hbm, const HM& h, const double* z,
                             const double* Rm, bool* ok) {
  using G = PG<DOF>;
  constexpr int M = 6, K = HJmax<HM, DOF>::value, NL = (K + 2) & ~1;
  static_assert(K < 64 && NL <= 64, "one point pair per lane, the centre in lane K");
  int l = olane();
  bool cok = true;
  eff_chol<DOF, 0>(sm.S, sm.stg, l, cok);
  l = olane();
  const bool pt = LANE_IF(l, l < K);
  const int j = pt ? l : 0;
  const double sg = pt ? 1.0 : 0.0;
  double zp[M], zn[M], zc[M];
  {
    // the two evaluations one after the other: a scheduling barrier and a
    // memory clobber keep the second's LDS reads (and the values the compiler
    // would otherwise share between them) out of the first (register peak)
    double qp[4], qn[4];
    eff_point_quat<DOF, SR>(sm, j, sg, qp);
    eff_point_quat<DOF, SR>(sm, j, -sg, qn);
    __builtin_amdgcn_sched_barrier(0);
    eff_point<DOF, K>(sm, h, j, sg, qp, zp);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    eff_point<DOF, K>(sm, h, j, -sg, qn, zn);
  }
#pragma unroll
  for (int a = 0; a < M; a++) zc[a] = readlane_d(zp[a], K);
  // C_r = 1/2 sum_{j < K} L[r][j] Dz_j, Dz_j = z_{j+} - z_{j-} from lane j,
  // staged CH columns at a time
  double C[M];
  {
    constexpr int CH = 16;
    static_assert(CH * M <= G::STG, "Dz chunk (PG::STG)");
    const int rr = l < DOF ? l : DOF - 1;
    const double* Lr = sm.S + ((rr * (rr + 1)) >> 1);
    double c[M];
#pragma unroll
    for (int a = 0; a < M; a++) c[a] = 0.0;
#pragma unroll
    for (int j0 = 0; j0 < K; j0 += CH) {
      if (l >= j0 && l < j0 + CH && l < K) {
#pragma unroll
        for (int a = 0; a < M; a++) sm.stg[(l - j0) * M + a] = zp[a] - zn[a];
      }
      wsync();
#pragma unroll
      for (int jj = 0; jj < CH && j0 + jj < K; jj++) {
        const int jv = j0 + jj;
        const double lv = Lr[jv <= rr ? jv : rr];
        const double lr = jv <= rr ? lv : 0.0;
#pragma unroll
        for (int a = 0; a < M; a++) c[a] += lr * sm.stg[jj * M + a];
#pragma unroll
        for (int a = 0; a < M; a++) asm volatile("" : "+v"(c[a])::"memory");
      }
      wsync();
    }
#pragma unroll
    for (int a = 0; a < M; a++) C[a] = 0.5 * c[a];
  }
  psync();  // every lane's reads of L: the triangle's area takes the sums
  constexpr int R = M + M * (M + 1) / 2;
  double sums[R];
  {
    double up[M], un[M], v[R];
#pragma unroll
    for (int a = 0; a < M; a++) {
      up[a] = pt ? zp[a] - zc[a] : 0.0;
      un[a] = pt ? zn[a] - zc[a] : 0.0;
      v[a] = up[a] + un[a];
    }
    int k = M;
#pragma unroll
    for (int a = 0; a < M; a++)
#pragma unroll
      for (int b2 = 0; b2 <= a; b2++) v[k++] = up[a] * up[b2] + un[a] * un[b2];
    lds_sums_cap<R, NL, G::NP>(v, sm.S, l, sums);
  }
  constexpr double wc = 1.0 + 2.0 * (DOF - K);
  constexpr int NS = M * (M + 1) / 2;
  double Sl[NS], nu[M];  // innovation covariance (lower, packed), z - zbar
  {
    double m[M], e[M];
#pragma unroll
    for (int a = 0; a < M; a++) {
      m[a] = sums[a] * (1.0 / (double)G::N);
      const double zb = zc[a] + m[a];
      e[a] = zc[a] - zb;
      nu[a] = z[a] - zb;
    }
    int k = M, t = 0;
#pragma unroll
    for (int a = 0; a < M; a++)
#pragma unroll
      for (int b2 = 0; b2 <= a; b2++) {
        const double s = sums[k++] - m[a] * sums[b2] - m[b2] * sums[a] + (2.0 * K) * m[a] * m[b2];
        Sl[t++] = 0.5 * (s + wc * e[a] * e[b2]) + Rm[a * M + b2];
      }
  }
  // K_r = S^-1 C_r (lane r), delta_r = C_r . S^-1 nu (S symmetric positive definite)
  double Kg[M], dl = 0.0;
  {
    double Ls[NS], idg[M], w[M];
    spd_factor<M>(Sl, Ls, idg);
    spd_solve<M>(Ls, idg, nu, w);
    spd_solve<M>(Ls, idg, C, Kg);
#pragma unroll
    for (int i = 0; i < M; i++) dl += C[i] * w[i];
  }
  *ok = cok;
  // Sigma back from HBM (the factor and the sums overwrote the triangle)
  {
    double sv[G::NSLOT];
#pragma unroll
    for (int t = 0; t < G::NSLOT; t++) {
      const int ee = l + 64 * t;
      sv[t] = ee < G::NP ? sig_hbm[ee] : 0.0;
    }
    wsync();  // the sums' reads of the area before its rewrite
#pragma unroll
    for (int t = 0; t < G::NSLOT; t++) {
      const int ee = l + 64 * t;
      if (ee < G::NP) sm.S[ee] = sv[t];
    }
  }
  psync();
  {
    double c0[3], k0[3], c1[3], k1[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      c0[i] = C[i];
      k0[i] = Kg[i];
      c1[i] = C[3 + i];
      k1[i] = Kg[3 + i];
    }
    rankm_mfma_o<DOF, 3>(sm.S, sm.stg, c0, k0, l);
    psync();
    rankm_mfma_o<DOF, 3>(sm.S, sm.stg, c1, k1, l);
  }
  psync();
  psp_apply_delta<DOF, SR>(sm, dl, l);
  return true;
}

#endif  // !PSP_PAIR

}  // namespace PSP_NS
}  // namespace uwvk
