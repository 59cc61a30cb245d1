// uwvk_pose_dev.hpp — PoseUKF predict / update as workgroup-per-filter device
// code for gfx950.
//
// Work split inside the workgroup of T = 64*NW threads (NW wavefronts, one
// PoseUKF instance; NW = 2 for the 53-DOF state, 1 for the 26-DOF subset):
//   * Sigma (n x n fp64) lives in LDS for the whole call.
//   * Cholesky: wavefront 0, lane r owns row r in VGPRs, right-looking, column
//     k broadcast through a 64-double LDS buffer.
//   * Sigma points: thread p owns sigma point p (N = 2n+1 <= T); process and
//     measurement models run per thread in VGPRs (one 54-double state each).
//   * Means and small reductions: shuffle folds + LDS transpose sums.
//   * Covariance reconstruction Sigma = 1/2 D D^T (+Q'): v_mfma_f64_16x16x4_f64
//     over the n x N deviation matrix D, staged through LDS in 32-point chunks;
//     the upper 16x16 tiles are dealt round-robin over the wavefronts and
//     accumulate in registers.
//
// The arithmetic follows the reference and the frozen [EXT] spec exactly like
// the CPU oracle (oracle/uwvk_oracle.c, citations there); only summation order
// and FMA contraction differ (parity tolerance in tests/test_gpu_parity.py).
#pragma once
#include "uwvk_dev.hpp"
#include "../../include/uwvk.h"

namespace uwvk {

// ---------------------------------------------------------------------------
// per-handle (batch-shared) parameters, passed by value to every kernel
// ---------------------------------------------------------------------------
struct PoseShared {
  uwvk_pose_parameter p;
  double lat0, lon0, rm, rn_cos, inv_rm;  // GeographicProjection [EXT]: lat = lat0 + x/rm, lon = lon0 - y/rn_cos
  double slat0, clat0;                    // sin / cos of lat0 (PSP: latitude by angle addition)
  double uwv_weight, uwv_buoyancy, cog[3], cob[3];
  int literal_apply_delta;  // 1: ukfom's literal re-spread (Cholesky + GEMM); 0: exact T Sigma T^T form
  // -1/tau of the first-order Markov states (host-computed; IEEE division, so
  // bitwise equal to evaluating (-1.0 / tau) in the process model)
  double ntau[8];  // gyro bias, acc bias, inertia, lin damping, quad damping, water velocity, ADCP bias, density
  double q_ori[9];  // Q's orientation block (PSP kernels; host copy of process_noise_cov)
  double q_wv[4];   // Q's water-velocity / water-velocity-below diagonal
  // dt^2 Q band of the rows >= 9 (PSP decay pass): row i holds cols [qlo[i], i]
  // at qb[qoff[i]...]; q_band = 0 when the band does not fit (global fallback)
  int qlo[56], qoff[56], q_band;
  int q_bw;  // max band width below the diagonal over rows >= 9 (PSP keeps <= 2 in registers)
  int q_simple;  // PSP: lane-resident dt^2 Q suffices (see psp::LaneQ)
  int so3_right;  // UWVK_OPT_SO3_RIGHT: body-frame SO3 [+]/[-] (default 1; literal kernels: qplus_side, PSP: the SR instantiation)
  // run_log's per-log measurement covariances, read by the PSP epoch kernel
  // through the per-epoch constant-space pointer (scalar loads where used):
  // from the kernel arguments they were SGPRs live across the epoch loop,
  // spilled to VGPR lanes and read back ~2x per epoch (tools/spill_report.py)
  double log_acc_cov[9], log_dvl_cov[9];
};

struct PoseBufs {
  int64_t batch;
  double* mu;         // [batch][store]
  double* sigma;      // [batch][dof*dof]
  const double* Q;    // [dof*dof] process_noise_cov (shared)
  double* rot;        // [batch][3] stored RotationRate (PoseUKF.cpp:492-496)
  double* off;        // [batch][28] inertia/lin/quad offsets (9 each, col-major) + density offset
  double* model;      // [batch][27] the shared DynamicModel's (surge,sway,yaw) blocks (PoseUKF.cpp:173)
  const double* uwv;  // [108] base M, D_l, D_q (row-major 6x6)
  uint32_t* status;   // [batch]
  const PoseShared* shared;  // device copy of the handle's PoseShared (PSP kernels)
  const double* Qp;          // {A_ii A_jj, dt^2 Q_ij} per packed entry (PSP kernels; host-made per dt)
  const double* qband;       // [128] dt^2 Q band of rows >= 9 (PSP kernels)
};

template <int DOF>
struct NWaves {
  static constexpr int value = (2 * DOF + 1 + 63) / 64;
};

// geometry of the LDS staging for the MFMA covariance GEMM
template <int DOF>
struct Geo {
  static constexpr int NW = NWaves<DOF>::value;
  static constexpr int T = 64 * NW;                    // threads per filter
  static constexpr int N = 2 * DOF + 1;                // sigma points (<= T)
  static constexpr int NT = (DOF + 15) / 16;           // 16-row tiles per dimension
  static constexpr int NTILE = NT * (NT + 1) / 2;      // upper tiles
  static constexpr int TPW = (NTILE + NW - 1) / NW;    // tiles per wave
  static constexpr int STR = 16 * NT + 1;              // staging row stride (odd: conflict-free writes)
  static constexpr int NCHUNK = (N + 31) / 32;         // 32-point chunks
  static constexpr int RS = DOF | 1;                   // transpose-sum row stride
  static constexpr int RROWS = 16 * NW;                // rows after folding each wave 64 -> 16
  static constexpr int A = DOF * DOF, B = 32 * STR, C = RROWS * RS;
  static constexpr int SZ = (A > B ? (A > C ? A : C) : (B > C ? B : C));
  static constexpr int LP = DOF * (DOF + 1) / 2;
  static constexpr int LC = 16 * (DOF | 1) + 16 * 8;   // update staging: dx rows + dz rows
  static constexpr int LK = DOF * 6;                   // Kalman gain rows
  static constexpr int LPSZ = LP > LC ? (LP > LK ? LP : LK) : (LC > LK ? LC : LK);  // packed L / staging / K
  static_assert(N <= T, "one sigma point per thread");
};

template <int NT>
struct TileIJ;
// compile-time (i, j) of upper tile TT (template constants: always folded)
template <int NT, int TT>
struct TileAt {
  static constexpr int i = TileIJ<NT>::i(TT);
  static constexpr int j = TileIJ<NT>::j(TT);
};
template <int NT>
struct TileIJ {  // t -> (i, j) over the upper tiles, row-major
  __host__ __device__ static constexpr int i(int t) {
    int r = 0, k = t;
    while (k >= NT - r) { k -= NT - r; r++; }
    return r;
  }
  __host__ __device__ static constexpr int j(int t) {
    int r = 0, k = t;
    while (k >= NT - r) { k -= NT - r; r++; }
    return r + k;
  }
};

template <int DOF>
struct alignas(16) Smem {
  double S[Geo<DOF>::SZ];  // Sigma (row-major, stride DOF) / D staging / reduction scratch
  double Lp[Geo<DOF>::LPSZ];  // Cholesky factor, packed lower triangle (row r at r(r+1)/2) / dx staging
  double mu[56];           // current mean (store layout)
  double ref[56];          // scratch state (X0 / mean under construction)
  double col[2][64];       // Cholesky column broadcast (double-buffered)
  double vec[64];          // broadcast vectors (sums, delta)
  double red[2][24];       // cross-wave partial sums
  double qori[9];          // R Q_ori R^T for the predict
  // ref .. red as one scratch run (the update's Dz staging, when none of them is live)
  static constexpr int kScratch = 56 + 2 * 64 + 64 + 2 * 24;
  UWVK_DEV double* scratch() { return ref; }
};

UWVK_DEV int tid() { return threadIdx.x; }
// wave index as a scalar (SGPR): branches on it are uniform (s_cbranch_scc)
UWVK_DEV int wid() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// intra-wavefront ordering point for LDS exchanges done by one wave
UWVK_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// sum of K values over all threads of the workgroup; result in every thread
template <int DOF, int K>
UWVK_DEV void block_sum(Smem<DOF>& sm, double (&v)[K]) {
  constexpr int NW = Geo<DOF>::NW;
#pragma unroll
  for (int k = 0; k < K; k++) v[k] = wave_sum(v[k]);
  if constexpr (NW > 1) {
    static_assert(K <= 24 && NW <= 2, "block_sum width");
    if (lane_id() == 0) {
#pragma unroll
      for (int k = 0; k < K; k++) sm.red[wid()][k] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; k++) {
      double s = sm.red[0][k];
#pragma unroll
      for (int w = 1; w < NW; w++) s += sm.red[w][k];
      v[k] = s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Cholesky of S into the packed factor sm.Lp by wavefront 0 (S is kept).  Returns false (uniform) if a
// pivot is not > 0.
// ---------------------------------------------------------------------------
// 1/sqrt(x): hardware v_rsq_f64 seed + one third-order correction
// (e = 1 - x r^2; r += r e (1/2 + 3/8 e)), full fp64 precision.
UWVK_DEV double rsqrt_f64(double x) {
  double r = __builtin_amdgcn_rsq(x);
  const double e = fma(-(x * r), r, 1.0);
  return fma(r * e, fma(0.375, e, 0.5), r);
}

// One right-looking column step; template recursion keeps every register index
// a compile-time constant (a runtime-indexed row would live in scratch).
// piv is the final value of A[K][K].  The next pivot comes from lane K+1's own
// registers (L[K+1][K]^2), so the LDS column broadcast is off the critical path.
template <int DOF, int K>
UWVK_DEV void chol_step(double (&a)[DOF], Smem<DOF>& sm, int r, bool& ok, double piv) {
  if constexpr (K < DOF) {
    ok = ok && (piv > 0.0);
    const double inv = rsqrt_f64(piv);
    const double d = piv * inv;
    a[K] = (r == K) ? d : a[K] * inv;
    double pnext = 0.0;
    if constexpr (K + 1 < DOF) pnext = readlane_d(a[K + 1] - a[K] * a[K], K + 1);
    sm.col[K & 1][r] = a[K];
    wave_sync();
#pragma unroll
    for (int c = K + 1; c < DOF; c++) a[c] -= a[K] * sm.col[K & 1][c];
    // keep the update eager: without this the compiler sinks every a[c]
    // update to its first use and keeps O(n^2) column values live (spills)
#pragma unroll
    for (int c = K + 1; c < DOF; c++) asm volatile("" : "+v"(a[c]));
    chol_step<DOF, K + 1>(a, sm, r, ok, pnext);
  }
}

// Two-wave form (NW = 2, the 53-DOF state): wave W keeps columns [C0, C1) of
// every row (27 + 26 doubles per lane instead of 53: no scratch spills), the
// owner of column J scales it and publishes it through the LDS column buffer,
// and both waves update their own later columns in parallel; one workgroup
// barrier per column.  The same operations per entry as chol_step, so the
// factor is bitwise the one-wave factor.
template <int DOF, int W, int C0, int C1, int J>
UWVK_DEV void chol2_step(double (&a)[C1 - C0], Smem<DOF>& sm, int r, bool& ok, double piv) {
  if constexpr (J < DOF) {
    constexpr int H = (DOF + 1) / 2;
    constexpr bool own = (J < H) == (W == 0);
    double pnext = 0.0;
    if constexpr (own) {
      constexpr int jj = J - C0;
      ok = ok && (piv > 0.0);
      const double inv = rsqrt_f64(piv);
      const double d = piv * inv;
      a[jj] = (r == J) ? d : a[jj] * inv;
      if constexpr (J + 1 < C1) pnext = readlane_d(a[jj + 1] - a[jj] * a[jj], J + 1);
      sm.col[J & 1][r] = a[jj];
    }
    __syncthreads();
    const double lr = own ? a[J - C0 < 0 ? 0 : (J - C0 >= C1 - C0 ? 0 : J - C0)] : sm.col[J & 1][r];
#pragma unroll
    for (int c = (J + 1 > C0 ? J + 1 : C0); c < C1; c++) a[c - C0] -= lr * sm.col[J & 1][c];
#pragma unroll
    for (int c = (J + 1 > C0 ? J + 1 : C0); c < C1; c++) asm volatile("" : "+v"(a[c - C0]));
    // the first column of wave 1 takes its pivot from its own updated registers
    if constexpr (W == 1 && J + 1 == C0) pnext = readlane_d(a[0], C0);
    chol2_step<DOF, W, C0, C1, J + 1>(a, sm, r, ok, pnext);
  }
}

// The same two-wave factor with up to kCholGroup columns per barrier
// (columns J .. J+g-1 of one owner): the owner takes each pivot in turn from
// its own lanes (readlane), scales the column and applies it to the group's
// later columns (L[m][k] by readlane), then publishes the g columns; after the
// barrier every wave applies them in order to its later columns.  Each entry
// sees the same fused multiply-adds in the same order as in chol2_step, so the
// factor is bitwise the one-column-per-barrier factor (tools/diag_lib_bitwise.py)
// with 18 barriers instead of 53 at g = 3.  S counts barriers (the buffer set);
// the 2 x g 64-double column buffers live in the factor region sm.Lp, which
// takes the factor only after the last barrier (no buffer is read after it).
// r05: kept form only; the look-ahead (2.51 against 2.42-2.44 ms per efforts
// epoch, profiles/r04/effla/) and cyclic block forms and the one-wave factor
// were measured and dropped (profiles/EXPERIMENTS.md).
constexpr int kCholGroup = 3;
template <int DOF, int J, int GS>
constexpr int chol_group() {  // columns J .. J+g-1 with one owner (the halves of the two waves)
  constexpr int H = (DOF + 1) / 2;
  int g = 1;
  while (g < GS && J + g < DOF && ((J < H) == (J + g < H))) g++;
  return g;
}
template <int DOF, int W, int C0, int C1, int J, int S>
UWVK_DEV void chol2g_step(double (&a)[C1 - C0], Smem<DOF>& sm, int r, bool& ok, double piv) {
  if constexpr (J < DOF) {
    constexpr int H = (DOF + 1) / 2;
    constexpr bool own = (J < H) == (W == 0);
    constexpr int g = chol_group<DOF, J, kCholGroup>();
    constexpr int b0 = (S & 1) * kCholGroup;
    constexpr int JN = J + g;  // first column after this step
    static_assert(Geo<DOF>::LPSZ >= 2 * kCholGroup * 64, "column buffers in the factor region");
    double* buf = sm.Lp + b0 * 64;
    if constexpr (own) {
      constexpr int jj = J - C0;
#pragma unroll
      for (int k = 0; k < g; k++) {
        const double p = k == 0 ? piv : readlane_d(a[jj + k], J + k);
        ok = ok && (p > 0.0);
        const double inv = rsqrt_f64(p);
        const double d = p * inv;
        a[jj + k] = (r == J + k) ? d : a[jj + k] * inv;
        buf[k * 64 + r] = a[jj + k];
#pragma unroll
        for (int m = k + 1; m < g; m++) {
          const double lmk = readlane_d(a[jj + k], J + m);  // L[J+m][J+k]
          a[jj + m] -= a[jj + k] * lmk;
          asm volatile("" : "+v"(a[jj + m]));
        }
      }
    }
    __syncthreads();
    constexpr int cs = JN > C0 ? JN : C0;
    if constexpr (cs < C1) {
#pragma unroll
      for (int k = 0; k < g; k++) {
        const double lk = own ? a[(J + k - C0) >= 0 && (J + k - C0) < (C1 - C0) ? J + k - C0 : 0] : buf[k * 64 + r];
#pragma unroll
        for (int c = cs; c < C1; c++) a[c - C0] -= lk * buf[k * 64 + c];
      }
#pragma unroll
      for (int c = cs; c < C1; c++) asm volatile("" : "+v"(a[c - C0]));
    }
    // the next pivot: lane JN's fully updated entry (owner of column JN only)
    double pnext = 0.0;
    if constexpr (JN < DOF && JN >= C0 && JN < C1) pnext = readlane_d(a[JN - C0], JN);
    chol2g_step<DOF, W, C0, C1, JN, S + 1>(a, sm, r, ok, pnext);
  }
}

template <int DOF, int W, int C0, int C1>
UWVK_DEV void chol2_wave(Smem<DOF>& sm) {
  const int r = lane_id();
  const int rr = r < DOF ? r : DOF - 1;  // lanes >= DOF shadow the last row (discarded)
  double a[C1 - C0];
#pragma unroll
  for (int c = C0; c < C1; c++) a[c - C0] = sm.S[rr * DOF + c];
  bool ok = true;
  chol2g_step<DOF, W, C0, C1, 0, 0>(a, sm, r, ok, W == 0 ? readlane_d(a[0], 0) : 0.0);
  if (r < DOF) {
    const int base = r * (r + 1) / 2;
#pragma unroll
    for (int c = C0; c < C1; c++)
      if (c <= r) sm.Lp[base + c] = a[c - C0];
  }
  if (r == 0) sm.vec[62 + W] = ok ? 1.0 : 0.0;
}

template <int DOF>
UWVK_DEV bool chol_lds(Smem<DOF>& sm) {
  if constexpr (Geo<DOF>::NW == 2) {
    constexpr int H = (DOF + 1) / 2;
    if (wid() == 0)
      chol2_wave<DOF, 0, 0, H>(sm);
    else
      chol2_wave<DOF, 1, H, DOF>(sm);
    __syncthreads();
    const bool ok = sm.vec[62] != 0.0 && sm.vec[63] != 0.0;
    __syncthreads();
    return ok;
  }
  if (wid() == 0) {
    const int r = lane_id();
    const int rr = r < DOF ? r : DOF - 1;  // lanes >= DOF shadow the last row (discarded)
    double a[DOF];
#pragma unroll
    for (int c = 0; c < DOF; c++) a[c] = sm.S[rr * DOF + c];
    bool ok = true;
    chol_step<DOF, 0>(a, sm, r, ok, readlane_d(a[0], 0));
    if (r < DOF) {
      const int base = r * (r + 1) / 2;
#pragma unroll
      for (int c = 0; c < DOF; c++)
        if (c <= r) sm.Lp[base + c] = a[c];
    }
    if (r == 0) sm.vec[63] = ok ? 1.0 : 0.0;
  }
  __syncthreads();
  const bool ok = sm.vec[63] != 0.0;
  __syncthreads();
  return ok;
}

// sigma point p (0..N-1) of (mu, L) into x (store layout):
// X0 = mu, X_{2j+1} = mu [+] L_j, X_{2j+2} = mu [+] -L_j
template <int DOF>
UWVK_DEV void gen_point(const Smem<DOF>& sm, int p, double x[Lay<DOF>::store], int right) {
  using L = Lay<DOF>;
#pragma unroll
  for (int s = 0; s < L::store; s++) x[s] = sm.mu[s];
  if (p <= 0 || p >= Geo<DOF>::N) return;
  const int j = (p - 1) >> 1;
  const double sg = (p & 1) ? 1.0 : -1.0;
#pragma unroll
  for (int d = 0; d < DOF; d++) {
    if (d >= 3 && d < 6) continue;
    const double l = (d >= j) ? sm.Lp[d * (d + 1) / 2 + j] : 0.0;
    x[d2s(d)] = sm.mu[d2s(d)] + sg * l;
  }
  if (j <= 5) {  // columns j > 5 of a lower-triangular L have no orientation entries
    double v[3], e[4];
#pragma unroll
    for (int i = 0; i < 3; i++) v[i] = sg * ((3 + i >= j) ? sm.Lp[(3 + i) * (4 + i) / 2 + j] : 0.0);
    so3_exp(v, e);
    qplus_side(e, sm.mu + L::s_quat, x + L::s_quat, right);
  }
}

// x [-] m (store -> tangent), m read from LDS
template <int DOF>
UWVK_DEV void boxminus_lds(const double x[Lay<DOF>::store], const double* m, double d[DOF], int right) {
#pragma unroll
  for (int k = 0; k < DOF; k++) {
    if (k >= 3 && k < 6) continue;
    d[k] = x[d2s(k)] - m[d2s(k)];
  }
  const double q[4] = {m[3], m[4], m[5], m[6]};
  qboxminus_side(x + 3, q, d + 3, right);
}

// x [+] delta (delta uniform, from LDS)
template <int DOF>
UWVK_DEV void boxplus_vec(double x[Lay<DOF>::store], const double* delta, int right) {
#pragma unroll
  for (int k = 0; k < DOF; k++) {
    if (k >= 3 && k < 6) continue;
    x[d2s(k)] = x[d2s(k)] + 1.0 * delta[k];
  }
  double e[4], q[4];
  const double dv[3] = {delta[3], delta[4], delta[5]};
  so3_exp(dv, e);
  qplus_side(e, x + 3, q, right);
#pragma unroll
  for (int i = 0; i < 4; i++) x[3 + i] = q[i];
}

// ---------------------------------------------------------------------------
// Sum over all threads of a per-thread vector v[DOF], result into sm.vec.
// Fold each wave 64 -> 16 with two shuffles, LDS transpose, thread c sums
// column c.  Uses sm.S as scratch (must be free).
// ---------------------------------------------------------------------------
template <int DOF>
UWVK_DEV void lane_sum_vec(Smem<DOF>& sm, double (&v)[DOF]) {
  using G = Geo<DOF>;
  const int l = lane_id(), w = wid();
#pragma unroll
  for (int k = 0; k < DOF; k++) {
    double a = v[k] + shfl_xor_d(v[k], 32);
    a = a + shfl_xor_d(a, 16);
    if (l < 16) sm.S[(16 * w + l) * G::RS + k] = a;
  }
  __syncthreads();
  const int t = tid();
  if (t < DOF) {
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
    for (int r = 0; r < G::RROWS; r += 4) {
      s0 += sm.S[r * G::RS + t];
      s1 += sm.S[(r + 1) * G::RS + t];
      s2 += sm.S[(r + 2) * G::RS + t];
      s3 += sm.S[(r + 3) * G::RS + t];
    }
    sm.vec[t] = (s0 + s1) + (s2 + s3);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Sigma = 0.5 * D D^T over the per-thread deviations d (point = thread), via
// v_mfma_f64_16x16x4_f64.  Upper tile t is owned by wave t % NW.
// ---------------------------------------------------------------------------
// MFMAs of wave W's tiles U, U+1, ... for one k-step (fragments f)
template <int DOF, int W, int U>
UWVK_DEV void mfma_tiles(const double (&f)[Geo<DOF>::NT], d4_t (&acc)[Geo<DOF>::TPW]) {
  using G = Geo<DOF>;
  constexpr int TT = W + G::NW * U;
  if constexpr (U < G::TPW && TT < G::NTILE) {
    acc[U] = mfma_f64(f[TileAt<G::NT, TT>::i], f[TileAt<G::NT, TT>::j], acc[U]);
    mfma_tiles<DOF, W, U + 1>(f, acc);
  }
}

// one staged chunk of KS k-steps for wave W: straight-line, static tile list
template <int DOF, int W, int KS>
UWVK_DEV void gemm_chunk(const Smem<DOF>& sm, d4_t (&acc)[Geo<DOF>::TPW]) {
  using G = Geo<DOF>;
  const int l = lane_id();
  double f[KS][G::NT];
#pragma unroll
  for (int s = 0; s < KS; s++)
#pragma unroll
    for (int i = 0; i < G::NT; i++) f[s][i] = sm.S[(4 * s + (l >> 4)) * G::STR + 16 * i + (l & 15)];
#pragma unroll
  for (int s = 0; s < KS; s++) mfma_tiles<DOF, W, 0>(f[s], acc);
}

// chunk C of 32 points: stage (threads 32C..32C+31), barrier, MFMAs, barrier
template <int DOF, int C>
UWVK_DEV void gemm_chunks(Smem<DOF>& sm, const double (&d)[DOF], d4_t (&acc)[Geo<DOF>::TPW]) {
  using G = Geo<DOF>;
  if constexpr (C < G::NCHUNK) {
    const int t = tid(), w = wid();
    if ((t >> 5) == C) {
      const int row = t & 31;
      const bool valid = t < G::N;
#pragma unroll
      for (int k = 0; k < 16 * G::NT; k++) sm.S[row * G::STR + k] = (k < DOF && valid) ? d[k] : 0.0;
    }
    __syncthreads();
    constexpr int NP = (G::N - 32 * C) < 32 ? (G::N - 32 * C) : 32;
    constexpr int KS = (NP + 3) / 4;
    if (w == 0) gemm_chunk<DOF, 0, KS>(sm, acc);
    if constexpr (G::NW > 1) {
      if (w == 1) gemm_chunk<DOF, 1, KS>(sm, acc);
    }
    __syncthreads();
    gemm_chunks<DOF, C + 1>(sm, d, acc);
  }
}

template <int DOF>
UWVK_DEV void cov_gemm(Smem<DOF>& sm, const double (&d)[DOF], d4_t (&acc)[Geo<DOF>::TPW]) {
#pragma unroll
  for (int u = 0; u < Geo<DOF>::TPW; u++) acc[u] = d4_t{0.0, 0.0, 0.0, 0.0};
  gemm_chunks<DOF, 0>(sm, d, acc);
}

template <int DOF, int W, int U, class QF>
UWVK_DEV void store_tiles(Smem<DOF>& sm, const d4_t (&acc)[Geo<DOF>::TPW], QF& qfun) {
  using G = Geo<DOF>;
  constexpr int TT = W + G::NW * U;
  if constexpr (U < G::TPW && TT < G::NTILE) {
    constexpr int i = TileAt<G::NT, TT>::i, j = TileAt<G::NT, TT>::j;
    const int l = lane_id();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int r = 16 * i + (l >> 4) + 4 * q, c = 16 * j + (l & 15);
      if (r < DOF && c < DOF) {
        const double v = 0.5 * acc[U][q] + qfun(r, c);
        sm.S[r * DOF + c] = v;
        if (i != j) sm.S[c * DOF + r] = v;
      }
    }
    store_tiles<DOF, W, U + 1>(sm, acc, qfun);
  }
}

// write 0.5*acc + qfun(r, c) into sm.S (full symmetric)
template <int DOF, class QF>
UWVK_DEV void store_cov(Smem<DOF>& sm, const d4_t (&acc)[Geo<DOF>::TPW], QF qfun) {
  const int w = wid();
  if (w == 0) store_tiles<DOF, 0, 0>(sm, acc, qfun);
  if constexpr (Geo<DOF>::NW > 1) {
    if (w == 1) store_tiles<DOF, 1, 0>(sm, acc, qfun);
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// process model, PoseUKF.cpp:12-84 (per sigma point, in registers)
// ---------------------------------------------------------------------------
struct ProcCtx {
  double w[3];        // stored rotation rate
  double dt;
  const double* off;  // per-instance offsets (global, uniform address)
  double off_lane;    // PSP: the one offset storage component `lane` decays towards
  double nt_lane;     // PSP: -1/tau of storage component `lane` (0: not a Markov state)
  double nt_tan;      // PSP: -1/tau of tangent DOF `lane` if it is time-scaled (scaled_dof), else 0
  int vpart;          // PSP: storage index added times dt (pos <- vel, vel <- acc), or -1
};

template <int DOF>
UWVK_DEV void process_point(double x[Lay<DOF>::store], const PoseShared& sh, const ProcCtx& c) {
  using L = Lay<DOF>;
  const double dt = c.dt;
  const uwvk_pose_parameter& P = sh.p;
  // orientation first (reads pre-step position / bias / orientation)
  const double lat = sh.lat0 + x[L::s_pos] * sh.inv_rm;  // navToWorld [EXT]
  double sl, cl;
  sincos(lat, &sl, &cl);
  const double er[3] = {kEarthW * cl, 0.0, kEarthW * sl};
  double wb[3], wn[3];
#pragma unroll
  for (int i = 0; i < 3; i++) wb[i] = c.w[i] - x[L::s_bg + i];
  qrot(x + L::s_quat, wb, wn);
#pragma unroll
  for (int i = 0; i < 3; i++) wn[i] = (wn[i] - er[i]) * dt;
  double e[4], q[4];
  so3_exp(wn, e);
  qplus_side(e, x + L::s_quat, q, sh.so3_right);
#pragma unroll
  for (int i = 0; i < 4; i++) x[L::s_quat + i] = q[i];
  // vector parts: every update reads only pre-step values of other blocks
#pragma unroll
  for (int i = 0; i < 3; i++) {
    x[L::s_pos + i] = x[L::s_pos + i] + dt * x[L::s_vel + i];
    x[L::s_vel + i] = x[L::s_vel + i] + dt * x[L::s_acc + i];
    const double dg = (-1.0 / P.gyro_bias_tau) * (x[L::s_bg + i] - P.gyro_bias_offset[i]);
    x[L::s_bg + i] = x[L::s_bg + i] + dt * dg;
    const double da = (-1.0 / P.acc_bias_tau) * (x[L::s_ba + i] - P.acc_bias_offset[i]);
    x[L::s_ba + i] = x[L::s_ba + i] + dt * da;
  }
  if constexpr (L::has_params) {
#pragma unroll
    for (int k = 0; k < 9; k++) {
      const double di = (-1.0 / P.inertia_tau) * (x[L::s_inertia + k] - c.off[k]);
      x[L::s_inertia + k] = x[L::s_inertia + k] + dt * di;
      const double dl = (-1.0 / P.lin_damping_tau) * (x[L::s_lin + k] - c.off[9 + k]);
      x[L::s_lin + k] = x[L::s_lin + k] + dt * dl;
      const double dq = (-1.0 / P.quad_damping_tau) * (x[L::s_quad + k] - c.off[18 + k]);
      x[L::s_quad + k] = x[L::s_quad + k] + dt * dq;
    }
  }
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const double dw = (-1.0 / P.water_velocity_tau) * x[L::s_wv + k];
    x[L::s_wv + k] = x[L::s_wv + k] + dt * dw;
    const double db = (-1.0 / P.water_velocity_tau) * x[L::s_wvb + k];
    x[L::s_wvb + k] = x[L::s_wvb + k] + dt * db;
    const double dad = (-1.0 / P.adcp_bias_tau) * x[L::s_badcp + k];
    x[L::s_badcp + k] = x[L::s_badcp + k] + dt * dad;
  }
  const double dr = (-1.0 / P.water_density_tau) * (x[L::s_rho] - c.off[27]);
  x[L::s_rho] = x[L::s_rho] + dt * dr;
}

// ---------------------------------------------------------------------------
// predictionStepImpl (PoseUKF.cpp:446-465) + ukf::predict [EXT]
// ---------------------------------------------------------------------------
template <int DOF>
UWVK_DEV bool pose_predict(Smem<DOF>& sm, const PoseShared& sh, const ProcCtx& pc, const double* Q,
                           Stamper* st = nullptr) {
  using L = Lay<DOF>;
  using G = Geo<DOF>;
  const int t = tid();
  const double dt = pc.dt;
  const bool mine = t < G::N;
  // --- process noise shaping with the PRE-predict mean (PoseUKF.cpp:448-460)
  if (t < 9) {
    double R[9];
    qmatrix(sm.mu + L::s_quat, R);
    const int r = t / 3, c = t % 3, o = L::d_ori;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      double u = 0.0;
#pragma unroll
      for (int m = 0; m < 3; m++) u += R[r * 3 + m] * Q[(o + m) * DOF + o + k];
      s += u * R[c * 3 + k];
    }
    sm.qori[t] = s;
  }
  const double vs0 = sm.mu[L::s_vel], vs1 = sm.mu[L::s_vel + 1], vs2 = 10 * sm.mu[L::s_vel + 2];
  const double wv_add = sh.p.water_velocity_scale * (vs0 * vs0 + vs1 * vs1 + vs2 * vs2) * dt;
  const double dt2 = dt * dt;
  // --- sigma points through the process model
  const bool ok = chol_lds<DOF>(sm);
  UWVK_STAMP(0);
  double x[L::store];
  gen_point<DOF>(sm, t, x, sh.so3_right);
  process_point<DOF>(x, sh, pc);
  // X0 (thread 0's point) as the first reference of the manifold mean
  if (t == 0) {
#pragma unroll
    for (int s = 0; s < L::store; s++) sm.ref[s] = x[s];
  }
  __syncthreads();  // L dead from here on; ref visible
  UWVK_STAMP(1);
  // --- manifold mean (Gauss-Newton, |delta| <= 1e-6, max 1e4 iterations)
  double nrm2 = 0.0;
  double dori[3];
  {
    double d[DOF];
    boxminus_lds<DOF>(x, sm.ref, d, sh.so3_right);
    if (!mine) {
#pragma unroll
      for (int k = 0; k < DOF; k++) d[k] = 0.0;
    }
    lane_sum_vec<DOF>(sm, d);
  }
  if (t < DOF) {
    const double dd = sm.vec[t] / (double)G::N;
    if (t < 3 || t >= 6) sm.ref[d2s(t)] = sm.ref[d2s(t)] + 1.0 * dd;
  }
#pragma unroll
  for (int k = 0; k < DOF; k++) {
    const double dd = sm.vec[k] / (double)G::N;
    nrm2 += dd * dd;
    if (k >= 3 && k < 6) dori[k - 3] = dd;
  }
  double mq[4];
  {
    double e[4];
    const double q0[4] = {sm.ref[3], sm.ref[4], sm.ref[5], sm.ref[6]};
    so3_exp(dori, e);
    qplus_side(e, q0, mq, sh.so3_right);
  }
  int it = 0;
  while (sqrt(nrm2) > 1e-6 && ++it < 10000) {
    // orientation-only refinement: the vect parts are already the exact mean
    double la[3];
    qboxminus_side(x + L::s_quat, mq, la, sh.so3_right);
    if (!mine) la[0] = la[1] = la[2] = 0.0;
    block_sum<DOF, 3>(sm, la);
    nrm2 = 0.0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      la[i] = la[i] / (double)G::N;
      nrm2 += la[i] * la[i];
    }
    double e[4], q[4];
    so3_exp(la, e);
    qplus_side(e, mq, q, sh.so3_right);
#pragma unroll
    for (int i = 0; i < 4; i++) mq[i] = q[i];
  }
  __syncthreads();
  if (t < 4) sm.ref[3 + t] = mq[t];
  __syncthreads();
  UWVK_STAMP(2);
  // --- deviations and covariance reconstruction
  d4_t acc[G::TPW];
  {
    double d[DOF];
    boxminus_lds<DOF>(x, sm.ref, d, sh.so3_right);
    cov_gemm<DOF>(sm, d, acc);
  }
  auto qf = [&](int r, int c) -> double {
    double q = Q[r * DOF + c];
    if (r >= L::d_ori && r < L::d_ori + 3 && c >= L::d_ori && c < L::d_ori + 3)
      q = sm.qori[(r - L::d_ori) * 3 + (c - L::d_ori)];
    if (r == c && ((r >= L::d_wv && r < L::d_wv + 2) || (r >= L::d_wvb && r < L::d_wvb + 2))) q = q + wv_add;
    return dt2 * q;
  };
  store_cov<DOF>(sm, acc, qf);
  if (t < L::store) sm.mu[t] = sm.ref[t];
  __syncthreads();
  UWVK_STAMP(3);
  return ok;
}

// ---------------------------------------------------------------------------
// small m x m inverse (m <= 6), identical formulas to the oracle
// ---------------------------------------------------------------------------
template <int M>
UWVK_DEV void small_inv(const double* A, double* X) {
  if constexpr (M == 1) {
    X[0] = 1.0 / A[0];
  } else if constexpr (M == 2) {
    const double det = A[0] * A[3] - A[1] * A[2];
    const double id = 1.0 / det;
    X[0] = A[3] * id; X[1] = -A[1] * id; X[2] = -A[2] * id; X[3] = A[0] * id;
  } else if constexpr (M == 3) {
    const double c00 = A[4] * A[8] - A[5] * A[7];
    const double c01 = A[5] * A[6] - A[3] * A[8];
    const double c02 = A[3] * A[7] - A[4] * A[6];
    const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
    const double id = 1.0 / det;
    X[0] = c00 * id;
    X[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    X[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    X[3] = c01 * id;
    X[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    X[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    X[6] = c02 * id;
    X[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    X[8] = (A[0] * A[4] - A[1] * A[3]) * id;
  } else {
    double Mx[M][2 * M];
#pragma unroll
    for (int i = 0; i < M; i++)
#pragma unroll
      for (int j = 0; j < 2 * M; j++) Mx[i][j] = j < M ? A[i * M + j] : (j - M == i ? 1.0 : 0.0);
#pragma unroll
    for (int c = 0; c < M; c++) {
      int p = c;
      double best = fabs(Mx[c][c]);
#pragma unroll
      for (int r = c + 1; r < M; r++) {
        const double v = fabs(Mx[r][c]);
        if (v > best) { best = v; p = r; }
      }
#pragma unroll
      for (int r = c + 1; r < M; r++) {
        if (r == p) {
#pragma unroll
          for (int j = 0; j < 2 * M; j++) { double tt = Mx[c][j]; Mx[c][j] = Mx[r][j]; Mx[r][j] = tt; }
        }
      }
      const double ip = 1.0 / Mx[c][c];
#pragma unroll
      for (int j = 0; j < 2 * M; j++) Mx[c][j] *= ip;
#pragma unroll
      for (int r = 0; r < M; r++) {
        if (r == c) continue;
        const double f = Mx[r][c];
        if (f == 0.0) continue;
#pragma unroll
        for (int j = 0; j < 2 * M; j++) Mx[r][j] -= f * Mx[c][j];
      }
    }
#pragma unroll
    for (int i = 0; i < M; i++)
#pragma unroll
      for (int j = 0; j < M; j++) X[i * M + j] = Mx[i][M + j];
  }
}

// ---------------------------------------------------------------------------
// apply_delta [EXT ukfom]: re-spread (mu, Sigma), shift every point and the
// mean by delta, Sigma = 1/2 sum (X'_p [-] mu')(X'_p [-] mu')^T.
// delta (tangent) is in sm.vec.
// ---------------------------------------------------------------------------
template <int DOF>
UWVK_DEV bool apply_delta_literal(Smem<DOF>& sm, int right, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  const int t = tid();
  const bool ok = chol_lds<DOF>(sm);
  UWVK_STAMP(8);
  double x[L::store];
  gen_point<DOF>(sm, t, x, right);
  boxplus_vec<DOF>(x, sm.vec, right);
  if (t == 0) {
    double m[L::store];
#pragma unroll
    for (int s = 0; s < L::store; s++) m[s] = sm.mu[s];
    boxplus_vec<DOF>(m, sm.vec, right);
#pragma unroll
    for (int s = 0; s < L::store; s++) sm.ref[s] = m[s];
  }
  __syncthreads();
  UWVK_STAMP(9);
  d4_t acc[Geo<DOF>::TPW];
  {
    double d[DOF];
    boxminus_lds<DOF>(x, sm.ref, d, right);
    cov_gemm<DOF>(sm, d, acc);
  }
  store_cov<DOF>(sm, acc, [](int, int) { return 0.0; });
  if (t < L::store) sm.mu[t] = sm.ref[t];
  __syncthreads();
  UWVK_STAMP(10);
  return ok;
}

// ---------------------------------------------------------------------------
// apply_delta, exact nav-frame form.  With X_p = mu [+] +-L_j and the left
// SO3 boxplus, (X_p [+] d) [-] (mu [+] d) = T (+-L_j) exactly, T = blockdiag(I,
// R(exp(d_ori)), I): the re-spread covariance of ukfom's apply_delta equals
// T (L L^T) T^T = T Sigma T^T.  So: mu <- mu [+] d, Sigma <- T Sigma T^T
// (O(n) work instead of a Cholesky + sigma spread + GEMM).  Differences to the
// literal form are rounding only; apply_delta_literal keeps the literal path.
// With the right (body-frame) boxplus, X_p = mu exp(l): (X_p [+] d) [-] (mu [+] d)
// = log(exp(-d) exp(l) exp(d)) = R(exp(d))^T l, so T carries R^T instead.
// ---------------------------------------------------------------------------
template <int DOF>
UWVK_DEV bool apply_delta_rot(Smem<DOF>& sm, int right, Stamper* st = nullptr) {
  using L = Lay<DOF>;
  const int t = tid();
  double R[9];
  {
    const double dv[3] = {sm.vec[3], sm.vec[4], sm.vec[5]};
    double e[4];
    so3_exp(dv, e);
    if (right) e[1] = -e[1], e[2] = -e[2], e[3] = -e[3];  // R(exp(d))^T = R(exp(d)^-1)
    qmatrix(e, R);
  }
  // Sigma T^T: columns 3..5 of every row
  if (t < DOF) {
    const double s0 = sm.S[t * DOF + 3], s1 = sm.S[t * DOF + 4], s2 = sm.S[t * DOF + 5];
#pragma unroll
    for (int i = 0; i < 3; i++) sm.S[t * DOF + 3 + i] = R[i * 3] * s0 + R[i * 3 + 1] * s1 + R[i * 3 + 2] * s2;
  }
  __syncthreads();
  // T (Sigma T^T): rows 3..5 of every column
  if (t < DOF) {
    const double s0 = sm.S[3 * DOF + t], s1 = sm.S[4 * DOF + t], s2 = sm.S[5 * DOF + t];
#pragma unroll
    for (int i = 0; i < 3; i++) sm.S[(3 + i) * DOF + t] = R[i * 3] * s0 + R[i * 3 + 1] * s1 + R[i * 3 + 2] * s2;
  }
  if (t == 0) {
    double m[L::store];
#pragma unroll
    for (int s = 0; s < L::store; s++) m[s] = sm.mu[s];
    boxplus_vec<DOF>(m, sm.vec, right);
#pragma unroll
    for (int s = 0; s < L::store; s++) sm.mu[s] = m[s];
  }
  __syncthreads();
  UWVK_STAMP(10);
  return true;
}

template <int DOF>
UWVK_DEV bool apply_delta(Smem<DOF>& sm, bool literal, int right, Stamper* st = nullptr) {
  if (literal) return apply_delta_literal<DOF>(sm, right, st);
  return apply_delta_rot<DOF>(sm, right, st);
}

// ---------------------------------------------------------------------------
// ukf::update [EXT] with measurement functor h (per sigma point, registers).
//   zmode 0: Eigen-vector measurement (plain average)
//   zmode 1: vect-manifold measurement (iterative mean, |d| <= 1e-6)
//   gate 0: accept_any_mahalanobis_distance; 1: d2p95 (PoseUKF.cpp:275-286)
// Returns the gate decision; *ok = false on a Cholesky failure.
// ---------------------------------------------------------------------------
// one past the highest tangent DOF measurement model H reads (Dz_j = 0 beyond)
template <class H, int DOF>
struct HJmax {
  static constexpr int value = DOF;
};

// LAD: -1 the apply_delta form from `literal` at run time; 0 / 1 fixed at compile
// time (the exact rotation identity / the literal re-spread), so a kernel built
// for one form carries only its registers
template <int DOF, int M, class H, int LAD = -1>
UWVK_DEV bool pose_update(Smem<DOF>& sm, const double (&z)[M], const double (&R)[M * M], int zmode, int gate, H h,
                          bool* ok, Stamper* st, bool literal, int right) {
  using L = Lay<DOF>;
  using G = Geo<DOF>;
  const int t = tid();
  const bool mine = t < G::N;
  const bool cok = chol_lds<DOF>(sm);
  UWVK_STAMP(4);
  double x[L::store];
  gen_point<DOF>(sm, t, x, right);
  __syncthreads();  // L dead from here on
  double zp[M], zm[M];
  h(x, zp);
  if (zmode == 0) {
#pragma unroll
    for (int a = 0; a < M; a++) zm[a] = mine ? zp[a] : 0.0;
    block_sum<DOF, M>(sm, zm);
#pragma unroll
    for (int a = 0; a < M; a++) zm[a] = zm[a] / (double)G::N;
  } else {
    if (t == 0) {
#pragma unroll
      for (int a = 0; a < M; a++) sm.vec[a] = zp[a];
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < M; a++) zm[a] = sm.vec[a];
    __syncthreads();
    int it = 0;
    double nrm;
    do {
      double d[M];
#pragma unroll
      for (int a = 0; a < M; a++) d[a] = mine ? (zp[a] - zm[a]) : 0.0;
      block_sum<DOF, M>(sm, d);
      nrm = 0.0;
#pragma unroll
      for (int a = 0; a < M; a++) {
        d[a] = d[a] / (double)G::N;
        nrm += d[a] * d[a];
      }
#pragma unroll
      for (int a = 0; a < M; a++) zm[a] = zm[a] + d[a];
      nrm = sqrt(nrm);
    } while (nrm > 1e-6 && ++it < 10000);
  }
  double dz[M];
#pragma unroll
  for (int a = 0; a < M; a++) dz[a] = mine ? (zp[a] - zm[a]) : 0.0;
  double S[M * M];
  {
    constexpr int NS = M * (M + 1) / 2;
    double sp[NS];
    int k = 0;
#pragma unroll
    for (int a = 0; a < M; a++)
#pragma unroll
      for (int b = a; b < M; b++) sp[k++] = dz[a] * dz[b];
    block_sum<DOF, NS>(sm, sp);
    k = 0;
#pragma unroll
    for (int a = 0; a < M; a++)
#pragma unroll
      for (int b = a; b < M; b++) {
        const double s = 0.5 * sp[k++];
        S[a * M + b] = s + R[a * M + b];
        S[b * M + a] = s + R[b * M + a];
      }
  }
  UWVK_STAMP(5);
  double Si[M * M];
  small_inv<M>(S, Si);
  double nu[M];
#pragma unroll
  for (int a = 0; a < M; a++) nu[a] = z[a] - zm[a];
  double d2 = 0.0;
#pragma unroll
  for (int b = 0; b < M; b++) {
    double u = 0.0;
#pragma unroll
    for (int a = 0; a < M; a++) u += nu[a] * Si[a * M + b];
    d2 += u * nu[b];
  }
  const bool accept = gate == 0 ? true : !(d2 > kD2P95);
  if (!accept) {
    *ok = cok;
    return false;
  }
  // cross covariance C = 1/2 sum_p dx_p dz_p^T.  The points are mu [+] +-L_j,
  // so dx_{2j+1} = L_j = -dx_{2j+2} (to rounding: [+] then [-] returns the
  // step) and each pair sums to L_j (z_{2j+1} - z_{2j+2}), the mean
  // cancelling: C = 1/2 L Dz^T with Dz_j = z_{2j+1} - z_{2j+2}, lower-
  // triangular L (row r sums j <= r).  Dz_j is exactly 0 for j >= JM when h
  // reads no tangent DOF >= JM (the two points' inputs are then bitwise mu's).
  // Dz is staged in sm.scratch(); the waves split the M components; C and the
  // gain K then go through the (dead) factor region for the Sigma update.
  constexpr int JM = HJmax<H, DOF>::value;
  static_assert(JM * M <= Smem<DOF>::kScratch, "Dz staging (Smem::scratch)");
  double* dzs = sm.scratch();
  {
    const int j = (t - 1) >> 1;
    if (t >= 1 && (t & 1) && j < JM) {
#pragma unroll
      for (int a = 0; a < M; a++) dzs[j * M + a] = zp[a];
    }
    __syncthreads();
    if (t >= 2 && !(t & 1) && j < JM) {
#pragma unroll
      for (int a = 0; a < M; a++) dzs[j * M + a] = dzs[j * M + a] - zp[a];
    }
    __syncthreads();
  }
  // components per wave: two waves split them (wave 0 the first NA), one wave takes all
  constexpr int NA = G::NW > 1 ? (M + 1) / 2 : M;
  const int w = G::NW > 1 ? (t >> 6) : 0, r = G::NW > 1 ? (t & 63) : t;
  const int a0 = w * NA, na = (M - a0) < NA ? (M - a0) : NA;
  double* cst = sm.Lp;  // C rows [DOF][M], then K rows [DOF][M] (the factor is dead by then)
  double* kst = sm.Lp + DOF * M;
  {
    double Cw[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) Cw[a] = 0.0;
    if (r < DOF && na > 0) {
      const int jn = r + 1 < JM ? r + 1 : JM;
      const double* lr = sm.Lp + r * (r + 1) / 2;
      for (int j = 0; j < jn; j++) {
        const double l = lr[j];
#pragma unroll
        for (int a = 0; a < NA; a++)
          if (a < na) Cw[a] += l * dzs[j * M + a0 + a];
      }
    }
    __syncthreads();  // every L row read: the factor region takes C
    if (r < DOF && na > 0) {
#pragma unroll
      for (int a = 0; a < NA; a++)
        if (a < na) cst[r * M + a0 + a] = 0.5 * Cw[a];
    }
  }
  __syncthreads();
  // K = C S^-1 and delta = K nu (rows r < DOF of wave 0)
  if (t < DOF) {
    double Cr[M];
#pragma unroll
    for (int a = 0; a < M; a++) Cr[a] = cst[t * M + a];
    double dl = 0.0;
#pragma unroll
    for (int a = 0; a < M; a++) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < M; b++) s += Cr[b] * Si[b * M + a];
      kst[t * M + a] = s;
      dl += s * nu[a];
    }
    sm.vec[t] = dl;
  }
  __syncthreads();
  // Sigma -= C K^T: the waves split the columns
  {
    constexpr int CW = (DOF + G::NW - 1) / G::NW;
    const int c0 = w * CW, c1 = c0 + CW < DOF ? c0 + CW : DOF;
    if (r < DOF) {
      double Cr[M];
#pragma unroll
      for (int a = 0; a < M; a++) Cr[a] = cst[r * M + a];
      for (int c = c0; c < c1; c++) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < M; a++) s += Cr[a] * kst[c * M + a];
        sm.S[r * DOF + c] -= s;
      }
    }
  }
  __syncthreads();
  UWVK_STAMP(7);
  const bool aok = apply_delta<DOF>(sm, LAD < 0 ? literal : LAD != 0, right, st);
  *ok = cok && aok;
  return true;
}

// ---------------------------------------------------------------------------
// measurement models (PoseUKF.cpp:87-219)
// ---------------------------------------------------------------------------
template <int DOF>
struct HAcc {  // measurementAcceleration, PoseUKF.cpp:125-131
  UWVK_DEV void operator()(const double* x, double (&z)[3]) const {
    using L = Lay<DOF>;
    const double a[3] = {x[L::s_acc], x[L::s_acc + 1], x[L::s_acc + 2] + x[L::s_grav]};
    double r[3];
    qrot_inv(x + L::s_quat, a, r);
#pragma unroll
    for (int i = 0; i < 3; i++) z[i] = r[i] + x[L::s_ba + i];
  }
};
template <int DOF>
struct HVel {  // measurementVelocity, PoseUKF.cpp:117-123
  UWVK_DEV void operator()(const double* x, double (&z)[3]) const {
    using L = Lay<DOF>;
    qrot_inv(x + L::s_quat, x + L::s_vel, z);
  }
};
template <int DOF>
struct HPressure {  // measurementPressureSensor, PoseUKF.cpp:107-115
  double s[3], patm;
  UWVK_DEV void operator()(const double* x, double (&z)[1]) const {
    using L = Lay<DOF>;
    double r[3];
    qrot(x + L::s_quat, s, r);
    const double pz = x[L::s_pos + 2] + r[2];
    z[0] = patm - pz * x[L::s_grav] * x[L::s_rho];
  }
};
template <int DOF>
struct HWater {  // measurementWaterCurrents, PoseUKF.cpp:133-151
  double cw;
  UWVK_DEV void operator()(const double* x, double (&z)[2]) const {
    using L = Lay<DOF>;
    const double vb[3] = {x[L::s_vel] - x[L::s_wvb], x[L::s_vel + 1] - x[L::s_wvb + 1], x[L::s_vel + 2] - 0.0};
    const double vw[3] = {x[L::s_vel] - x[L::s_wv], x[L::s_vel + 1] - x[L::s_wv + 1], x[L::s_vel + 2] - 0.0};
    double rb[3], rw[3];
    qrot_inv(x + L::s_quat, vb, rb);
    qrot_inv(x + L::s_quat, vw, rw);
#pragma unroll
    for (int i = 0; i < 2; i++) z[i] = cw * rb[i] + (1 - cw) * rw[i] + x[L::s_badcp + i];
  }
};
template <int DOF>
struct HXY {  // measurementXYPosition, PoseUKF.cpp:87-92
  UWVK_DEV void operator()(const double* x, double (&z)[2]) const { z[0] = x[0]; z[1] = x[1]; }
};
template <int DOF>
struct HZ {  // measurementZPosition, PoseUKF.cpp:100-105
  UWVK_DEV void operator()(const double* x, double (&z)[1]) const { z[0] = x[2]; }
};

// [EXT] DynamicModel::calcEfforts: tau = M a + C(nu) nu + D_l nu + D_q |nu| nu + g(q)
// M/Dl/Dq: base 6x6 (row-major, global) with the (0,1,5) blocks overridden by blk
struct Efforts6 {
  const double* base;  // M[36], Dl[36], Dq[36]
  double weight, buoyancy, cog[3], cob[3];
  UWVK_DEV static constexpr int blk_index(int r, int c) {  // -> a + 3b of the 3x3 block or -1
    const int a = r == 0 ? 0 : r == 1 ? 1 : r == 5 ? 2 : -1;
    const int b = c == 0 ? 0 : c == 1 ? 1 : c == 5 ? 2 : -1;
    return (a < 0 || b < 0) ? -1 : a + 3 * b;
  }
  template <class BLK>
  UWVK_DEV double m(int which, int r, int c, const BLK& blk) const {
    const int k = blk_index(r, c);
    if (k >= 0 && blk.has) return blk.v[which * 9 + k];
    // the batch-shared base matrices by scalar loads: base is global memory no
    // kernel writes, read through the constant address space (s_load into
    // SGPRs, used as FMA operands); as vector loads they were ~80 doubles of
    // VGPRs held across a model evaluation
    using CD = const __attribute__((address_space(4))) double;
    return ((CD*)base)[which * 36 + r * 6 + c];
  }
  template <class BLK>
  UWVK_DEV void eval(const double acc6[6], const double nu[6], const double q[4], const BLK& blk, double tau[6]) const {
    double a[3], b[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      double sa = 0, sb = 0;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        sa += m(0, i, j, blk) * nu[j];
        sb += m(0, 3 + i, j, blk) * nu[j];
      }
      a[i] = sa; b[i] = sb;
    }
    double t0[3], t1[3], t2[3], cor[6];
    cross3(nu + 3, a, t0);
    cross3(nu, a, t1);
    cross3(nu + 3, b, t2);
#pragma unroll
    for (int i = 0; i < 3; i++) { cor[i] = t0[i]; cor[3 + i] = t1[i] + t2[i]; }
    const double fw[3] = {0, 0, -weight}, fb[3] = {0, 0, buoyancy};
    double fg[3], fbb[3], mg[3], mb[3], g[6];
    qrot_inv(q, fw, fg);
    qrot_inv(q, fb, fbb);
    cross3(cog, fg, mg);
    cross3(cob, fbb, mb);
#pragma unroll
    for (int i = 0; i < 3; i++) { g[i] = -(fg[i] + fbb[i]); g[3 + i] = -(mg[i] + mb[i]); }
#pragma unroll
    for (int i = 0; i < 6; i++) {
      double sl = 0, sq = 0, mm = 0;
#pragma unroll
      for (int j = 0; j < 6; j++) {
        sl += m(1, i, j, blk) * nu[j];
        sq += m(2, i, j, blk) * (fabs(nu[j]) * nu[j]);
        mm += m(0, i, j, blk) * acc6[j];
      }
      tau[i] = mm + cor[i] + (sl + sq) + g[i];
    }
  }
};

struct BlkPtr { bool has; const double* v; };

template <int DOF>
struct HEfforts {  // measurementEfforts, PoseUKF.cpp:153-196
  Efforts6 ef;
  double wb[3], imu[3];
  UWVK_DEV void operator()(const double* x, double (&z)[6]) const {
    using L = Lay<DOF>;
    struct BlkState { bool has; double v[27]; } blk;
    blk.has = L::has_params != 0;
    if constexpr (L::has_params) {
#pragma unroll
      for (int k = 0; k < 9; k++) {
        blk.v[k] = x[L::s_inertia + k];
        blk.v[9 + k] = x[L::s_lin + k];
        blk.v[18 + k] = x[L::s_quad + k];
      }
    }
    const double wv[3] = {x[L::s_wv], x[L::s_wv + 1], 0.0};
    double vb[3], cr[3], rw[3], vel6[6], acc6[6], ab[3], cc[3];
    qrot_inv(x + L::s_quat, x + L::s_vel, vb);
    cross3(wb, imu, cr);
#pragma unroll
    for (int i = 0; i < 3; i++) vb[i] = vb[i] - cr[i];
    qrot_inv(x + L::s_quat, wv, rw);
#pragma unroll
    for (int i = 0; i < 3; i++) { vel6[i] = vb[i] - rw[i]; vel6[3 + i] = wb[i]; }
    qrot_inv(x + L::s_quat, x + L::s_acc, ab);
    cross3(wb, cr, cc);
#pragma unroll
    for (int i = 0; i < 3; i++) { acc6[i] = ab[i] - cc[i]; acc6[3 + i] = 0.0; }
    ef.eval(acc6, vel6, x + L::s_quat, blk, z);
  }
};

template <int DOF>
struct HConstrain {  // constrainVelocity, PoseUKF.cpp:199-219
  Efforts6 ef;
  BlkPtr blk;  // the shared model's current (surge,sway,yaw) blocks
  double wb[3], imu[3], w3[3], q[4], ab[3];
  UWVK_DEV void operator()(const double* x, double (&z)[6]) const {
    using L = Lay<DOF>;
    double vb[3], cr[3], rw[3], vel6[6], acc6[6];
    qrot_inv(q, x + L::s_vel, vb);
    cross3(wb, imu, cr);
#pragma unroll
    for (int i = 0; i < 3; i++) vb[i] = vb[i] - cr[i];
    qrot_inv(q, w3, rw);
#pragma unroll
    for (int i = 0; i < 3; i++) { vel6[i] = vb[i] - rw[i]; vel6[3 + i] = wb[i]; acc6[i] = ab[i]; acc6[3 + i] = 0.0; }
    ef.eval(acc6, vel6, q, blk, z);
  }
};

// measurementEfforts reads orientation, velocity, acceleration, the model blocks
// and the water velocity; constrainVelocity only the velocity
template <int DOF>
struct HJmax<HEfforts<DOF>, DOF> {
  static constexpr int value = Lay<DOF>::d_wv + 2;
};
template <int DOF>
struct HJmax<HConstrain<DOF>, DOF> {
  static constexpr int value = Lay<DOF>::d_vel + 3;
};

// getRotationRate (PoseUKF.cpp:693-699) at the current mean
template <int DOF>
UWVK_DEV void rotation_rate_body_mu(const double* mu, const PoseShared& sh, const double w[3], double out[3]) {
  using L = Lay<DOF>;
  const double lat = sh.lat0 + mu[L::s_pos] * sh.inv_rm;
  double sl, cl;
  sincos(lat, &sl, &cl);
  const double er[3] = {kEarthW * cl, 0.0, kEarthW * sl};
  const double q[4] = {mu[L::s_quat], mu[L::s_quat + 1], mu[L::s_quat + 2], mu[L::s_quat + 3]};
  double r[3];
  qrot_inv(q, er, r);
#pragma unroll
  for (int i = 0; i < 3; i++) out[i] = (w[i] - mu[L::s_bg + i]) - r[i];
}
template <int DOF>
UWVK_DEV void rotation_rate_body(const Smem<DOF>& sm, const PoseShared& sh, const double w[3], double out[3]) {
  using L = Lay<DOF>;
  const double lat = sh.lat0 + sm.mu[L::s_pos] * sh.inv_rm;
  double sl, cl;
  sincos(lat, &sl, &cl);
  const double er[3] = {kEarthW * cl, 0.0, kEarthW * sl};
  const double q[4] = {sm.mu[L::s_quat], sm.mu[L::s_quat + 1], sm.mu[L::s_quat + 2], sm.mu[L::s_quat + 3]};
  double r[3];
  qrot_inv(q, er, r);
#pragma unroll
  for (int i = 0; i < 3; i++) out[i] = (w[i] - sm.mu[L::s_bg + i]) - r[i];
}

}  // namespace uwvk
