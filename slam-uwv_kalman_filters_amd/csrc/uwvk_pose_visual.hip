// uwvk_pose_visual.hip — PoseUKF::integrateMeasurement(vector<VisualFeatureMeasurement>,
// feature_positions, marker_pose, cov_marker_pose, camera_config, camera_in_IMU)
// (PoseUKF.cpp:613-654) on gfx950.
//
// The reference augments the filter with the marker pose (PoseStateWithMarker,
// PoseUKF.cpp:221-229: n = 53 + 6 = 59 DOF, 119 sigma points), runs one
// S2-valued ukf::update per feature and keeps the leading n x n block.  Here:
// one 128-lane workgroup per instance, one sigma point per lane, the 59 x 59
// augmented Sigma and the deviation matrix in LDS (uwvk_aug_dev.hpp).  This is
// a camera-rate event, not the per-IMU-epoch hot path.
#include "uwvk_aug_dev.hpp"
#include "uwvk_pose_dev.hpp"

namespace uwvk {

namespace {

// SR: the handle's SO3 side (UWVK_OPT_SO3_RIGHT); both SO3 segments follow it
// (MTK has one SO3::boxplus, so the marker orientation takes the filter's side)
template <int DOF, int SR>
using PoseMarkerM = aug::Manifold<aug::Seg<aug::SEG_V, 3>, aug::Seg<SR ? aug::SEG_SO3R : aug::SEG_SO3>,
                                  aug::Seg<aug::SEG_V, DOF - 6>, aug::Seg<aug::SEG_V, 3>,
                                  aug::Seg<SR ? aug::SEG_SO3R : aug::SEG_SO3>>;

template <int DOF, int SR>
__global__ __launch_bounds__((aug::Engine<PoseMarkerM<DOF, SR>>::BLOCK)) void k_pose_visual(PoseBufs b, aug::VisArgs va) {
  using E = aug::Engine<PoseMarkerM<DOF, SR>>;
  static_assert(E::IPB == 1, "one instance per workgroup");
  constexpr int n = DOF, na = E::n, S = Lay<DOF>::store;
  __shared__ double smem[E::words];
  const int64_t inst = blockIdx.x;
  E e;
  e.g = threadIdx.x;
  e.sm = smem;
  e.live = inst < b.batch && (!va.mask || va.mask[inst]);
  if (e.live) {
    // augmented_state_cov: blockdiag(Sigma, cov_marker_pose) (PoseUKF.cpp:624-627)
    for (int i = e.g; i < na * na; i += E::G) {
      const int r = i / na, c = i % na;
      double v = 0.0;
      if (r < n && c < n) v = b.sigma[inst * tri_n<n>() + pidx(r, c)];
      else if (r >= n && c >= n) v = va.cov_marker[(r - n) * 6 + (c - n)];
      e.sm[E::o_sig + i] = v;
    }
    for (int k = e.g; k < E::S; k += E::G)
      e.sm[E::o_mu + k] = k < S ? b.mu[inst * S + k] : va.marker[inst * va.marker_stride + (k - S)];
  }
  __syncthreads();
  const bool ok = aug::visual_loop<E, S, false>(e, va, inst);
  // ukf.reset(new MTK_UKF(mu.filter_state, sigma.block(0, 0, n, n))) (PoseUKF.cpp:652)
  if (e.live && ok) {
    for (int i = e.g; i < tri_n<n>(); i += E::G) {
      int r, c;
      unpack(i, r, c);
      b.sigma[inst * tri_n<n>() + i] = e.sm[E::o_sig + r * na + c];
    }
    for (int k = e.g; k < S; k += E::G) b.mu[inst * S + k] = e.sm[E::o_mu + k];
  }
  if (e.live && !ok && e.g == 0) b.status[inst] |= UWVK_ST_NOTPD;
}

}  // namespace

template <int SR>
static void launch_pose_visual_sr(int dof, hipStream_t st, const PoseBufs& b, const aug::VisArgs& va) {
  const dim3 g((unsigned)b.batch);
  if (dof == 53)
    hipLaunchKernelGGL((k_pose_visual<53, SR>), g, dim3(aug::Engine<PoseMarkerM<53, SR>>::BLOCK), 0, st, b, va);
  else
    hipLaunchKernelGGL((k_pose_visual<26, SR>), g, dim3(aug::Engine<PoseMarkerM<26, SR>>::BLOCK), 0, st, b, va);
}

hipError_t launch_pose_visual(int dof, int right, hipStream_t st, const PoseBufs& b, const aug::VisArgs& va) {
  if (right) launch_pose_visual_sr<1>(dof, st, b, va);
  else launch_pose_visual_sr<0>(dof, st, b, va);
  return hipGetLastError();
}

}  // namespace uwvk
