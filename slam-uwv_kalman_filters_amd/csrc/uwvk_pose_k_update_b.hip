// PoseUKF single-measurement update kernels, group b (MK_WATER MK_EFFORTS).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_update_b(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const MeasArgs& ma, int m) {
  const dim3 g((unsigned)b.batch);
  switch (kind) {
    case MK_WATER:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_WATER>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_WATER>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_EFFORTS:  // one instantiation per model (efforts / velocity-only) with the exact apply_delta
      if (dof == 53) {
        if (sh.literal_apply_delta) hipLaunchKernelGGL((k_pose_update<53, MK_EFFORTS>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
        else if (ma.only_vel) hipLaunchKernelGGL((k_pose_update<53, MK_EFFORTS, 1, 0>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
        else hipLaunchKernelGGL((k_pose_update<53, MK_EFFORTS, 0, 0>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      } else {
        if (sh.literal_apply_delta) hipLaunchKernelGGL((k_pose_update<26, MK_EFFORTS>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
        else if (ma.only_vel) hipLaunchKernelGGL((k_pose_update<26, MK_EFFORTS, 1, 0>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
        else hipLaunchKernelGGL((k_pose_update<26, MK_EFFORTS, 0, 0>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      }
      return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace uwvk
