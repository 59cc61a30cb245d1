// PoseUKF single-measurement update kernels, group c (MK_XY MK_Z MK_GEO MK_DELAYED).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_update_c(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const MeasArgs& ma, int m) {
  const dim3 g((unsigned)b.batch);
  switch (kind) {
    case MK_XY:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_XY>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_XY>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_Z:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_Z>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_Z>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_GEO:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_GEO>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_GEO>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_DELAYED:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_DELAYED>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_DELAYED>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace uwvk
