// PoseUKF single-measurement update kernels, group a (MK_ACC MK_VEL MK_PRESSURE).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_update_a(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const MeasArgs& ma, int m) {
  const dim3 g((unsigned)b.batch);
  switch (kind) {
    case MK_ACC:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_ACC>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_ACC>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_VEL:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_VEL>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_VEL>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
    case MK_PRESSURE:
      if (dof == 53) hipLaunchKernelGGL((k_pose_update<53, MK_PRESSURE>), g, dim3(Geo<53>::T), 0, st, b, sh, ma, m);
      else hipLaunchKernelGGL((k_pose_update<26, MK_PRESSURE>), g, dim3(Geo<26>::T), 0, st, b, sh, ma, m);
      return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace uwvk
