// BodyEfforts update of one epoch for run_log's PSP split (k_pose_efforts_epoch).
// Its own translation unit: sharing one with k_pose_epoch changes that kernel's
// register allocation (more scratch spills).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_efforts_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                     const EpochArgs& ea) {
  if (dof == 53)
    hipLaunchKernelGGL(k_pose_efforts_epoch<53>, dim3((unsigned)b.batch), dim3(Geo<53>::T), 0, st, b, sh, ea);
  else
    hipLaunchKernelGGL(k_pose_efforts_epoch<26>, dim3((unsigned)b.batch), dim3(Geo<26>::T), 0, st, b, sh, ea);
  return hipGetLastError();
}

}  // namespace uwvk
