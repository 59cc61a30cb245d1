// PoseUKF predict / rotation-rate / ensemble-statistics kernels (gfx950).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_predict(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt) {
  if (dof == 53)
    hipLaunchKernelGGL(k_pose_predict<53>, dim3((unsigned)b.batch), dim3(Geo<53>::T), 0, st, b, sh, dt);
  else
    hipLaunchKernelGGL(k_pose_predict<26>, dim3((unsigned)b.batch), dim3(Geo<26>::T), 0, st, b, sh, dt);
  return hipGetLastError();
}

hipError_t launch_pose_rotation_rate(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double* out) {
  if (dof == 53)
    hipLaunchKernelGGL(k_pose_rotation_rate<53>, dim3((unsigned)b.batch), dim3(64), 0, st, b, sh, out);
  else
    hipLaunchKernelGGL(k_pose_rotation_rate<26>, dim3((unsigned)b.batch), dim3(64), 0, st, b, sh, out);
  return hipGetLastError();
}

hipError_t launch_pose_stats(int dof, hipStream_t st, const PoseBufs& b, const StatTruth& truth, double* out,
                             double* part) {
  const int64_t nb = (b.batch + 63) / 64;
  const int nout = 3 * (dof == 53 ? Lay<53>::store : Lay<26>::store) + 2;
  if (dof == 53) {
    hipLaunchKernelGGL(k_pose_stats<53>, dim3((unsigned)nb), dim3(64), 0, st, b, truth, part);
    hipLaunchKernelGGL(k_pose_stats_sum<53>, dim3(nout), dim3(256), 0, st, (const double*)part, nb, nout, out);
  } else {
    hipLaunchKernelGGL(k_pose_stats<26>, dim3((unsigned)nb), dim3(64), 0, st, b, truth, part);
    hipLaunchKernelGGL(k_pose_stats_sum<26>, dim3(nout), dim3(256), 0, st, (const double*)part, nb, nout, out);
  }
  return hipGetLastError();
}

}  // namespace uwvk
