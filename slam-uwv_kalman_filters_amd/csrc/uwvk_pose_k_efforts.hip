// BodyEfforts update of one epoch for run_log's PSP split (k_pose_efforts_epoch).
// Its own translation unit: sharing one with k_pose_epoch changes that kernel's
// register allocation (more scratch spills).
#define UWVK_POSE_KERNEL_BODIES
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_efforts_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                     const EpochArgs& ea, int vo) {
  const dim3 g((unsigned)b.batch);
  if (dof == 53) {
    if (sh.literal_apply_delta) hipLaunchKernelGGL((k_pose_efforts_epoch<53, -1, -1>), g, dim3(Geo<53>::T), 0, st, b, sh, ea);
    else if (vo) hipLaunchKernelGGL((k_pose_efforts_epoch<53, 1, 0>), g, dim3(Geo<53>::T), 0, st, b, sh, ea);
    else hipLaunchKernelGGL((k_pose_efforts_epoch<53, 0, 0>), g, dim3(Geo<53>::T), 0, st, b, sh, ea);
  } else {
    if (sh.literal_apply_delta) hipLaunchKernelGGL((k_pose_efforts_epoch<26, -1, -1>), g, dim3(Geo<26>::T), 0, st, b, sh, ea);
    else if (vo) hipLaunchKernelGGL((k_pose_efforts_epoch<26, 1, 0>), g, dim3(Geo<26>::T), 0, st, b, sh, ea);
    else hipLaunchKernelGGL((k_pose_efforts_epoch<26, 0, 0>), g, dim3(Geo<26>::T), 0, st, b, sh, ea);
  }
  return hipGetLastError();
}

}  // namespace uwvk

#ifdef UWVK_STAMPS
// diagnostic build only: per-phase cycle sums of k_pose_efforts_epoch
extern "C" int uwvk_debug_read_stamps_eff(unsigned long long* sum, unsigned long long* cnt, int reset) {
  if (hipMemcpyFromSymbol(sum, HIP_SYMBOL(uwvk::uwvk_stamp_sum), 64 * 8) != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(cnt, HIP_SYMBOL(uwvk::uwvk_stamp_cnt), 64 * 8) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[64] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(uwvk::uwvk_stamp_sum), z, 64 * 8) != hipSuccess) return 1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(uwvk::uwvk_stamp_cnt), z, 64 * 8) != hipSuccess) return 1;
  }
  return 0;
}
#endif
