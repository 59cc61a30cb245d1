// uwvk_psp.hpp — host launchers of the PSP PoseUKF kernels (uwvk_psp_k.hip).
#pragma once
#include "uwvk_pose_kernels.hpp"

namespace uwvk {
hipError_t launch_psp_predict(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt);
hipError_t launch_psp_update(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                             const MeasArgs& ma, int m);
hipError_t launch_psp_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea);
}  // namespace uwvk
