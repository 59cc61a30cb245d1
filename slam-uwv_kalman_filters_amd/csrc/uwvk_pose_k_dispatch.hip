// Dispatch of PoseUKF update kinds to their translation units.
#include "uwvk_pose_kernels.hpp"

namespace uwvk {

hipError_t launch_pose_update_a(int, int, hipStream_t, const PoseBufs&, const PoseShared&, const MeasArgs&, int);
hipError_t launch_pose_update_b(int, int, hipStream_t, const PoseBufs&, const PoseShared&, const MeasArgs&, int);
hipError_t launch_pose_update_c(int, int, hipStream_t, const PoseBufs&, const PoseShared&, const MeasArgs&, int);

hipError_t launch_pose_update(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                              const MeasArgs& ma, int m) {
  switch (kind) {
    case MK_ACC: case MK_VEL: case MK_PRESSURE: return launch_pose_update_a(dof, kind, st, b, sh, ma, m);
    case MK_WATER: case MK_EFFORTS: return launch_pose_update_b(dof, kind, st, b, sh, ma, m);
    default: return launch_pose_update_c(dof, kind, st, b, sh, ma, m);
  }
}

}  // namespace uwvk
