// uwvk_psp.hpp — host launchers of the PSP PoseUKF kernels (uwvk_psp_k.hip).
#pragma once
#include "uwvk_pose_kernels.hpp"

namespace uwvk {
// Per-side launchers (SR = 0 nav-frame / left, 1 body-frame / right SO3 [+]),
// each instantiated in one object: uwvk_psp_k.hip (0) and uwvk_psp_k_r.hip (1).
template <int SR>
hipError_t launch_psp_predict_sr(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt);
template <int SR>
hipError_t launch_psp_update_sr(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                const MeasArgs& ma, int m);
template <int SR>
hipError_t launch_psp_epoch_sr(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                               int64_t grid, uint32_t ev_any, uint32_t lds_pad, int pd);
template <int SR>
hipError_t launch_psp_efforts_sr(int dof, int vo, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                                 const EpochArgs& ea);
extern template hipError_t launch_psp_efforts_sr<0>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                    const EpochArgs&);
extern template hipError_t launch_psp_efforts_sr<1>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                    const EpochArgs&);
extern template hipError_t launch_psp_predict_sr<0>(int, hipStream_t, const PoseBufs&, const PoseShared&, double);
extern template hipError_t launch_psp_predict_sr<1>(int, hipStream_t, const PoseBufs&, const PoseShared&, double);
extern template hipError_t launch_psp_update_sr<0>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                   const MeasArgs&, int);
extern template hipError_t launch_psp_update_sr<1>(int, int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                   const MeasArgs&, int);
extern template hipError_t launch_psp_epoch_sr<0>(int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                  const EpochArgs&, int64_t, uint32_t, uint32_t, int);
extern template hipError_t launch_psp_epoch_sr<1>(int, hipStream_t, const PoseBufs&, const PoseShared&,
                                                  const EpochArgs&, int64_t, uint32_t, uint32_t, int);
// the handle's side (sh.so3_right) picks the launcher
hipError_t launch_psp_predict(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, double dt);
hipError_t launch_psp_update(int dof, int kind, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                             const MeasArgs& ma, int m);
// run_log's BodyEfforts epoch ea.first: vo 1 the velocity-only form
// (constrainVelocity, PEffVO), 0 the full measurementEfforts (psp_update_eff)
hipError_t launch_psp_efforts(int dof, int vo, hipStream_t st, const PoseBufs& b, const PoseShared& sh,
                              const EpochArgs& ea);
#include <vector>
// grid 0: one block per instance; otherwise 8 (n_x + (chunks - 1) r_x)
// ev_any: the OR of the launch's epoch flags (selects the kernel instantiation;
// all bits set is always correct)
// lds_pad: UWVK_OPT_LDS_PAD's dynamic LDS bytes per workgroup (diagnostic)
// pd: dof 53 on the parameter-decoupled kernel (psp::PspSmemPD; b.Qp the host's
// PD table, sh.q_simple required)
hipError_t launch_psp_epoch(int dof, hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                            int64_t grid = 0, uint32_t ev_any = 0xffffffffu, uint32_t lds_pad = 0, int pd = 0);
// static LDS of one k_psp_epoch workgroup (sizeof PspSmem<dof>)
size_t psp_epoch_lds_bytes(int dof);
// resident k_psp_epoch blocks per XCD (occupancy x CUs / 8), 0 if unknown
int64_t psp_epoch_slots_per_xcd(int dof, int device, int pd = 0);
// resident blocks of the static (k_psp_epoch) or persistent (k_psp_epoch_p)
// epoch kernel on the device (occupancy x CUs), 0 if unknown; pd: the
// parameter-decoupled kernel's
int64_t psp_epoch_slots(int dof, int device, bool persist, int pd = 0);
// chunks per tail instance for one XCD's n instances over s resident blocks in
// a count-epoch launch (1: no tail spreading)
int plan_tail(int64_t n, int64_t s, int64_t count);
// the two-instances-per-wave parameter-decoupled kernel (uwvk_psp_pair.hip):
// persistent only (ea.ticket), pair units (EpochArgs units / tail0 / r_x count
// pairs of instances 2u, 2u + 1), the PD table in b.Qp, sh.q_simple
hipError_t launch_psp_epoch_pair(hipStream_t st, const PoseBufs& b, const PoseShared& sh, const EpochArgs& ea,
                                 int64_t grid, uint32_t ev_any, int pd);
// its resident blocks on the device (occupancy x CUs), 0 if unknown
int64_t psp_pair_slots(int device);
// 1 once a probe grid has shown round-robin block placement over 8 XCCs on
// device (what tail spreading relies on), else 0; cached per device
int xcd_round_robin(int device);
}  // namespace uwvk
