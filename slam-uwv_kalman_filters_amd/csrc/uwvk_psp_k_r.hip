// uwvk_psp_k_r.hip — the PSP PoseUKF kernels for the body-frame (right) SO3
// boxplus, UWVK_OPT_SO3_RIGHT: the same kernel templates as uwvk_psp_k.hip,
// instantiated with SR = 1 in their own object (the build parallelises).
#define PSP_SIDE 1
#include "uwvk_psp_k.hip"
