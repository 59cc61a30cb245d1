// <uwv_kalman_filters/PoseUKF.hpp> — the reference's include path and namespace
// (src/PoseUKF.hpp, namespace uwv_kalman_filters) over this engine's facade, so
// that a caller written against the reference compiles unchanged: its
// PoseUKF / VelocityUKF, the nested MEASUREMENT types, PoseUKFConfig and its
// parts, PoseState, and uwv_dynamic_model::UWVParameters [EXT] resolve to the
// facade's (uwv_kalman_filters_amd/PoseUKF.hpp).  Where the real
// uwv_dynamic_model headers are installed, define UWVK_NO_UWV_DYNAMIC_MODEL_ALIAS
// and convert its UWVParameters field by field.
#pragma once
#include "../uwv_kalman_filters_amd/PoseUKF.hpp"

namespace uwv_kalman_filters {
using namespace ::uwv_kalman_filters_amd;
}  // namespace uwv_kalman_filters

#ifndef UWVK_NO_UWV_DYNAMIC_MODEL_ALIAS
namespace uwv_dynamic_model {
using UWVParameters = ::uwv_kalman_filters_amd::UWVParameters;
}  // namespace uwv_dynamic_model
#endif
