// <uwv_kalman_filters/PoseUKFConfig.hpp> — the reference's include path
// (src/PoseUKFConfig.hpp); the config types live in reference_types.hpp.
#pragma once
#include "PoseUKF.hpp"
