// <uwv_kalman_filters/VelocityUKF.hpp> — the reference's include path
// (src/VelocityUKF.hpp); VelocityUKF lives in the same facade header as PoseUKF.
#pragma once
#include "PoseUKF.hpp"
