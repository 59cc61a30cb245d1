// BottomUKF.hpp — C++ host facade for the batched BottomUKF (uwvk_bottom_* C ABI).
//
// Mirrors src/BottomUKF.hpp:26-53: state {distance, normal (S2)}, stored per
// instance as {d, nx, ny, nz}; 3x3 covariance.  One object = a batch of
// independent filters on one gfx950 device.
#pragma once
#include "PoseUKF.hpp"

namespace uwv_kalman_filters_amd {

struct RangeMeasurement : BatchMeasurement<1> {};  // MEASUREMENT(RangeMeasurement, 1) (BottomUKF.hpp:30)
// NormalType measurement: mu batch*3 (normalised by the filter), cov batch*4 or shared_cov
struct NormalMeasurement : BatchMeasurement<3> {};

class BottomUKF {
 public:
  // BottomUKF(initial_state, state_cov) (BottomUKF.cpp:40-46): state batch*4, cov batch*9
  BottomUKF(int64_t batch, const std::vector<double>& initial_state, const std::vector<double>& state_cov,
            int device = 0)
      : batch_(batch) {
    check(uwvk_bottom_create(batch, device, &h_), "uwvk_bottom_create");
    if (initial_state.size() != (size_t)batch * 4 || state_cov.size() != (size_t)batch * 9) {
      uwvk_bottom_destroy(h_);
      throw std::invalid_argument("BottomUKF: wrong size");
    }
    check(uwvk_bottom_init(h_, initial_state.data(), state_cov.data()), "BottomUKF");
  }
  BottomUKF(const BottomUKF&) = delete;
  BottomUKF& operator=(const BottomUKF&) = delete;
  virtual ~BottomUKF() { uwvk_bottom_destroy(h_); }

  int64_t batch() const { return batch_; }
  // setProcessNoiseCovariance [EXT base]: 3x3 shared by the batch
  void setProcessNoiseCovariance(const std::array<double, 9>& Q) {
    check(uwvk_bottom_set_process_noise(h_, Q.data()), "setProcessNoiseCovariance");
  }
  // setVelocity (BottomUKF.cpp:69-72): batch*3
  void setVelocity(const std::vector<double>& v) {
    if (v.size() != (size_t)batch_ * 3) throw std::invalid_argument("setVelocity: wrong size");
    check(uwvk_bottom_set_velocity(h_, v.data()), "setVelocity");
  }
  void predictionStep(double delta_t) { check(uwvk_bottom_predict(h_, delta_t), "predictionStep"); }
  // integrateMeasurement(RangeMeasurement, unit_direction, origin) (BottomUKF.cpp:56-61)
  void integrateMeasurement(const RangeMeasurement& m, const std::array<double, 3>& unit_direction,
                            const std::array<double, 3>& origin) {
    if (m.mu.size() != (size_t)batch_) throw std::invalid_argument("RangeMeasurement: wrong size");
    check(uwvk_bottom_update_range(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(), m.shared_cov[0],
                                   unit_direction.data(), origin.data(), m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(RangeMeasurement)");
  }
  // integrateMeasurement(NormalType, measurement_cov) (BottomUKF.cpp:63-67)
  void integrateMeasurement(const NormalMeasurement& m, const std::array<double, 4>& measurement_cov) {
    if (m.mu.size() != (size_t)batch_ * 3) throw std::invalid_argument("NormalType: wrong size");
    check(uwvk_bottom_update_normal(h_, m.mu.data(), m.cov.empty() ? nullptr : m.cov.data(),
                                    measurement_cov.data(), m.mask.empty() ? nullptr : m.mask.data()),
          "integrateMeasurement(NormalType)");
  }
  void getState(std::vector<double>& x, std::vector<double>* P = nullptr) {
    x.resize((size_t)batch_ * 4);
    if (P) P->resize((size_t)batch_ * 9);
    check(uwvk_bottom_get_state(h_, x.data(), P ? P->data() : nullptr), "getState");
  }

 private:
  int64_t batch_;
  uwvk_bottom* h_ = nullptr;
};

}  // namespace uwv_kalman_filters_amd
