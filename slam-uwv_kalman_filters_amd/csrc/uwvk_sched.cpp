// uwvk_sched.cpp — recorded-mission ingestion: the event-ordered replay that
// the reference leaves to its caller (the Rock orogen task and its stream
// aligner), turned into the epoch-indexed log the
// persistent run_log kernels consume (uwvk_pose_log / uwvk_vel_log).
//
// Host-only integer/index work, run once per recording: no device code here.
//
// Semantics:
//  * every IMU sample opens one epoch: RotationRate -> predictionStep(dt) ->
//    Acceleration (PoseUKF.cpp:446-496), dt the mean IMU interval; the IMU
//    stream must be uniform to within dt_tolerance * dt (else UWVK_EINVAL:
//    split the recording at the gap and replay the pieces with their own dt);
//  * a lower-rate sample stamped t is released at the first IMU epoch whose
//    stamp is >= t - time_epsilon (the aligner releases it once the IMU stream
//    has passed it) and integrated after that epoch's predict + acceleration
//    update, in the fixed order DVL, pressure, ADCP cells, BodyEfforts;
//  * two samples of one sensor landing in one epoch are queued: the later
//    one moves to the next free epoch (order is kept, nothing is merged);
//  * samples before the first IMU stamp or queued past the last epoch are
//    dropped and counted.
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/uwvk.h"

namespace {

// assign the ascending stamps t[0..n) to epochs of imu[0..E); returns dropped
int64_t place(const double* imu, int64_t E, const double* t, int64_t n, double eps, uint32_t bit,
              uint32_t* flags, int32_t* index, const uint8_t* extra, uint32_t extra_bit) {
  for (int64_t e = 0; e < E; e++) index[e] = -1;
  int64_t dropped = 0, e = 0, next_free = 0;
  int32_t row = 0;
  for (int64_t s = 0; s < n; s++) {
    const double ts = t[s];
    if (!(ts >= imu[0] - eps)) {  // before the first epoch (or NaN stamp)
      dropped++;
      continue;
    }
    while (e < E && imu[e] < ts - eps) e++;
    int64_t at = e > next_free ? e : next_free;
    if (at >= E) {
      dropped++;
      continue;
    }
    flags[at] |= bit;
    if (extra && extra[s]) flags[at] |= extra_bit;
    index[at] = row++;  // rows of the per-sensor payload are the kept samples, in order
    next_free = at + 1;
  }
  return dropped;
}

bool ascending(const double* t, int64_t n) {
  for (int64_t i = 1; i < n; i++)
    if (!(t[i] >= t[i - 1])) return false;
  return true;
}

}  // namespace

extern "C" uwvk_status uwvk_schedule_streams(const uwvk_stream_times* in, double dt_tolerance, double time_epsilon,
                                             uwvk_schedule* out) {
  if (!in || !out || !in->imu || in->n_imu < 1 || !out->flags) return UWVK_EINVAL;
  if (!(dt_tolerance >= 0.0) || !(time_epsilon >= 0.0)) return UWVK_EINVAL;
  const int64_t E = in->n_imu;
  const double* imu = in->imu;
  if (!ascending(imu, E)) return UWVK_EINVAL;
  double dt = 0.0;
  if (E > 1) {
    dt = (imu[E - 1] - imu[0]) / (double)(E - 1);
    if (!(dt > 0.0)) return UWVK_EINVAL;
    for (int64_t e = 1; e < E; e++)
      if (std::fabs((imu[e] - imu[e - 1]) - dt) > dt_tolerance * dt) return UWVK_EINVAL;
  }
  out->dt = dt;
  out->epochs = E;
  for (int64_t e = 0; e < E; e++) out->flags[e] = UWVK_EV_ACC;
  struct K {
    const double* t;
    int64_t n;
    int32_t* idx;
    uint32_t bit;
  } ks[4] = {{in->dvl, in->n_dvl, out->dvl_index, UWVK_EV_DVL},
             {in->pressure, in->n_pressure, out->pressure_index, UWVK_EV_PRESSURE},
             {in->adcp, in->n_adcp, out->adcp_index, UWVK_EV_ADCP},
             {in->efforts, in->n_efforts, out->efforts_index, UWVK_EV_EFFORTS}};
  for (int k = 0; k < 4; k++) {
    out->kept[k] = 0;
    out->dropped[k] = 0;
    if (ks[k].n < 0 || (ks[k].n > 0 && !ks[k].t)) return UWVK_EINVAL;
    if (!ks[k].idx) {
      if (ks[k].n > 0) return UWVK_EINVAL;
      continue;
    }
    if (!ascending(ks[k].t, ks[k].n)) return UWVK_EINVAL;
    const uint8_t* extra = k == 3 ? in->efforts_velocity_only : nullptr;
    out->dropped[k] = place(imu, E, ks[k].t, ks[k].n, time_epsilon, ks[k].bit, out->flags, ks[k].idx, extra,
                            UWVK_EV_EFFORTS_VELOCITY_ONLY);
    out->kept[k] = ks[k].n - out->dropped[k];
  }
  return UWVK_OK;
}

// ADCP cell weighting for PoseUKF::integrateMeasurement(WaterVelocityMeasurement,
// cell_weighting) (PoseUKF.cpp:133-151, 604-611): the weight of the deeper
// water layer in cell i.  Cell centres sit at r_i = first_cell_blank +
// (i + 1/2) cell_size from the transducer (PoseUKFConfig.hpp:34-38); the
// nearest cell measures the vehicle's layer (weight 0), the farthest the layer
// below (weight 1), linear in range between.  Cells whose beam correlation is
// below minimum_correlation (PoseUKFConfig.hpp:40-41) are marked invalid (the
// caller skips them).  The reference computes this in its caller; this rule
// is the engine's (unpinned).
extern "C" uwvk_status uwvk_adcp_cell_weighting(const uwvk_water_velocity* wv, int32_t cells,
                                                const double* correlation, double* weighting, uint8_t* valid) {
  if (!wv || cells < 1 || cells > 64 || !weighting) return UWVK_EINVAL;
  if (!(wv->cell_size > 0.0) || !(wv->first_cell_blank >= 0.0)) return UWVK_EINVAL;
  const double r0 = wv->first_cell_blank + 0.5 * wv->cell_size;
  const double r1 = wv->first_cell_blank + (cells - 0.5) * wv->cell_size;
  for (int32_t i = 0; i < cells; i++) {
    const double r = wv->first_cell_blank + (i + 0.5) * wv->cell_size;
    weighting[i] = cells == 1 ? 0.0 : (r - r0) / (r1 - r0);
    if (valid) valid[i] = correlation ? (uint8_t)(correlation[i] >= wv->minimum_correlation) : (uint8_t)1;
  }
  return UWVK_OK;
}
