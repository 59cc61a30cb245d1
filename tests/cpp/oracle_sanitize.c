/* oracle_sanitize.c — the CPU oracle (oracle/uwvk_oracle.c, uwvk_small_oracle.c;
 * test infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (the oracle is the only correctness reference).
 * tests/test_oracle_sanitize.py compiles this file together with the oracle
 * sources (-fsanitize=address,undefined -fno-sanitize-recover=all) and runs it:
 * every PoseUKF entry point (both layouts, both SO3 sides, every update kind,
 * reset, rotation rate, the visual-landmark update), VelocityUKF, BottomUKF and
 * IndirectPoseUKF (its visual update too).  Exit 0 and no sanitizer report = clean. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/uwvk_oracle.h"

static uint64_t g_s = 88172645463325252ull;
static double urand(void) { /* xorshift64*, deterministic */
  g_s ^= g_s >> 12; g_s ^= g_s << 25; g_s ^= g_s >> 27;
  return (double)((g_s * 2685821657736338717ull) >> 11) * (1.0 / 9007199254740992.0);
}
static double nrand(void) { return sqrt(-2.0 * log(urand() + 1e-300)) * cos(6.283185307179586 * urand()); }

static void config(uwvk_pose_config* c, uwvk_uwv_params* u) {
  memset(c, 0, sizeof(*c));
  memset(u, 0, sizeof(*u));
  for (int i = 0; i < 3; i++) {
    c->acceleration.randomwalk[i] = 1e-3; c->acceleration.bias_instability[i] = 1e-4;
    c->rotation_rate.randomwalk[i] = 1e-4; c->rotation_rate.bias_instability[i] = 1e-5;
    c->water_velocity.measurement_std[i] = 0.05; c->max_jerk[i] = 0.5;
  }
  c->acceleration.bias_tau = c->rotation_rate.bias_tau = 600;
  for (int i = 0; i < 6; i++) c->model_noise_parameters.body_efforts_std[i] = i < 3 ? 5 : 1;
  for (int i = 0; i < 9; i++) {
    c->model_noise_parameters.inertia_instability[i] = 10;
    c->model_noise_parameters.lin_damping_instability[i] = 5;
    c->model_noise_parameters.quad_damping_instability[i] = 5;
  }
  c->model_noise_parameters.inertia_tau = c->model_noise_parameters.lin_damping_tau =
      c->model_noise_parameters.quad_damping_tau = 3600;
  c->water_velocity.tau = 900; c->water_velocity.limits = 0.1; c->water_velocity.scale = 1e-3;
  c->water_velocity.adcp_bias_tau = 900; c->water_velocity.adcp_bias_limits = 0.05;
  c->location.latitude = 0.925; c->location.longitude = 0.154;
  c->hydrostatics.water_density = 1025; c->hydrostatics.water_density_limits = 2;
  c->hydrostatics.water_density_tau = 3600; c->hydrostatics.atmospheric_pressure = 101325;
  const double M[6] = {200, 250, 300, 20, 30, 30}, Dl[6] = {20, 30, 40, 5, 5, 5}, Dq[6] = {50, 80, 100, 10, 10, 10};
  for (int i = 0; i < 6; i++) {
    u->inertia_matrix[i * 7] = M[i];
    u->damping_matrices[0][i * 7] = Dl[i];
    u->damping_matrices[1][i * 7] = Dq[i];
  }
  u->weight = u->buoyancy = 2000;
  u->distance_body2centerofbuoyancy[2] = 0.05;
}

static int pose_run(int dof, int right) {
  uwvk_pose_config c;
  uwvk_uwv_params u;
  config(&c, &u);
  or_set_so3_right(right);
  or_pose* f = (or_pose*)calloc(1, or_pose_sizeof());
  const double pos[3] = {1, -2, -10}, pcov[9] = {1, 0, 0, 0, 1, 0, 0, 0, 0.25};
  const double rot[4] = {0.99, 0.01, -0.02, 0.1}, rcov[9] = {1e-4, 0, 0, 0, 1e-4, 0, 0, 0, 2.5e-3};
  double q[4];
  const double nq = sqrt(rot[0] * rot[0] + rot[1] * rot[1] + rot[2] * rot[2] + rot[3] * rot[3]);
  for (int i = 0; i < 4; i++) q[i] = rot[i] / nq;
  int bad = 0, acc = 0;
  bad |= or_pose_init_from_config(f, dof, pos, pcov, q, rcov, &c, &u, NULL);
  or_pose_set_process_noise_from_config(f, &c, 1e-3, NULL);
  const double I3[9] = {1e-4, 0, 0, 0, 1e-4, 0, 0, 0, 1e-4}, I2[4] = {0.05 * 0.05, 0, 0, 0.05 * 0.05};
  double E6[36] = {0};
  for (int i = 0; i < 6; i++) E6[i * 7] = i < 3 ? 25 : 1;
  for (int e = 0; e < 400; e++) {
    const double w[3] = {1e-3 * nrand(), 1e-3 * nrand(), 0.01 + 1e-3 * nrand()};
    const double a[3] = {0.03 * nrand(), 0.03 * nrand(), 9.81 + 0.03 * nrand()};
    bad |= or_pose_set_rotation_rate(f, w, NULL);
    bad |= or_pose_predict(f, 1e-3);
    bad |= or_pose_update_acceleration(f, a, I3, &acc);
    if (e % 50 == 49) {
      const double v[3] = {1 + 0.01 * nrand(), 0.01 * nrand(), 0.01 * nrand()};
      bad |= or_pose_update_velocity(f, v, I3, &acc);
      const double p[1] = {101325 + 10 * 9.81 * 1025 + 100 * nrand()}, pc[1] = {1e4}, s[3] = {0.1, 0, -0.2};
      bad |= or_pose_update_pressure(f, p, pc, s, &acc);
      const double wv[2] = {0.05 * nrand(), 0.05 * nrand()};
      bad |= or_pose_update_water_velocity(f, wv, I2, 0.5, &acc);
      const double xy[2] = {1 + nrand(), -2 + nrand()}, xyc[4] = {0.5, 0, 0, 0.5}, dxy[2] = {0.7, -1.8};
      bad |= or_pose_update_xy(f, xy, xyc, &acc);
      bad |= or_pose_update_delayed_xy(f, xy, xyc, dxy, &acc);
      const double z[1] = {-10 + 0.1 * nrand()}, zc[1] = {0.01};
      bad |= or_pose_update_z(f, z, zc, &acc);
      const double geo[2] = {0.925 + 1e-7 * nrand(), 0.154 + 1e-7 * nrand()}, gc[4] = {4, 0, 0, 4}, gb[3] = {0.5, 0, 0};
      bad |= or_pose_update_geographic(f, geo, gc, gb, &acc);
      double tau[6];
      for (int i = 0; i < 6; i++) tau[i] = 20 * nrand();
      bad |= or_pose_update_efforts(f, tau, E6, (e / 50) % 2, &acc);
    }
  }
  double rr[3];
  or_pose_get_rotation_rate(f, rr);
  {
    const double feat[2] = {320.5, 240.2}, fcov[4] = {1, 0, 0, 1}, fpos[3] = {0.1, 0.05, 0};
    const double marker[7] = {3, -2, -10, 1, 0, 0, 0}, cam[4] = {500, 500, 320, 240},
                 cib[7] = {0, 0, 0, 0.5, 0.5, 0.5, 0.5};
    double cm[36] = {0};
    for (int i = 0; i < 6; i++) cm[i * 7] = 1e-4;
    (void)or_pose_update_visual(f, 1, feat, fcov, fpos, marker, cm, cam, cib);
  }
  const double pose7[7] = {0, 0, -10, 1, 0, 0, 0};
  or_pose_reset_with_external_pose(f, pose7);
  bad |= or_pose_predict(f, 1e-3);
  double x[54], P[53 * 53];
  or_pose_get_state(f, x, P);
  for (int i = 0; i < dof * dof; i++)
    if (!isfinite(P[i])) bad |= 1;
  free(f);
  or_set_so3_right(1); /* back to the default side */
  return bad;
}

static int vel_run(void) {
  uwvk_pose_config c;
  uwvk_uwv_params u;
  config(&c, &u);
  or_vel* v = (or_vel*)calloc(1, or_vel_sizeof());
  const double x[4] = {1, 0, 0, -10}, P[16] = {0.01, 0, 0, 0, 0, 0.01, 0, 0, 0, 0, 0.01, 0, 0, 0, 0, 0.01};
  or_vel_init(v, x, P);
  int bad = or_vel_predict(v, 1e-3) == 0;  /* VelocityUKF.cpp:117-118: no model -> error */
  or_vel_setup_motion_model(v, &u);
  const double I3[9] = {1e-4, 0, 0, 0, 1e-4, 0, 0, 0, 1e-4}, pc[1] = {1e-4};
  for (int e = 0; e < 300; e++) {
    const double w[3] = {0, 0, 0.01}, tau[6] = {20, 0, 0, 0, 0, 0};
    bad |= or_vel_set_gyro(v, w, NULL);
    bad |= or_vel_set_efforts(v, tau, NULL);
    bad |= or_vel_predict(v, 1e-3);
    if (e % 100 == 99) {
      const double d[3] = {1 + 0.01 * nrand(), 0, 0}, z[1] = {-10};
      bad |= or_vel_update_dvl(v, d, I3);
      bad |= or_vel_update_pressure(v, z, pc);
    }
  }
  free(v);
  return bad;
}

static int small_run(void) {
  int bad = 0;
  or_bottom* b = (or_bottom*)calloc(1, or_bottom_sizeof());
  const double bx[4] = {10, 0, 0, 1}, bP[9] = {0.3, 0, 0, 0, 0.003, 0, 0, 0, 0.003}, bQ[9] = {0.02, 0, 0, 0, 1e-3, 0, 0, 0, 1e-3};
  or_bottom_init(b, bx, bP);
  or_bottom_set_process_noise(b, bQ);
  const double vv[3] = {1, 0, 0}, dir[3] = {0.2, 0.1, 0.97}, org[3] = {0, 0, 0}, n[3] = {0, 0.05, 1},
               nc[4] = {1e-3, 0, 0, 1e-3};
  or_bottom_set_velocity(b, vv);
  for (int e = 0; e < 50; e++) {
    bad |= or_bottom_predict(b, 0.1);
    bad |= or_bottom_update_range(b, 10.2 + 0.01 * nrand(), 1e-4, dir, org);
    bad |= or_bottom_update_normal(b, n, nc);
  }
  free(b);
  or_ipose* p = (or_ipose*)calloc(1, or_ipose_sizeof());
  const double ps[3] = {0.1, 0.1, 0.1}, os[3] = {0.01, 0.01, 0.01};
  double Q[36] = {0};
  for (int i = 0; i < 6; i++) Q[i * 7] = 1e-4;
  const double pe[3] = {0.05, -0.02, 0.01}, pes[3] = {0.1, 0.1, 0.1};
  or_ipose_init(p, ps, os, 10.0, pe, pes);
  or_ipose_set_process_noise(p, Q);
  const double ref[7] = {1, 2, -3, 1, 0, 0, 0};
  or_ipose_set_pose_reference(p, ref);
  /* one visual marker feature: marker 2 m in front of the camera (camera frame
   * z forward), pinhole (fx, fy, cx, cy); return codes not checked (the point is
   * memory / UB cleanliness of the augmented update) */
  const double feat[2] = {320.5, 240.2}, fcov[4] = {1, 0, 0, 1}, fpos[3] = {0.1, 0.05, 0};
  const double marker[7] = {3, 2, -3, 1, 0, 0, 0}, cam[4] = {500, 500, 320, 240}, cib[7] = {0, 0, 0, 0.5, 0.5, 0.5, 0.5};
  double cm[36] = {0};
  for (int i = 0; i < 6; i++) cm[i * 7] = 1e-4;
  for (int e = 0; e < 20; e++) {
    bad |= or_ipose_predict(p, 0.1);
    (void)or_ipose_update_visual(p, 1, feat, fcov, fpos, marker, cm, cam, cib);
  }
  double cp[7];
  or_ipose_get_corrected_pose(p, cp);
  free(p);
  return bad;
}

int main(void) {
  int bad = 0;
  for (int right = 0; right < 2; right++) {
    bad |= pose_run(53, right) << 0;
    bad |= pose_run(26, right) << 1;
  }
  bad |= vel_run() << 2;
  bad |= small_run() << 3;
  printf("oracle sanitize run: status %d\n", bad);
  return bad != 0;
}
