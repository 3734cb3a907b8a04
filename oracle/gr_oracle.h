/*
 * gr_oracle.h — CPU restatement of the reference racing-env step.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so; the product path
 * (generalizableracing_amd) never does.
 *
 * Array-of-structs, one env at a time, following the reference's op order
 * line by line (citations in gr_oracle.c).  Parity is pinned two ways:
 *   1. against golden vectors produced by running the reference's own
 *      DroneDynamics / CTBRController / ThrustController (tests/golden/);
 *   2. against hand-derived known answers for the manager-level logic whose
 *      reference implementation lives in Isaac Lab (absent; "parity
 *      unpinned" for those Isaac-Lab formulas).
 */
#ifndef GR_ORACLE_H
#define GR_ORACLE_H

#include "../include/gr.h"

typedef struct gro_env {
  float p[3], q[4], v[3], w[3], alpha[3];
  float T, tau[3];
  float lag[4];
  float thr_err, noise_level, k2[3], k1[3];
  float ep_sum[7], m_actrate;
  float Kp[3], cT, Kd[3], m_plant, ctau[3], m_ctrl, J[3], motor_w[4];
  float rotor[4]; /* k2 k1 k0 kappa (dr_rotor; else the nominal constants) */
  int32_t ep_len, acc, epoch, gate_id, level, type, azero;
} gro_env;

typedef struct gro_out {
  float* obs_policy; /* [n][16] */
  float* obs_critic; /* [n][16] */
  float* obs_aux;    /* [n] */
  float* reward;     /* [n] */
  uint8_t* terminated;
  uint8_t* time_out;
  int64_t* dones;
  float* log_out; /* [GR_LOG_SLOTS] */
} gro_out;

typedef struct gro_tracks {
  const float* gates;  /* [T*L][G][20] */
  const float* tracks; /* [T*L][4] */
  const float* obst;         /* [T*L][max_obst][GR_OBST_FLOATS] (NULL: no obstacles) */
  const int32_t* obst_count; /* [T*L] */
  int32_t max_obst;
} gro_tracks;

size_t gro_env_size(void);
/* env type boundaries: type of env i = #{t >= 1 : i >= type_start[t]} */
void gro_type_starts(const gr_config* cfg, int32_t* type_start /* [num_types+1] */);
void gro_init(const gr_config* cfg, gro_env* envs, int n, gro_out* out);
void gro_reset(const gr_config* cfg, gro_env* envs, int n, const uint8_t* mask, const gro_tracks* tr,
               uint32_t* counter, gro_out* out);
void gro_step(const gr_config* cfg, gro_env* envs, int n, const float* actions, const gro_tracks* tr,
              uint32_t* counter, gro_out* out);
void gro_observe(const gr_config* cfg, gro_env* envs, int n, const gro_tracks* tr, uint32_t* counter,
                 gro_out* out);
/* same contract as gr_test_dynamics (include/gr.h) */
void gro_test_dynamics(const gr_config* cfg, int n, int mode, const float* state_in, const float* ang_acc_b,
                       const float* cmd, const float* ctrl_in, const float* par, const float* drag,
                       float* state_out, float* ctrl_out, float* extra_out);
/* collision lattice count for one pose (exposed for known-answer tests) */
int gro_collision_count(const gr_config* cfg, const gro_tracks* tr, int track, const float p[3], const float q[4]);
void gro_test_math(int fn, int n, const float* x, const float* y, float* out);
void gro_test_philox(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                     uint32_t* out4);
void gro_test_fields6(int n, const uint32_t* in4, uint32_t* out6);
void gro_test_normal24(int n, const uint32_t* w, float* z);
void gro_test_cam_noise(uint32_t gid, uint32_t cnt, uint32_t q0, int nq, uint32_t k0, uint32_t k1, float* z);
/* depth camera + depth_image observation, same contract as gr_camera_render (include/gr.h);
 * cnt = the observation counter of the call the images belong to */
void gro_camera(const gr_config* cfg, const gr_camera_config* kcfg, const gro_env* envs, int n, const gro_tracks* tr,
                int mode, const uint8_t* mask, const uint8_t* terminated, const uint8_t* time_out, uint32_t cnt,
                float* depth, int32_t* age, const float* obs_p16, const float* obs_c16, float* out_p, float* out_c);
/* one ray: distance_to_image_plane of pixel (u, v) from body pose (p, q) on track `track` */
float gro_camera_ray(const gr_config* cfg, const gr_camera_config* kcfg, const gro_tracks* tr, int track,
                     const float p[3], const float q[4], int u, int v);
void gro_camera_cull_check(const gr_config* cfg, const gr_camera_config* kcfg, const gro_tracks* tr, int track,
                           const float p[3], const float q[4], int64_t out[8]);
void gro_camera_frame(const gr_config* cfg, const gr_camera_config* kcfg, const float p[3], const float q[4],
                      float* out);
/* the random values env i consumes (kind 0 observation noise, 1 gate noise, 2 reset, 3 startup; gr_oracle.c) */
void gro_draws(const gr_config* cfg, int i, int kind, uint32_t c1, uint32_t c3, float* out);
/* OpenMP threads gro_step uses (1 without OpenMP) */
int gro_num_threads(void);

#endif
