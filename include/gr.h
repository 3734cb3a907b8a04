/*
 * gr.h — C ABI of libgr.so, the MI355X-native step of the drone-racing task
 * `DiffLab-Quadcopter-CTBR-Racing-v0` (yufengsjtu/GeneralizableRacing).
 *
 * The reference has no native boundary of its own: the env step is Python
 * (Isaac Lab managers + PhysX).  The entry points below are what its Python
 * layer would bind to replace that step; each cites the reference code it
 * replaces (paths relative to the reference repo root):
 *
 *   gr_create / gr_bind_* / gr_init   ManagerBasedDiffRLEnv.__init__ + load_managers
 *                                     (extensions/diff.lab/diff/lab/envs/manager_based_diff_rl_env.py:108-141)
 *                                     + startup events (.../quadcopter_diff/mdp/events.py:30-137)
 *   gr_reset                          ManagerBasedEnv.reset -> _reset_idx
 *                                     (manager_based_diff_rl_env.py:362-410)
 *   gr_step                           ManagerBasedDiffRLEnv.step (manager_based_diff_rl_env.py:160-267)
 *   gr_observe                        RslRlVecEnvWrapper.get_observations -> ObservationManager.compute
 *   gr_test_dynamics                  DroneDynamics.step / CTBRController.compute in isolation
 *                                     (.../mdp/dynamics/droneDynamics.py:119-135,
 *                                      extensions/diff.lab/diff/lab/controllers/controller_diff.py:120-144)
 *
 * Conventions: plain C, no exceptions cross the ABI, every function returns 0
 * on success and a negative code on failure (gr_last_error() has the text).
 * All per-env buffers are allocated by the caller (PyTorch) on the device;
 * the library never allocates inside gr_step/gr_reset/gr_observe, never
 * synchronises the host, and launches only on the caller's stream, so the
 * calls are hipGraph-capturable.
 */
#ifndef GR_H
#define GR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: GR_NUM_PLANES 17 (obstacle hint, rotor constants), gr_policy_args.precision, the observation sink and the
 * status word; gr_policy_args_size.  3: gr_stem1_* y_rows / gy_rows.  4: the gr_stem1_* / gr_stem12_* row indices
 * (`rows` after `off`).  5: gr_stem12_backward_w2 (conv2's weight gradient inside the first block's backward).
 * 6: gr_test_camera_slots; gr_stem12_forward / gr_stem12_backward_w2 `moments` */
#define GR_ABI_VERSION 6

/* ---- status codes ---- */
#define GR_OK 0
#define GR_ERR_ARG -1
#define GR_ERR_HIP -2
#define GR_ERR_STATE -3

/* ---- integrators ---- */
#define GR_INTEGRATOR_DD_EXPLICIT 0   /* DroneDynamics.step order, one explicit step of step_dt */
#define GR_INTEGRATOR_SEMI_IMPLICIT 1 /* `decimation` semi-implicit Euler substeps of sim_dt (PhysX-like) */

/* ---- state layout: float planes, each [num_envs][4] fp32, plane-major ---- */
#define GR_P_POSQ 0   /* px py pz qw            (env-local frame: world - env_origin) */
#define GR_P_QV 1     /* qx qy qz vwx           (q = w,x,y,z body->world; v world frame) */
#define GR_P_VW 2     /* vwy vwz wbx wby        (w = body angular rate) */
#define GR_P_WA 3     /* wbz abx aby abz        (a = last body angular acceleration) */
#define GR_P_CTRL 4   /* T tx ty tz             (CTBR thrust/torque delay-filter state) */
#define GR_P_LAG 5    /* action-lag buffer: tanh(previous raw action) (only its tanh is ever used) */
#define GR_P_RST0 6   /* thr_est_err noise_level k2x k2y */
#define GR_P_RST1 7   /* k2z k1x k1y k1z        (quadratic / linear drag) */
#define GR_P_EP0 8    /* episode reward sums 0..3 */
#define GR_P_EP1 9    /* episode reward sums 4..6, last action_rate metric */
#define GR_P_PAR0 10  /* Kp xyz, thrust filter coefficient exp(-dt/tau_T) */
#define GR_P_PAR1 11  /* Kd xyz, plant mass */
#define GR_P_PAR2 12  /* torque filter coefficients exp(-dt/tau_tau) xyz, controller mass */
#define GR_P_PAR3 13  /* plant inertia diag xyz, spare */
#define GR_P_MOTOR 14 /* rotor speeds (motor model only) */
#define GR_P_OHINT 15 /* obstacle tracks only: the obstacle-grid list of the env's cell (int first, int count + 1,
                         lower corner x, y of the cell grown by the margin); all-zero = no hint */
#define GR_P_ROTOR 16 /* rotor constants of the env (thrust map k2 k1 k0, torque ratio kappa): config C5's
                         rotor-constant DR, read only when dr_rotor */
#define GR_NUM_PLANES 17
/* int plane [num_envs][4] int32: episode_length, accumulate_gates, epoch, packed */
#define GR_I_EPLEN 0
#define GR_I_ACC 1
#define GR_I_EPOCH 2
#define GR_I_PACKED 3 /* bits 0-7 gate_id, 8-15 terrain level, bit 16: action-manager buffers zeroed */

#define GR_OBS_DIM 16
#define GR_GATE_FLOATS 20 /* per-gate record, see DESIGN.md "track table" */
#define GR_TRACK_FLOATS 4 /* per-track record: ground_z, origin_z, start_gate, num_gates */
#define GR_OBST_FLOATS 20 /* per-obstacle record, see generalizableracing_amd/csrc/gr_obstacles.h */
/* obstacle primitive kinds (record float 16) */
#define GR_OBST_BOX 0
#define GR_OBST_CYLINDER 1
#define GR_OBST_SPHERE 2
#define GR_OBST_CAPSULE 3

/* ---- log slots (extras["log"]) ---- */
#define GR_LOG_NRESET 0
#define GR_LOG_EPSUM0 1 /* 7 reward terms, declaration order of RewardsCfg */
#define GR_LOG_ACC 8
#define GR_LOG_M_ACTRATE 9
#define GR_LOG_M_LINSPD 10
#define GR_LOG_M_ANGSPD 11
#define GR_LOG_T_TIMEOUT 12
#define GR_LOG_T_CONTACT 13 /* base_contact (stage 1/2) or outofbound (stage 0) */
#define GR_LOG_T_BADPOSE 14
#define GR_LOG_LEVEL 15
#define GR_LOG_NOISE 16
#define GR_LOG_SLOTS 20

/*
 * Task configuration.  Field meanings follow the reference cfg classes; the
 * defaults (gr_config_default) are those of QuadcopterRacingCTBREnvCfg with
 * TRAINING_STAGE=1 (racing_ctbr_env.py:97-398) and CTBRControllerCfg
 * (controller_diff_cfg.py:22-54).  All fields are 4 bytes: no padding.
 */
typedef struct gr_config {
  int32_t num_envs;
  int32_t env_id_offset; /* rank * num_envs: distinct RNG streams per shard */
  uint32_t seed_lo, seed_hi;
  int32_t num_types;      /* terrain columns (20) */
  int32_t num_levels;     /* terrain rows (10) */
  int32_t max_gates;      /* gates per track (8; 32 for config C5) */
  int32_t max_init_level; /* max_init_terrain_level (5) */
  int32_t stage;          /* TRAINING_STAGE 0/1/2 */
  int32_t integrator;
  int32_t decimation;         /* 3 */
  int32_t max_episode_length; /* ceil(episode_length_s / step_dt) */
  float sim_dt;               /* 0.01 */
  float step_dt;              /* sim_dt * decimation */
  float episode_length_s;     /* 6.0 */
  float gravity;              /* 9.81 */
  /* vehicle */
  float mass;        /* nominal (USD) mass: ASSUMPTION 0.6 kg, the USD is not in the reference */
  float inertia[3];  /* diag(0.0015, 0.002, 0.004) diff_action.py:59 */
  float arm_length;  /* 0.09 */
  float kappa;       /* 0.016 */
  float motor_tau;   /* 1e-4 */
  float motor_omega[2];
  float thrustmap[3];
  float max_thrust_weight_ratio; /* 3 */
  float body_rate_bound;         /* 6 */
  float rate_gain_p[3];
  float rate_gain_d[3];
  float thrust_ctrl_delay;
  float torque_ctrl_delay[3];
  int32_t use_motor_model;
  int32_t action_lag; /* 0 or 1 */
  /* drag, dynamics.yaml */
  float drag1[3];
  float drag1_rand;
  float drag2[3];
  float drag2_rand;
  float z_drag;
  float z_drag_rand;
  int32_t random_drag;
  /* startup domain randomisation (EventCfg) */
  float mass_add_range[2];
  float inertia_scale_range[2];
  float pid_scale_range[2];
  float delay_scale_range[2];
  int32_t dr_startup; /* apply the startup events */
  int32_t dr_plant;   /* integrate with the randomised plant mass/inertia (PhysX role) */
  /* reset (reset_root_state_racing) */
  float spawn_pos[3];       /* default root pos (0,0,0.5) */
  float reset_pos_half[3];  /* U(-h, h) */
  float reset_att_half[3];  /* roll, pitch, yaw offset */
  float reset_vel_half[6];
  /* command (RacingCommandCfg) */
  float gate_threshold; /* 0.35 */
  float gate_noise_pos[3]; /* half ranges */
  int32_t add_gate_noise;
  /* curriculum */
  int32_t level_up_threshold;   /* 3 */
  int32_t level_down_threshold; /* 2 */
  int32_t noise_curriculum;     /* stage 1 */
  int32_t noise_enhance_threshold; /* 4 */
  int32_t noise_decay_threshold;   /* 3 */
  float noise_enhance;  /* 0.02 */
  float noise_decay;    /* 0.03 */
  /* observation noise */
  int32_t obs_noise;
  float obs_lin_vel_noise; /* 0.03 */
  float obs_att_noise;     /* 0.05 */
  /* reward weights in RewardsCfg order (0 disables a term) */
  float w_progress, w_body_rate, w_action_rate, w_collision, w_perception, w_success, w_bad_pose;
  /* collision body: lattice half extents (0.707*0.09, 0.707*0.09, 0.5*0.05) */
  float collider_half[3];
  int32_t collision_count_threshold; /* contact if #lattice points inside > this (stage1: 0, stage0: 2) */
  float out_of_bound[2];             /* stage 0 world-z bounds (0, 10) */
  int32_t term_contact;  /* base_contact / outofbound termination enabled */
  int32_t term_bad_pose;
  /* config C5: per-env rotor constants (thrust map k2, k1, k0 and kappa, each x U(lo, hi)) drawn at start-up;
   * the gross-thrust clamp and, with the motor model, the allocation and motor map follow them per env */
  int32_t dr_rotor;
  float rotor_scale_range[2]; /* (0.9, 1.1) */
  int32_t reserved[5];
} gr_config;

/*
 * Output buffers are written by every call; callers that keep the previous
 * call's tensors alive (rsl_rl stores `obs` from step t while step t+1 runs)
 * rebind a second output set each call and point the prev_* fields at the
 * set written last (ping-pong).  prev_* may alias the outputs.
 */
typedef struct gr_buffers {
  float* state;        /* [GR_NUM_PLANES][num_envs][4] */
  int32_t* istate;     /* [num_envs][4] */
  float* obs_policy;   /* [num_envs][16] */
  float* obs_critic;   /* [num_envs][16] */
  float* obs_aux;      /* [num_envs] */
  float* reward;       /* [num_envs] */
  uint8_t* terminated; /* [num_envs] (bool) */
  uint8_t* time_out;   /* [num_envs] (bool) */
  int64_t* dones;      /* [num_envs] */
  const float* prev_obs_critic; /* last action (cols 12-15) carried by gr_reset/gr_observe */
  const float* prev_obs_aux;
  const uint8_t* prev_time_out;
  float* log_partial;    /* [gr_num_log_rows()][GR_LOG_SLOTS]: this call's per-wave log sums */
  uint32_t* counters;    /* [2]: observation-noise call counter, double-buffered by call parity */
  int32_t counter_index; /* 0/1: this call reads counters[i] and writes counters[i^1] = counters[i] + 1 */
  int32_t reserved;
} gr_buffers;

/*
 * Front depth camera (optional).  Reference: `front_camera = RayCasterCameraCfg(...)`
 * (extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/racing_ctbr_env.py:77-95,
 * update_period :390-391) and the `depth_image` observation term (.../quadcopter_diff/mdp/
 * observation.py:65-94), whose output the policy / critic groups concatenate after the 16
 * state terms (racing_ctbr_env.py:141-160): obs rows are [16 state | H*W image].
 * Defaults (gr_camera_config_default) are those of the reference cfg.
 */
typedef struct gr_camera_config {
  int32_t width, height;  /* 96, 72 */
  float fx, fy, cx, cy;   /* pinhole intrinsics in pixels (from_intrinsic_matrix, :87-91) */
  float offset_pos[3];    /* (0.01, 0, 0) in the body frame */
  float offset_rot[4];    /* (0.991, 0, -0.131, 0) w,x,y,z, "world" convention; normalised */
  float max_distance;     /* 10, depth_clipping_behavior "max" */
  float update_period;    /* 0.04 s */
  float noise_std;        /* 0.02: policy image x (1 + N(0,1) * std) */
  int32_t add_noise;      /* policy group add_noise=True (critic: False) */
  float obs_scale;        /* 10: depth_image normalize (> 10 -> 10, / 10) */
  int32_t reserved[6];
} gr_camera_config;

/* Camera buffers (caller-owned device memory, 16-byte aligned). */
typedef struct gr_camera_buffers {
  float* depth;      /* [num_envs][H*W] persistent distance_to_image_plane (m), the sensor's data buffer */
  int32_t* age;      /* [num_envs] env steps since the last render; -1 = outdated (render at next call) */
  float* obs_policy; /* [num_envs][16 + H*W]: state terms copied from gr_buffers.obs_policy, noisy image */
  float* obs_critic; /* [num_envs][16 + H*W]: state terms from gr_buffers.obs_critic, clean image */
} gr_camera_buffers;

/* gr_camera_render modes: which envs are outdated before the image observation is formed */
#define GR_CAM_STEP 0    /* after gr_step: terminated|time_out envs, and envs whose period elapsed */
#define GR_CAM_RESET 1   /* after gr_reset(mask): the masked envs (mask NULL: all) */
#define GR_CAM_OBSERVE 2 /* after gr_observe: only envs still outdated (age -1) */

typedef struct gr_ctx gr_ctx;

int gr_abi_version(void);
/* SHA-256 (64 hex digits) of the sources this library was built from: generalizableracing_amd/csrc's SRCS then HDRS
 * in the order its Makefile lists them, concatenated (a stale binary next to newer sources shows as a mismatch). */
const char* gr_source_sha256(void);
int gr_config_default(gr_config* cfg);
size_t gr_config_size(void);
int gr_create(const gr_config* cfg, gr_ctx** out);
int gr_destroy(gr_ctx* ctx);
/* the last error's text; safe from any host thread (a copy per calling thread, valid until its next call) */
const char* gr_last_error(const gr_ctx* ctx);
/* number of workgroups of the step kernel */
int gr_num_blocks(const gr_ctx* ctx);
/* rows of a call's log slab (one per wave) */
int gr_num_log_rows(const gr_ctx* ctx);
/* extras["log"] on demand: reduce one call's log slab into GR_LOG_SLOTS means
 * (prev: the previous call's finalized values, kept when no env reset; may be NULL) */
int gr_log_finalize(gr_ctx* ctx, const float* log_partial, const float* prev, float* out, void* stream);
/* algorithmic HBM bytes per env-step of the fused step kernel (read, written; with the bound observation sink) */
int gr_bytes_per_env_step(const gr_ctx* ctx, int64_t* read_bytes, int64_t* written_bytes);

/* Track table on the device (caller-owned):
 *   gates  [num_types*num_levels][max_gates][GR_GATE_FLOATS] fp32
 *   tracks [num_types*num_levels][GR_TRACK_FLOATS] fp32
 * track index = type * num_levels + level (the reference stores gate_pose as
 * [col=type][row=level], terrain_importer.py:150-153). */
int gr_bind_tracks(gr_ctx* ctx, const float* gates, const float* tracks);

/* Track obstacles (caller-owned device memory, kept alive while bound): the walls, orbits and
 * ground obstacles the reference's sub-terrain generators add to the terrain mesh
 * (extensions/diff.lab/diff/lab/terrains/trimesh/racing_terrains.py:87-150,254-319,510-610,
 * 750-815; primitives trimesh/utils.py:35-131).  They count in the collision test (PhysX
 * contact, racing_ctbr_env.py:253-256,306-311) and in the depth camera (the terrain mesh the
 * RayCasterCamera casts against).  Records: GR_OBST_FLOATS each (gr_obstacles.h).
 * Per track a uniform xy grid over the obstacles: cell (ix, iy) of track k is
 * cells[grid_i[k].z + iy * grid_i[k].x + ix] = (first item, item count) into `items`, which
 * holds copies of the records whose cull sphere reaches into that cell. */
typedef struct gr_obstacles {
  const float* records;   /* [num_types*num_levels][max_obstacles][GR_OBST_FLOATS] */
  const int32_t* counts;  /* [num_types*num_levels] obstacles per track */
  const float* grid_f;    /* [num_types*num_levels][4]: x0, y0 (env-local), 1/cell, cell */
  const int32_t* grid_i;  /* [num_types*num_levels][4]: nx, ny, first cell, 0 */
  const int32_t* cells;   /* [num_cells][2]: first item, item count */
  const float* items;     /* [num_items][GR_OBST_FLOATS] */
  int32_t max_obstacles, num_cells, num_items, reserved;
} gr_obstacles;
/* obst == NULL unbinds (obstacle-free tracks).  Validates counts and the grid (host copies of
 * the small index arrays). */
int gr_bind_obstacles(gr_ctx* ctx, const gr_obstacles* obst);
/* Terrain swap of the periodic regeneration (EventCfg.reset_terrain -> reset_terrain_period,
 * extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/mdp/events.py:180-204) without a host
 * synchronisation: the new tables are validated from HOST copies (`tracks_host` [num_types*num_levels]
 * [GR_TRACK_FLOATS]; `obst_host` with the host counts / grid_f / grid_i / cells, sizes as `obst`), then, ordered on
 * `stream`, the device gate table is packed into the context's table and the obstacle hints are cleared; `obst`
 * (device arrays, caller-owned, kept alive while bound) is bound, or NULL unbinds.  Launches enqueued earlier on
 * `stream` run on the previous tables.  Same tables -> same steps as gr_bind_tracks + gr_bind_obstacles. */
int gr_swap_terrain(gr_ctx* ctx, const float* gates, const float* tracks, const float* tracks_host,
                    const gr_obstacles* obst, const gr_obstacles* obst_host, void* stream);

/* Resident terrain: the periodic regeneration (EventCfg.reset_terrain -> reset_terrain_period, .../quadcopter_diff/
 * mdp/events.py:180-204) as a swap with fixed device addresses, so the interval step can be captured in a hipGraph.
 *   gr_terrain_reserve: the context allocates, once, the arrays the kernels read the terrain from (the packed gate
 *     table; for obstacle tracks records [T*L][max_obstacles][GR_OBST_FLOATS], counts, grids, cells [max_cells][2],
 *     items [max_items][GR_OBST_FLOATS]) and a staging copy of them, and binds the live ones (max_obstacles == 0:
 *     obstacle-free tracks).  Synchronises the device.  Called again it reallocates (the kernel arguments change:
 *     graphs captured before must be captured again).  Each call increments the terrain epoch (gr_terrain_epoch):
 *     a graph owner records the epoch at capture and must not replay once it changed.
 *   gr_terrain_stage: validates a generation from HOST arrays (gates / tracks as gr_bind_tracks; obst_host: every
 *     array a host pointer, max_obstacles / num_cells / num_items its sizes; NULL iff reserved obstacle-free) and
 *     uploads it into the staging arrays on `stream` (asynchronous from pinned memory).  Touches only the staging
 *     set: it may run on another host thread and stream while the env's calls run; the caller orders it after the
 *     previous gr_terrain_commit (a stream wait).  The only context fields it writes are the staging set, its
 *     staged header / grid scalars (read by the next commit) and, under a lock, the error text; the caller must not
 *     run gr_terrain_reserve, _commit or another _stage concurrently with it.  GR_ERR_CAPACITY: the generation exceeds the reservation.
 *   gr_terrain_commit: makes the last staged generation live, ordered on `stream`: one kernel copies the staged
 *     arrays over the live ones (extents from the staged header, on the device), packs the gate table and clears
 *     the per-env obstacle hints.  No host argument, check or synchronisation: capturable, and a graph replay
 *     commits whatever was staged last.  Same tables -> same steps as gr_bind_tracks + gr_bind_obstacles. */
#define GR_ERR_CAPACITY -4
int gr_terrain_reserve(gr_ctx* ctx, int32_t max_obstacles, int32_t max_cells, int32_t max_items);
int gr_terrain_stage(gr_ctx* ctx, const float* gates_host, const float* tracks_host, const gr_obstacles* obst_host,
                     void* stream);
int gr_terrain_commit(gr_ctx* ctx, void* stream);
/* number of gr_terrain_reserve calls so far (0: the terrain arrays are the caller's, gr_bind_tracks) */
int64_t gr_terrain_epoch(const gr_ctx* ctx);
int gr_bind_buffers(gr_ctx* ctx, const gr_buffers* bufs);

/* Observation sink (config C5's bf16 rollout buffers): every following gr_step / gr_reset / gr_observe also
 * writes the policy and critic rows it computes into policy[num_envs][16] / critic[num_envs][16] of `dtype`
 * (GR_DTYPE_BF16: round-to-nearest-even, as torch's float -> bfloat16; GR_DTYPE_F32: the rows as they are)
 * — the rollout storage's slot for the next transition (standalone/rsl_rl/ext/storage/rollout_storage.py:
 * 74-88 add_transitions), so the storage takes the observations without a copy / cast pass.  Rebind per
 * call (each step has its own slot); policy == NULL unbinds.  16-byte aligned device memory. */
#define GR_DTYPE_F32 0
#define GR_DTYPE_BF16 1
int gr_bind_obs_sink(gr_ctx* ctx, void* policy, void* critic, int dtype);

/* startup: nominal state, startup DR (gains/delays/mass/inertia), initial levels */
int gr_init(gr_ctx* ctx, void* stream);
/* reset envs whose mask byte is non-zero (mask == NULL: all), then observe all */
int gr_reset(gr_ctx* ctx, const uint8_t* mask, void* stream);
/* one policy step: actions [num_envs][4] fp32 pre-tanh, device memory */
int gr_step(gr_ctx* ctx, const float* actions, void* stream);
/* recompute observations (fresh observation noise), no state change */
int gr_observe(gr_ctx* ctx, void* stream);
/* Which step_kernel instantiation gr_step launches with the current bindings (so a test can assert it checks the
 * kernel a benchmark times).  Same selection as the launcher (gr_kernels.hip step_variant). */
#define GR_STEP_L2 0          /* step_kernel<false, false>: track table read from L2 (too large for the LDS slice) */
#define GR_STEP_LDS 1         /* step_kernel<true, false>: LDS track slice, any gate count */
#define GR_STEP_LDS8 2        /* step_kernel<true, false, 8>: LDS slice, tracks of <= 8 gates */
#define GR_STEP_LDS8_LEAN 3   /* step_kernel<true, false, 8, 1>: + C3's configuration compiled in (the bench headline) */
#define GR_STEP_OBST 4        /* step_kernel<false, true>: obstacle tracks */
#define GR_STEP_OBST_LEAN 5   /* step_kernel<false, true, 0, 1>: obstacle tracks, C3's configuration */
int gr_step_kernel_variant(const gr_ctx* ctx);

/* Depth camera.  gr_enable_camera validates the cfg and derives its constants (once);
 * gr_bind_camera_buffers binds the image outputs of the next render (rebind per call like
 * gr_bind_buffers).  gr_camera_render forms the image observation of the call just made
 * (gr_step / gr_reset / gr_observe, same gr_buffers binding, same stream): it re-renders the
 * outdated envs (Isaac Lab RayCasterCamera._update_buffers_impl), then writes both obs rows
 * (fresh image noise from the call's observation counter).  Graph-capturable. */
int gr_camera_config_default(gr_camera_config* cfg);
size_t gr_camera_config_size(void);
int gr_enable_camera(gr_ctx* ctx, const gr_camera_config* cfg);
int gr_bind_camera_buffers(gr_ctx* ctx, const gr_camera_buffers* bufs);
int gr_camera_render(gr_ctx* ctx, int mode, const uint8_t* mask, void* stream);
/* algorithmic HBM bytes per env of one render call, with and without the re-render */
int gr_camera_bytes_per_env(const gr_ctx* ctx, int64_t* render_bytes, int64_t* reuse_bytes);

/*
 * Rollout inference of the rsl_rl ActorCritic (PPO.act: standalone/rsl_rl/ext/algorithms/ppo.py:71-85
 * -> ActorCritic.act / evaluate / get_actions_log_prob) on MFMA: bf16 operands with fp32 accumulation
 * (GR_POLICY_BF16, gr_policy.hip), or fp32 operands, the reference's precision (GR_POLICY_FP32,
 * v_mfma_f32_16x16x4_f32, gr_policy_f32.hip).
 * Both MLPs (num_obs -> H -> H -> num_out, H = 128 or 256, LeakyReLU(0.01) or ELU) for all envs in
 * one graph-capturable launch; the actor also samples Normal(mean, std) (Philox, keyed by env and
 * `counter`) and sums the log prob over the actions.  GR_POLICY_BF16: weights packed by the caller into
 * the kernel's fragment order (generalizableracing_amd/rsl_rl/fused_inference.py).  GR_POLICY_FP32: the
 * module's own row-major fp32 weights W1 [H][num_obs], W2 [H][H], W3 [num_out][H] (16-byte aligned).
 * Both precisions draw the same Normal noise for the same (seed, env, counter).  Context-free.
 */
#define GR_POLICY_BF16 0
#define GR_POLICY_FP32 1
#define GR_POLICY_ACT_LRELU 0
#define GR_POLICY_ACT_ELU 1
/* With GR_POLICY_ACT_LRELU, W1, b1, W2 and b2 are packed multiplied by this factor ((1 + 0.01) / 2): the
 * kernel forms LeakyReLU(y) from v = 0.505 y as v + (0.99 / 1.01) |v| (one fused multiply-add).  W3, b3
 * are not scaled. */
#define GR_POLICY_LRELU_PRESCALE 0.505f
typedef struct gr_policy_net {
  const float* obs; /* [num_envs][num_obs] fp32, 16-byte aligned, num_obs <= 32 and a multiple of 4 */
  const void* w1;   /* bf16 fragments [H/16][64][8] (GR_POLICY_FP32: fp32 [H][num_obs], likewise below) */
  const float* b1;  /* [H] */
  const void* w2;   /* bf16 fragments [H/16][H/32][64][8] */
  const float* b2;  /* [H] */
  const void* w3;   /* bf16 fragments [H/32][64][8] (rows >= num_out zero) */
  const float* b3;  /* [num_out] */
  float* out;       /* actor: action mean [num_envs][num_out]; critic: value [num_envs] */
  int32_t num_obs, num_out, reserved[2];
} gr_policy_net;
typedef struct gr_policy_args {
  gr_policy_net net[2]; /* 0: actor (num_out = num_actions <= 4), 1: critic (num_out = 1); net[1].obs == NULL:
                           actor only (no value; the actor's workgroups take every CU) */
  const float* std;     /* [num_actions] the policy's std */
  float* actions;       /* [num_envs][num_actions] sampled actions */
  float* log_prob;      /* [num_envs] */
  uint32_t* counters;   /* [2] sampling call counter, double-buffered like gr_buffers.counters: this */
  int32_t counter_index; /* call reads counters[i] and writes counters[i ^ 1] = counters[i] + 1 */
  int32_t num_envs, hidden, activation, env_id_offset;
  uint32_t seed_lo, seed_hi;
  int32_t precision; /* GR_POLICY_BF16 or GR_POLICY_FP32 */
  int32_t reserved;
} gr_policy_args;
int gr_policy_forward(const gr_policy_args* args, void* stream);
/* sizeof(gr_policy_args): the binding checks its mirror against it at load time */
size_t gr_policy_args_size(void);

/*
 * Training-mode BatchNorm fused with its activation, on channels-last rows x [m][c] (fp32, 16-byte aligned,
 * c in {4, 8, 16, 32, 64}): the Conv -> BatchNorm2d -> LeakyReLU / ELU blocks of the vision stem
 * (standalone/rsl_rl/ext/modules/vision_actor_critic.py:43-144 as patch GEMMs, rsl_rl/vision_actor_critic.py),
 * replacing torch's batch_norm (stats + transform) + activation passes and their backward (gr_bn.hip).
 *   forward:  y = act((x - mean) * invstd * w + b) with the batch statistics; stats [4][c] = mean, invstd,
 *             biased var, unbiased var (the caller updates the running statistics from them);
 *   backward: gx, gw, gb from gy and x (the activation's derivative is recomputed).
 * act: GR_POLICY_ACT_LRELU (negative slope `slope`) or GR_POLICY_ACT_ELU (alpha 1).  `part` is a device
 * workspace of gr_bn_scratch_doubles(m, c) doubles.  Deterministic (fixed-order fp64 channel sums).
 */
int64_t gr_bn_scratch_doubles(int64_t m, int32_t c);
int gr_bn_act_forward(const float* x, int64_t m, int32_t c, const float* w, const float* b, float eps, int32_t act,
                      float slope, float* y, float* stats, double* part, void* stream);
int gr_bn_act_backward(const float* x, const float* gy, int64_t m, int32_t c, const float* w, const float* b,
                       const float* stats, int32_t act, float slope, float* gx, float* gw, float* gb, double* part,
                       void* stream);
/* The running-statistics update of `uses` training-mode forwards over the same rows from a forward's stats [4][c]
 * (nn.BatchNorm2d / F.batch_norm with a momentum, torch/nn/modules/batchnorm.py; the reference's stem BatchNorms,
 * vision_actor_critic.py:93-105): per forward running = running * keep + momentum * batch stat (mean; unbiased
 * variance), keep = 1 - momentum as fp32; then num_batches += count (num_batches may be NULL when count is 0). */
int gr_bn_running_update(float* running_mean, float* running_var, int64_t* num_batches, const float* stats, int32_t c,
                         float keep, float momentum, int32_t uses, int32_t count, void* stream);

/*
 * The vision stem's first block from the depth image itself: Conv2d(1, c, 3, stride 3, no bias) -> BatchNorm2d
 * (training mode) -> act, for `nimg` images at obs + b * ld + off (fp32 pixels), or at obs + rows[b] * ld + off
 * when `rows` is not NULL (a mini-batch read through its permutation instead of a gathered copy; the caller
 * guarantees every rows[b] indexes a row of obs — the library cannot see the source's extent).  Output rows follow
 * VisionActorCritic.stem_gemm: nimg x na rows whose 3x3 cells are pix[0 .. na) (int16 pixel offsets, 9 per
 * row), then nimg x nb rows from pix[na .. na + nb); y [rows][c].  The patch matrix and the conv output are
 * never written (recomputed per pass); the backward returns the conv weight's gradient [c][9] and the BN
 * affine gradients (the image needs none).  Only the first y_rows rows of y are stored and only the first
 * gy_rows of gy are read (ABI 3): the table-b rows (cells no later conv reads) still enter the BN statistics,
 * their gradient is zero, so y [y_rows][c] can be exactly the next layer's input and no zero-padded gradient is
 * ever built.  c in {4, 8, 16, 32, 64}, na + nb <= 1024; `part`: a workspace of
 * gr_stem1_scratch_doubles(nimg, na + nb, c) doubles; stats as gr_bn_act_forward.
 */
int64_t gr_stem1_scratch_doubles(int32_t nimg, int32_t rows_per_img, int32_t c);
int gr_stem1_forward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                     int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b, float eps,
                     int32_t act, float slope, float* y, int64_t y_rows, float* stats, double* part, void* stream);
int gr_stem1_backward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                      int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                      const float* stats, int32_t act, float slope, const float* gy, int64_t gy_rows, float* g_conv_w,
                      float* g_bn_w, float* g_bn_b, double* part, void* stream);
/* Tall-skinny patch GEMM: C[m][n] = A[m][k] B[k][n] (fp32; A rows `lda` floats apart, 4-byte aligned; C rows `ldc`
 * apart), B small and held in registers: with b_nk B = b^T for b [n][k] (a Conv2d / Linear forward, x W^T), else B = b
 * [k][n] (its input gradient, gy W).  The vision stem's conv3 forward (k 128, n 64, b_nk), its input gradient (k 64,
 * n 128) and the final Linear's input gradient (k 192, n a multiple of 64 up to 4096)
 * (standalone/rsl_rl/ext/modules/vision_actor_critic.py:93-105 as patch GEMMs).  Each output one fixed-order
 * fp32 MFMA chain over k. */
int gr_tsgemm(const float* a, int64_t lda, const float* b, int32_t b_nk, float* c, int64_t ldc, int64_t m, int32_t k,
              int32_t n, void* stream);
/* The same GEMMs with a BatchNorm + activation applied to A as it is loaded: A = act(bn(z)) with the batch statistics
 * `stats` [4][bn_c] (gr_bn_stats / gr_bn_act_forward's), affine bn_w / bn_b, act GR_POLICY_ACT_LRELU (slope) or ELU;
 * column k of z is channel k % bn_c (bn_c 32 for gr_tsgemm_bnact).  The vision stem's block 2 feeds conv3 this way (vision_actor_critic.py:93-105:
 * BatchNorm2d(32) -> LeakyReLU -> Conv2d(32, 64, 2, 2)): act(bn(z2)) is never written.  gr_tsgemm_bnact: conv3's
 * forward (k 128, n 64, b = W3 [64][128]); gr_patch_wgrad_bnact: its weight gradient gy^T act(bn(z)) (n a multiple
 * of 64, bn_c a multiple of 8 dividing 128).  Values bit-identical to the materialised act(bn(z)) (gr_bn_act_forward's
 * arithmetic). */
int gr_tsgemm_bnact(const float* z, int64_t lda, const float* b, float* c, int64_t ldc, int64_t m, int32_t k, int32_t n,
                    int32_t bn_c, const float* stats, const float* bn_w, const float* bn_b, int32_t act, float slope,
                    void* stream);
int gr_patch_wgrad_bnact(const float* z, int64_t ld, const float* gy, int64_t m, int32_t n, int32_t k, float* part,
                         float* gw, int32_t bn_c, const float* stats, const float* bn_w, const float* bn_b, int32_t act,
                         float slope, void* stream);
/* A training-mode BatchNorm's batch statistics alone (gr_bn_act_forward's stats pass): stats [4][c] = mean, invstd,
 * biased var, unbiased var of x [m][c]; `part` as gr_bn_act_forward's. */
int gr_bn_stats(const float* x, int64_t m, int32_t c, float eps, float* stats, double* part, void* stream);
/* Weight gradient of a tall patch GEMM: gw[n][k] = gy[m][n]^T x[m][k] (fp32; gy row-major, 16-byte aligned; x rows
 * `ld` floats apart, 4-byte aligned), the vision stem's conv2 (n 32, k 144), conv3 (n 64, k 128) and final Linear
 * (n 192, k 1280) weight gradients (standalone/rsl_rl/ext/modules/vision_actor_critic.py:93-105; torch's
 * Conv2d / Linear backward).  Covered: n 32 with k 128 or 144; n a multiple of 64 up to 256 with k a multiple of
 * 128 up to 4096.
 * Deterministic (fixed-order sums, no atomics).  `part`: a workspace of gr_patch_wgrad_floats(m, n, k) floats. */
int64_t gr_patch_wgrad_floats(int64_t m, int32_t n, int32_t k);
int gr_patch_wgrad(const float* x, int64_t ld, const float* gy, int64_t m, int32_t n, int32_t k, float* part,
                   float* gw, void* stream);
/* The first block's forward with the stem's conv2, Conv2d(c = 16, 32, 3, stride 3, no bias), fused into its apply
 * pass: y [nimg * na][16] as gr_stem1_forward stores it (y_rows = nimg * na: the table-a rows) and conv2's output
 * z2 [nimg * n2][32] (na = 9 n2; row 9 p + j of an image = position j of patch p).  w2f: conv2's weight as
 * [9][4][32][4] floats, w2f[((j * 4 + g) * 32 + o) * 4 + v] = W[o][4 g + v][j / 3][j % 3] (16-byte aligned).
 * Same workspace and stats as gr_stem1_forward.  y may be NULL (a forward with no backward: y is only kept for
 * conv2's weight gradient).  moments (64 doubles, 8-byte aligned, may be NULL): the statistics pass's pixel moments
 * over every cell (sums of d = p - p0 and of d d^T, and p0), for gr_stem12_backward_w2. */
int gr_stem12_forward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                      int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b, float eps,
                      int32_t act, float slope, const float* w2f, int32_t n2, float* y, float* z2, float* stats,
                      double* moments, double* part, void* stream);
/* The same backward when the next layer is the stem's conv2, Conv2d(c = 16, 32, 3, stride 3, no bias), on the
 * nimg x na table-a rows grouped as its patches (row 9 p + j of an image = position j of patch p, na = 9 n2): takes
 * conv2's OUTPUT gradient gz2 [nimg * n2][32] (16-byte aligned) and forms conv2's input gradient inside the passes
 * instead of reading a [nimg * na][16] gy (VisionActorCritic stem; reference vision_actor_critic.py:93-105).
 * w2t: conv2's weight as [9][4][16][8] floats, w2t[((j * 4 + g) * 16 + ch) * 8 + s] = W[o = 8 g + s][ch][j / 3][j % 3]
 * (16-byte aligned).  conv2's own weight gradient is not computed here.  Same workspace as gr_stem1_backward. */
int gr_stem12_backward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                       int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                       const float* stats, int32_t act, float slope, const float* gz2, int32_t n2, const float* w2t,
                       float* g_conv_w, float* g_bn_w, float* g_bn_b, double* part, void* stream);
/* gr_stem12_backward plus conv2's own weight gradient g_w2 [32][144] (columns (j, ch), w2's layout in
 * VisionActorCritic's patch GEMM): y1 = act(bn(conv1)) is recomputed from the image (bit-identical to the forward's),
 * so gr_stem12_forward may be called with y = NULL.  n2 <= 80 (72 x 96 images: 80).  Workspace:
 * gr_stem12_backward_w2_scratch_doubles(nimg) doubles.  Deterministic (fixed-order sums).  Replaces the pair
 * gr_stem12_backward + gr_patch_wgrad(gz2, y1) of the reference's conv2 backward (vision_actor_critic.py:93-105).
 * moments: the same forward's (gr_stem12_forward), or NULL: with them the conv1 weight gradient's sums of the pixels
 * and of xhat x pixels come from the moments in fp64 and the pass skips those products. */
int64_t gr_stem12_backward_w2_scratch_doubles(int32_t nimg);
int gr_stem12_backward_w2(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix,
                          int32_t na, int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                          const float* stats, const double* moments, int32_t act, float slope, const float* gz2,
                          int32_t n2, const float* w2t, float* g_conv_w, float* g_bn_w, float* g_bn_b, float* g_w2,
                          double* part, void* stream);

/* Device status: the GR_STATUS_* bits the kernels of this context raised since the last clear (0: none).
 * Synchronises `stream` (the stream the steps ran on); clear != 0 resets the word.  A raised bit means the
 * outputs of some step since the last check are not trustworthy. */
#define GR_STATUS_OBST_WAIT_TIMEOUT 1u /* a physics wave gave up waiting for its obstacle mask (stale mask used) */
int gr_device_status(gr_ctx* ctx, uint32_t* status, int clear, void* stream);
/* Fault injection for the status path's tests (0: none, production). */
#define GR_FAULT_NONE 0
#define GR_FAULT_OBST_NO_SIGNAL 1 /* the policy waves never signal the obstacle mask */
int gr_test_inject_fault(gr_ctx* ctx, int fault);
/* Obstacle slots per camera wave (tests: the path for obstacles beyond the slots; 0: the launch's own choice,
 * 40-64 by the LDS; 1-64: that many). */
int gr_test_camera_slots(gr_ctx* ctx, int32_t slots);

/* Column sums of a row-major [rows][cols] matrix (fp32 or bf16 elements), fp32 out: the bias gradients of
 * the PPO update's tall mini-batches (standalone/rsl_rl/ext/algorithms/ppo.py:168-190 -> loss.backward()
 * through nn.Linear; generalizableracing_amd/rsl_rl/linear.py bias_grad).  Two launches on `stream`, fixed
 * summation order, no atomics; `partial` is caller-owned scratch of gr_column_sum_partials(rows) * cols
 * floats.  Context-free and graph-capturable. */
int gr_column_sum_partials(int64_t rows);
int gr_column_sum(const void* x, int dtype, int64_t rows, int32_t cols, float* partial, float* out, void* stream);

/* The memory-bound layers of the actor's / critic's MLP for the PPO update's tall mini-batches
 * (standalone/rsl_rl/ext/algorithms/ppo.py:103-190: update() -> policy.act / evaluate through upstream rsl_rl
 * ActorCritic's MLP x -> Linear(d, h1) -> LeakyReLU -> Linear(h1, h2) -> LeakyReLU -> Linear(h2, k), and
 * loss.backward() through it; generalizableracing_amd/rsl_rl/linear.py MLP).  The h1 x h2 GEMM stays on
 * hipBLASLt; these do everything around it, each matrix read once.  Row-major fp32, 16-byte aligned matrices,
 * widths multiples of 4; slope is LeakyReLU's.  Context-free, on `stream`, graph-capturable, no atomics, fixed
 * summation order; `partial` is caller-owned scratch of the *_partials(...) floats.
 *   gr_mlp_in_forward : y [rows][h] = lrelu(x w^T + b); x [rows][ldx] (first d <= 32 columns), w [h][d], h <= 256
 *   gr_mlp_in_backward: with gz = gh * lrelu'(hv) (hv = the forward's y): sums [h d + h] = [gz^T x | sum gz]
 *   gr_head_forward   : y [rows][k] = lrelu(z) w^T + b;  z [rows][h], w [k][h], b [k], k <= 8, h <= 256
 *   gr_head_backward  : gz [rows][h] = (gy w) * lrelu'(z); sums [k h + k + h] = [gy^T lrelu(z) | sum gy | sum gz] */
int64_t gr_head_partials(int64_t rows, int32_t k, int32_t h);
int gr_head_forward(const float* z, int64_t rows, int32_t h, const float* w, const float* b, int32_t k, float slope,
                    float* y, void* stream);
int gr_head_backward(const float* z, const float* gy, int64_t rows, int32_t h, const float* w, int32_t k, float slope,
                     float* gz, float* partial, float* sums, void* stream);
int64_t gr_mlp_in_partials(int64_t rows, int32_t d, int32_t h);
int gr_mlp_in_forward(const float* x, int64_t rows, int32_t d, int32_t ldx, const float* w, const float* b, int32_t h,
                      float slope, float* y, void* stream);
int gr_mlp_in_backward(const float* gh, const float* hv, const float* x, int64_t rows, int32_t d, int32_t ldx,
                       int32_t h, float slope, float* partial, float* sums, void* stream);

/* The actor and critic MLPs of the PPO update as whole-network fp32-MFMA kernels (round 4): the mini-batch's
 * forward and backward through x -> Linear(d, H) -> LeakyReLU -> Linear(H, H) -> LeakyReLU -> Linear(H, k) of both
 * networks (upstream rsl_rl ActorCritic's MLPs as PPO.update runs them, standalone/rsl_rl/ext/algorithms/ppo.py:
 * 103-190; loss.backward() through them), fp32 operands on v_mfma_f32_16x16x4_f32, one launch per direction for
 * both networks (blockIdx.y = network) plus the weight gradient of the hidden layer and one fixed-order reduction:
 *   gr_mlp_forward : y = MLP(x); saves h1 = lrelu(x W1^T + b1) and z2 = h1 W2^T + b2 for the backward
 *   gr_mlp_backward: from gy [rows][k]: gz2 = (gy W3) * lrelu'(z2), gh1 = gz2 W2, gz1 = gh1 * lrelu'(h1);
 *                    gW3 = gy^T lrelu(z2), gb3 = sum gy, gb2 = sum gz2, gW2 = gz2^T h1, gW1 = gz1^T x, gb1 = sum gz1
 * H = 128 or 256, d <= 32 (a multiple of 4), k <= 4.  Row-major fp32, 16-byte aligned; the x rows may be strided
 * (ldx floats: the update's packed mini-batch).  Context-free, graph-capturable, no atomics, fixed summation order;
 * `partial` is caller-owned scratch of gr_mlp_partials(rows, H, nets) floats.
 * Size limit: rows * max(H, ldx) < GR_MLP_MAX_ELEMS (2^31; the kernels use 32-bit offsets), else GR_ERR_ARG. */
#define GR_MLP_MAX_ELEMS 2147483647LL
typedef struct gr_mlp_net {
  const float* x;    /* [rows][ldx]: the first d columns are the input */
  const float* w1;   /* [H][d] */
  const float* b1;   /* [H] */
  const float* w2;   /* [H][H] */
  const float* b2;   /* [H] */
  const float* w3;   /* [k][H] */
  const float* b3;   /* [k] */
  float* h1;         /* [rows][H]: forward output (saved), backward input */
  float* z2;         /* [rows][H]: forward output (saved), backward input */
  float* y;          /* [rows][k]: forward output */
  const float* gy;   /* [rows][k]: backward input */
  float* gz2;        /* [rows][H]: backward scratch (the hidden layer's output gradient) */
  float* grads;      /* backward output [H d | H | H H | H | k H | k] = gW1, gb1, gW2, gb2, gW3, gb3 */
  int64_t ldx;
  int32_t d, k;
  /* optional, 16-byte aligned, gr_mlp_h1mask_words(rows, H) words: the sign of h1 as bits, written by the forward
   * when non-null; given to the backward (H = 256) it replaces the h1 rows there (mlp_bwd256h: 1/32 of their bytes,
   * two workgroups per CU).  NULL in the backward: the h1 rows are read (mlp_bwd256 / mlp_bwd). */
  uint64_t* h1mask;
} gr_mlp_net;
int64_t gr_mlp_h1mask_words(int64_t rows, int32_t hidden);
typedef struct gr_mlp_args {
  gr_mlp_net net[2];
  int64_t rows;
  int32_t nets;   /* 1 or 2 */
  int32_t hidden; /* H */
  float slope;    /* LeakyReLU negative slope */
  int32_t reserved;
  float* partial; /* scratch */
} gr_mlp_args;
int64_t gr_mlp_partials(int64_t rows, int32_t hidden, int32_t nets);
int gr_mlp_forward(const gr_mlp_args* args, void* stream);
int gr_mlp_backward(const gr_mlp_args* args, void* stream);
size_t gr_mlp_args_size(void);

/* The PPO losses of one mini-batch, forward and backward (standalone/rsl_rl/ext/algorithms/ppo.py:133-169: the
 * adaptive-rate KL, the clipped surrogate, the (clipped) value loss; the Gaussian log prob of rsl_rl's
 * ActorCritic with a state-independent std).  Row-strided fp32 inputs (ld_* in floats; the mini-batch's packed
 * rows), k <= 8 actions, one thread per sample, fixed summation order, context-free and graph-capturable.
 *   gr_ppo_loss_forward : sums [3] = [sum max(surrogate, clipped), sum value term, sum KL]  (means: / rows)
 *   gr_ppo_loss_backward: g [2] = upstream gradients of the surrogate and value means (device scalars);
 *                         dmu [rows][k], dvalue [rows], dstd [k] (summed over the rows)
 * `partial` is caller-owned scratch of gr_ppo_loss_partials(rows) floats. */
typedef struct {
  int64_t rows;
  int32_t k;
  int32_t clipped_value; /* use_clipped_value_loss */
  float clip;            /* clip_param */
  const float* mu;       /* [rows] x ld_mu: the policy's action mean (the graph's output) */
  const float* std;      /* [k]: the policy's action std */
  const float* value;    /* the critic's value */
  const float* act;      /* the stored actions */
  const float* logp_old; /* the stored log probs */
  const float* adv;
  const float* value_old; /* the stored values (target_values_batch) */
  const float* ret;
  const float* mu_old;
  const float* sig_old;
  int64_t ld_mu, ld_value, ld_act, ld_logp_old, ld_adv, ld_value_old, ld_ret, ld_mu_old, ld_sig_old;
} gr_ppo_loss_args;
int64_t gr_ppo_loss_partials(int64_t rows);
int gr_ppo_loss_forward(const gr_ppo_loss_args* args, float* partial, float* sums, void* stream);
int gr_ppo_loss_backward(const gr_ppo_loss_args* args, const float* g, float* dmu, float* dvalue, float* partial,
                         float* dstd, void* stream);
/* The same with the means and the combined loss finished on the device (rsl_rl/fused_loss.py; ppo.py:171-172
 * `loss = surrogate_loss + value_loss_coef * value_loss`): gr_ppo_loss_forward_loss writes sums [3], loss [1] =
 * sums[0] / rows + value_coef * (sums[1] / rows), stats [3] = the three means; acc [2] (may be null) += (surrogate,
 * value) means; kl_out [1] (may be null) = the KL mean.  gr_ppo_loss_backward_loss takes the loss's upstream
 * gradient g_loss [1]: the value mean's is value_coef * g_loss[0], as torch's MulBackward gives it. */
int gr_ppo_loss_forward_loss(const gr_ppo_loss_args* args, float* partial, float* sums, float value_coef, float* loss,
                             float* stats, float* acc, float* kl_out, void* stream);
int gr_ppo_loss_backward_loss(const gr_ppo_loss_args* args, const float* g_loss, float value_coef, float* dmu,
                              float* dvalue, float* partial, float* dstd, void* stream);
/* gr_ppo_loss_forward_loss + gr_ppo_loss_backward_loss in one pass over the rows (+ one final reduction), for a caller
 * that knows the upstream gradient's device address before the backward runs (the graph-captured update's persistent
 * seed, generalizableracing_amd/rsl_rl/fused_loss.py): the per-row gradients dmu / dvalue and dstd come out of the
 * forward pass, bit-identical to the two-pass form.  partial / dpartial: two distinct gr_ppo_loss_partials(rows)
 * buffers. */
int gr_ppo_loss_forward_backward(const gr_ppo_loss_args* args, const float* g_loss, float value_coef, float* partial,
                                 float* sums, float* loss, float* stats, float* acc, float* kl_out, float* dmu,
                                 float* dvalue, float* dpartial, float* dstd, void* stream);
/* The graph-captured update's adaptive learning-rate rule (ppo.py:133-150, device form): lr[0] = max(lr_min,
 * lr / 1.5) if kl[0] > 2 desired_kl; min(lr_max, lr * 1.5) if desired_kl / 2 > kl[0] > 0; else unchanged (fp32
 * arithmetic, the thresholds rounded to fp32 as torch's scalar comparisons do). */
int gr_adaptive_lr(const float* kl, float* lr, double desired_kl, double lr_min, double lr_max, void* stream);

/* Adam and the gradient-norm clip of the PPO update (standalone/rsl_rl/ext/algorithms/ppo.py:179-181:
 * nn.utils.clip_grad_norm_(max_grad_norm) then torch.optim.Adam.step) over a table of parameter segments
 * (generalizableracing_amd/rsl_rl/flat_adam.py).  The table lives in DEVICE memory (the kernels read it, so a
 * launch's arguments stay small); gr_adam_prepare checks a host copy of it and numbers its blocks (1024 elements
 * each, GR_ADAM_BLOCK) before the caller uploads it.  step[step_slot] is a segment's Adam step count (fp32,
 * device; one slot per segment); lr_ptr (device) overrides lr when not null (the graph-captured update's rate
 * tensor).  Context-free, graph-capturable, on `stream`.
 *   gr_adam_prepare: fills block_start, *nblocks = the launch's blocks (the size of `part`); GR_ERR_ARG if a
 *                    pointer is null, a size not positive, a slot negative or shared, or nseg outside 1..64
 *   gr_adam_clip:    grads *= min(1, max_norm / (||all grads|| + 1e-6)); norm_out[0] = the norm (may be null);
 *                    the norm in double, per block then in one fixed order (deterministic)
 *   gr_adam_step:    step[slot] += 1 per segment (and its coefficients into coef), then the Adam update of every
 *                    element.  Matches torch's foreach Adam (torch/optim/adam.py _multi_tensor_adam,
 *                    non-capturable): m.lerp_(g, 1 - b1); v = v * b2 + (1 - b2) * g * g; step_size = lr / (1 - b1^t)
 *                    and sqrt(1 - b2^t) in double, rounded to fp32; p += -step_size * m / (sqrt(v) / bc2_sqrt + eps) */
#define GR_ADAM_MAX_SEGMENTS 64
#define GR_ADAM_BLOCK 1024
typedef struct {
  float* param;
  float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  int32_t step_slot;
  int32_t block_start; /* gr_adam_prepare */
} gr_adam_segment;
typedef struct {
  int32_t nseg;
  int32_t nblocks;          /* gr_adam_prepare */
  double lr, beta1, beta2;  /* host doubles as in torch's foreach Adam (bias corrections in double) */
  float eps;
  int32_t pad;
  const float* lr_ptr;
  float* step;                 /* [slots] */
  float* coef;                 /* [slots][2] scratch: lr / (1 - b1^t), sqrt(1 - b2^t) */
  double* part;                /* [nblocks] scratch of the clip */
  const gr_adam_segment* seg;  /* device table [nseg] */
} gr_adam_args;
int gr_adam_prepare(gr_adam_segment* table, int32_t nseg, int32_t* nblocks);
int gr_adam_clip(const gr_adam_args* args, float max_norm, float* norm_out, void* stream);
int gr_adam_step(const gr_adam_args* args, void* stream);
/* gr_adaptive_lr (when kl is not null; lr must then be args->lr_ptr) + gr_adam_clip + gr_adam_step in two launches
 * instead of five, the same arithmetic (the graph-captured update's segment B, generalizableracing_amd/rsl_rl/ppo.py
 * _GraphedStep): the rate rule and the step counts ride in the launch of the per-block norms, the clip coefficient,
 * the bias corrections and the clipped gradient (still written back) in the Adam pass. */
int gr_adam_clip_step(const gr_adam_args* args, float max_norm, float* norm_out, const float* kl, float* lr,
                      double desired_kl, double lr_min, double lr_max, void* stream);

/* The rollout loop's per-step bookkeeping (generalizableracing_amd/rsl_rl/rollout_ops.py), one launch each, the
 * torch ops' arithmetic in their order (bit-identical stored rollouts).  Context-free, graph-capturable.
 *   gr_store_transition: PPO.process_env_step + RolloutStorage.add_transitions (standalone/rsl_rl/ext/algorithms/
 *       ppo.py:83-95, rsl_rl rollout_storage.py:74-98) for everything but the observations: out_reward = r +
 *       gamma * (v * time_out) (time_out null: r), out_dones = dones != 0, and the action / value / log prob /
 *       mean / std rows.  Inputs are row-strided (ld_* in floats; 0 repeats row 0, e.g. the expanded std); the
 *       outputs are the storage slot's contiguous [n, k] / [n] rows.  k <= 8; dones_bytes 1 (bool, uint8), 4 or 8.
 *   gr_episode_accumulate: the runner's episode sums (standalone/rsl_rl/ext/runners/on_policy_runner.py:167-173):
 *       cur_rew += reward, cur_len += 1; fin_rew / fin_len = those sums and fin_done = dones != 0 (the finished
 *       episodes go to the deques from there); cur_* of done envs zeroed.
 *   gr_gae: RolloutStorage.compute_returns (rollout_storage.py:113-127) over [t_steps][n] planes (rewards, dones
 *       as bytes, values), last_values row-strided by ld_last; writes returns and advantages = returns - values. */
typedef struct {
  int64_t n;
  int32_t k;
  int32_t dones_bytes;
  float gamma;
  int32_t pad;
  const float* reward;
  const void* dones;
  const uint8_t* time_out; /* null: no bootstrap */
  const float* value;
  const float* action;
  const float* logp;
  const float* mu;
  const float* sigma;
  int64_t ld_value, ld_action, ld_logp, ld_mu, ld_sigma;
  float* out_reward;
  uint8_t* out_dones;
  float* out_action;
  float* out_value;
  float* out_logp;
  float* out_mu;
  float* out_sigma;
} gr_transition_args;
int gr_store_transition(const gr_transition_args* args, void* stream);
int gr_episode_accumulate(int64_t n, const float* reward, const void* dones, int32_t dones_bytes, float* cur_rew,
                          float* cur_len, float* fin_rew, float* fin_len, uint8_t* fin_done, void* stream);
/* PPOL2C2's mixed observations (standalone/rsl_rl/ext/algorithms/ppo_l2c2.py:179-180, `obs + w * (next - obs)`):
 * out [rows][cols] = obs + w[row] * (next_obs - obs), the torch expression's three fp32 roundings, one pass; contiguous
 * rows, cols a multiple of 4, 16-byte aligned. */
int gr_l2c2_mix(const float* obs, const float* next_obs, const float* w, int64_t rows, int32_t cols, float* out,
                void* stream);
/* The same with the pair read through row indices: out[r] = obs[rows_obs[r]] + w[r] (next_obs[rows_next[r]] -
 * obs[rows_obs[r]]), source rows `ld` floats apart (a multiple of 4): the mini-batch's rows straight from the rollout
 * storage (rollout_storage_l2c2.py:131-167 gathers them first); the caller guarantees the indices are in range. */
int gr_l2c2_mix_rows(const float* obs, const float* next_obs, int64_t ld, const int64_t* rows_obs,
                     const int64_t* rows_next, const float* w, int64_t rows, int32_t cols, float* out, void* stream);
int gr_gae(int64_t n, int32_t t_steps, float gamma, float lam, const float* rewards, const uint8_t* dones,
           const float* values, const float* last_values, int64_t ld_last, float* returns, float* advantages,
           void* stream);

/* In-library HIP-event timing of the fused step kernel alone (not the log
 * finalize): when enabled, gr_step brackets the env kernel with a pair of
 * events on the caller's stream (ring of 4096 pairs; do not capture into a
 * graph while enabled).  gr_read_timing synchronises, sums the elapsed times
 * of the recorded launches and clears the ring. */
int gr_set_timing(gr_ctx* ctx, int enable);
int gr_read_timing(gr_ctx* ctx, double* total_ms, int64_t* launches);

/* Standalone controller + integrator on n envs, for parity against the
 * reference's DroneDynamics / CTBRController golden vectors.
 *   state_in/out [n][13] p(3) q(4) v_w(3) w_b(3)  (DroneDynamics keeps w in the body frame)
 *   ang_acc_b [n][3] controller D-term input
 *   cmd [n][4] scaled CTBR command (mode 0) or (thrust, torque) (mode 1)
 *   ctrl_in/out [n][4] CTBR filter state (T, tau)
 *   par [n][16] = PAR0..PAR3 planes of one env (Kp3 cT Kd3 m_plant ctau3 m_ctrl J3 pad)
 *   drag [n][6] k2(3) k1(3)
 *   extra_out [n][13] = DD.step linear acceleration a(3), angular acceleration alpha(3), w_world(3),
 *                       then mode 0: the controller's output [T, tau] (post motor model when enabled,
 *                       controller_diff.py:137-144); mode 2: the realised rotor thrusts
 *   mode: 0 CTBR controller then integrator ; 1 integrator only (cmd = [T, tau]) ;
 *         2 ThrustController.update alone (cmd = desired rotor thrusts, thrust_controller_diff.py:182-186;
 *           motor speeds start at 0; the integrator runs with a zero wrench) */
int gr_test_dynamics(gr_ctx* ctx, int n, int mode, const float* state_in, const float* ang_acc_b,
                     const float* cmd, const float* ctrl_in, const float* par, const float* drag,
                     float* state_out, float* ctrl_out, float* extra_out, void* stream);
/* Elementwise portable math on the device (parity of gr_math.h host vs device).
 * fn: 0 exp 1 tanh 2 log 3 sin 4 cos 5 atan2(x, y2) 6 sqrt 7 div(x/y2) */
int gr_test_math(gr_ctx* ctx, int fn, int n, const float* x, const float* y2, float* out, void* stream);
/* Philox words for counters (c0+i, c1, c2, c3), key = ctx seed */
int gr_test_philox(gr_ctx* ctx, int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t* out4,
                   void* stream);
/* Diagnostic builds only (-DGR_STAMPS, scripts/stamps.py): copy the per-wave phase
 * timestamps of the most recent step launch (12 u64 per wave).  Product builds
 * return GR_ERR_STATE. */
int gr_debug_read_stamps(uint64_t* host, int n);
/* The same for the fused policy kernel (16 u64 per wave, gr_policy.hip). */
int gr_debug_read_policy_stamps(uint64_t* host, int n);

#ifdef __cplusplus
}
#endif
#endif /* GR_H */
