// gr_capi.cpp — C ABI of libgr.so (declared in include/gr.h).
//
// Host side only: validates arguments, derives per-config constants once,
// owns the packed copy of the track table, and launches the kernels of
// gr_kernels.hip on the caller's stream.  No allocation, host sync or
// exception crosses gr_step / gr_reset / gr_observe.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/gr.h"
#include "gr_camera.h"
#include "gr_kernels.h"
#include "gr_math.h"

struct gr_ctx {
  gr_config cfg;
  gr_buffers buf;
  bool have_buf = false;
  float* table = nullptr;  // packed [T*L][stride]
  bool have_tracks = false;
  gr_obstacles obst;       // caller-owned device arrays (records null: none)
  gr::KArgs args;
  gr::KConst kc;                   // host copy of the per-context constants
  gr::KConst* kc_dev = nullptr;    // device copy read by the kernels
  std::vector<int> blk_types;      // per workgroup: first | last terrain type << 16
  int* blk_dev = nullptr;
  unsigned* status_dev = nullptr;  // GR_STATUS_* word the kernels OR into
  std::string err;
  // optional depth camera
  bool cam_enabled = false;
  int cam_test_slots = 0;  // gr_test_camera_slots (0: the launch's own choice)
  gr_cam_const cam_k;
  gr_cam_const* cam_dev = nullptr;
  gr_camera_buffers cam_buf;
  bool have_cam_buf = false;
  // optional kernel timing (gr_set_timing)
  std::vector<hipEvent_t> ev;  // [2 * GR_TIMING_RING]
  int ev_next = 0;
  bool timing = false;
  // resident terrain (gr_terrain_reserve / _stage / _commit): the live obstacle block the kernels read and a staging
  // block [gates | tracks | obstacle block | header]; obstacle block (floats) = [records | counts | grid_f | grid_i |
  // cells | items], every part 16-byte aligned
  struct Resident {
    bool on = false, staged = false, span_set = false;
    int32_t cap_obst = 0, cap_cells = 0, cap_items = 0;
    float* stage = nullptr;
    float* live = nullptr;
    size_t off_tracks = 0, off_obst = 0, off_hdr = 0, obst_floats = 0;
    size_t o_cnt = 0, o_gf = 0, o_gi = 0, o_cells = 0, o_items = 0;
    float inv_cell = 0.0f, margin = 0.0f;         // the obstacle grid's (same for every generation)
    float staged_inv_cell = 0.0f, staged_margin = 0.0f;
    int32_t hdr_host[4] = {0, 0, 0, 0};
  } res;
  std::mutex err_mu;  // gr_terrain_stage may fail on another host thread
  int64_t terrain_epoch = 0;  // gr_terrain_reserve calls: each one moves the terrain arrays a graph may have baked in
};

#define GR_TIMING_RING 4096

namespace {

int fail(gr_ctx* c, int code, const std::string& msg) {
  if (c) {
    std::lock_guard<std::mutex> lk(c->err_mu);
    c->err = msg;
  }
  return code;
}
int hip_fail(gr_ctx* c, hipError_t e, const char* what) {
  return fail(c, GR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}
bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// device copy of the constants, made on first device use (gr_create stays host-only)
int ensure_dev(gr_ctx* c, const char* what) {
  if (c->kc_dev) return GR_OK;
  const size_t nbt = c->blk_types.size() * sizeof(int);
  hipError_t e = hipMalloc(&c->kc_dev, sizeof(gr::KConst));
  if (e == hipSuccess) e = hipMalloc(&c->blk_dev, nbt);
  if (e == hipSuccess) e = hipMalloc(&c->status_dev, 16);
  if (e == hipSuccess) e = hipMemset(c->status_dev, 0, 16);
  if (e == hipSuccess) e = hipMemcpy(c->kc_dev, &c->kc, sizeof(gr::KConst), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->blk_dev, c->blk_types.data(), nbt, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    if (c->kc_dev) (void)hipFree(c->kc_dev);
    if (c->blk_dev) (void)hipFree(c->blk_dev);
    if (c->status_dev) (void)hipFree(c->status_dev);
    c->kc_dev = nullptr;
    c->blk_dev = nullptr;
    c->status_dev = nullptr;
    return hip_fail(c, e, what);
  }
  c->args.kc = c->kc_dev;
  c->args.blk_types = c->blk_dev;
  c->args.status = c->status_dev;
  e = gr::allow_large_lds();
  if (e != hipSuccess) return hip_fail(c, e, "hipFuncSetAttribute(MaxDynamicSharedMemorySize)");
  return GR_OK;
}

void derive(gr_ctx* c) {
  const gr_config& g = c->cfg;
  gr::KConst& a = c->kc;
  std::memset(&a, 0, sizeof(a));
  std::memset(&c->args, 0, sizeof(c->args));
  a.cfg = g;
  a.track_stride = g.max_gates * GR_GATE_FLOATS + GR_TRACK_FLOATS;
  // env -> terrain type: IL floor(arange(N) / (N / num_cols)) with an fp32 divisor
  const float s = (float)((double)g.num_envs / (double)g.num_types);
  for (int t = 0; t <= g.num_types; ++t) {
    double lim = (double)t * (double)s;
    int i = (int)std::ceil(lim);
    a.type_start[t] = i > g.num_envs ? g.num_envs : i;
  }
  // gross thrust bounds, controller_diff.py:96-99 (python double, cast at clamp)
  const double k2 = g.thrustmap[0], k1 = g.thrustmap[1], k0 = g.thrustmap[2];
  const double w0 = g.motor_omega[0], w1 = g.motor_omega[1];
  const double tmin = k2 * w0 * w0 + k1 * w0 + k0, tmax = k2 * w1 * w1 + k1 * w1 + k0;
  a.thrust_lo = (float)(tmin * 4.0);
  a.thrust_hi = (float)(tmax * 4.0);
  const double reach = std::sqrt((double)g.collider_half[0] * g.collider_half[0] +
                                 (double)g.collider_half[1] * g.collider_half[1] +
                                 (double)g.collider_half[2] * g.collider_half[2]);
  a.lat_reach = (float)(reach * 1.001 + 1e-5);
  const float w[7] = {g.w_progress, g.w_body_rate, g.w_action_rate, g.w_collision,
                      g.w_perception, g.w_success, g.w_bad_pose};
  for (int k = 0; k < 7; ++k) a.w[k] = w[k];
  // motor model constants (same expressions as the oracle)
  const float l = g.arm_length * 0.707106769f, kap = g.kappa;
  const float sx[4] = {1, -1, -1, 1}, sy[4] = {-1, -1, 1, 1}, sz[4] = {1, -1, 1, -1};
  for (int j = 0; j < 4; ++j) {
    a.B[0][j] = 1.0f; a.B[1][j] = l * sx[j]; a.B[2][j] = l * sy[j]; a.B[3][j] = kap * sz[j];
    a.Bi[j][0] = 0.25f; a.Bi[j][1] = sx[j] / (4.0f * l); a.Bi[j][2] = sy[j] / (4.0f * l);
    a.Bi[j][3] = sz[j] / (4.0f * kap);
  }
  a.motor_fmax = (float)tmax;
  a.motor_c = gr_expf(-(float)(1.0 / (double)g.motor_tau) * g.step_dt);
  a.tm_k2 = (float)k2; a.tm_k1 = (float)k1; a.tm_k0 = (float)k0;
  a.tm_k1sq = (float)(k1 * k1); a.tm_4k2 = (float)(4.0 * k2);
  a.tm_inv2k2 = (float)(1.0 / (2.0 * k2)); a.tm_negk1 = (float)(-k1);
  // per-workgroup terrain-type range; LDS = the widest span of any workgroup, all levels
  int span = 1;
  const int nb = (g.num_envs + GR_BLOCK - 1) / GR_BLOCK;
  c->blk_types.assign(nb, 0);
  for (int b = 0; b < nb; ++b) {
    int f = b * GR_BLOCK, last = std::min(f + GR_BLOCK, g.num_envs) - 1, t0 = 0, t1 = 0;
    for (int t = 1; t < g.num_types; ++t) { t0 += f >= a.type_start[t]; t1 += last >= a.type_start[t]; }
    span = std::max(span, t1 - t0 + 1);
    c->blk_types[b] = t0 | (t1 << 16);
  }
  const long bytes = (long)span * g.num_levels * a.track_stride * 4;
  // table + handovers within the CU's LDS (one workgroup per CU at the bench size); beyond that the
  // (L2-resident) table is read directly
  a.lds_bytes = bytes + GR_XCH_BYTES <= GR_LDS_MAX ? (int)bytes : 0;
  gr::KHot& h = c->args.h;
  h.num_envs = g.num_envs;
  h.num_levels = g.num_levels;
  h.max_gates = g.max_gates;
  h.track_stride = a.track_stride;
  h.env_id_offset = g.env_id_offset;
  h.use_motor_model = g.use_motor_model;
  h.dr_rotor = g.dr_rotor;
  h.integrator = g.integrator;
  h.obs_noise = g.obs_noise;
  h.lds_tab_vec = a.lds_bytes / 16;
  h.seed_lo = g.seed_lo;
  h.seed_hi = g.seed_hi;
  h.obs_lin_vel_noise = g.obs_lin_vel_noise;
  h.obs_att_noise = g.obs_att_noise;
}

}  // namespace

extern "C" {

int gr_abi_version(void) { return GR_ABI_VERSION; }
size_t gr_config_size(void) { return sizeof(gr_config); }
size_t gr_policy_args_size(void) { return sizeof(gr_policy_args); }

int gr_config_default(gr_config* c) {
  if (!c) return GR_ERR_ARG;
  std::memset(c, 0, sizeof(*c));
  c->num_envs = 2048;  // racing_ctbr_env.py:357
  c->seed_lo = 42;
  c->num_types = 20;   // RacingComplexTerrainCfg num_cols (racing_terrains.py:137-147)
  c->num_levels = 10;  // num_rows
  c->max_gates = 8;
  c->max_init_level = 5;
  c->stage = 1;
  c->integrator = GR_INTEGRATOR_DD_EXPLICIT;
  c->decimation = 3;
  c->sim_dt = 0.01f;
  c->step_dt = (float)(0.01 * 3);
  c->episode_length_s = 6.0f;
  c->max_episode_length = (int)std::ceil(6.0 / (0.01 * 3));  // 200 (manager_based_diff_rl_env.py:99-102)
  c->gravity = 9.81f;
  c->mass = 0.6f;  // ASSUMPTION: drone_175_v8.usd (defines the mass) is not in the reference
  c->inertia[0] = 0.0015f; c->inertia[1] = 0.002f; c->inertia[2] = 0.004f;
  c->arm_length = 0.09f;
  c->kappa = 0.016f;
  c->motor_tau = 0.0001f;
  c->motor_omega[0] = 150.0f; c->motor_omega[1] = 3000.0f;
  c->thrustmap[0] = 1.3298253500372892e-06f;
  c->thrustmap[1] = 0.0038360810526746033f;
  c->thrustmap[2] = -1.7689986848125325f;
  c->max_thrust_weight_ratio = 3.0f;
  c->body_rate_bound = 6.0f;
  for (int k = 0; k < 3; ++k) c->rate_gain_p[k] = 35.0f;
  c->rate_gain_d[0] = 0.0005f; c->rate_gain_d[1] = 0.0005f; c->rate_gain_d[2] = 0.0003f;
  c->thrust_ctrl_delay = 0.03f;
  for (int k = 0; k < 3; ++k) c->torque_ctrl_delay[k] = 0.03f;
  c->use_motor_model = 0;
  c->action_lag = 1;
  for (int k = 0; k < 3; ++k) { c->drag1[k] = 0.18f; c->drag2[k] = 0.01f; }
  c->drag1_rand = 0.1f;
  c->drag2_rand = 0.005f;
  c->z_drag = 4.0f;
  c->z_drag_rand = 0.4f;
  c->random_drag = 1;
  c->mass_add_range[0] = -0.02f; c->mass_add_range[1] = 0.02f;
  c->inertia_scale_range[0] = 0.9f; c->inertia_scale_range[1] = 1.1f;
  c->pid_scale_range[0] = 0.9f; c->pid_scale_range[1] = 1.1f;
  c->delay_scale_range[0] = 0.8f; c->delay_scale_range[1] = 1.3f;
  c->dr_startup = 1;
  c->dr_plant = 1;
  c->spawn_pos[2] = 0.5f;  // DRONE_CFG init_state.pos (quadcopter.py:30-31)
  for (int k = 0; k < 3; ++k) c->reset_pos_half[k] = 0.5f;
  c->reset_att_half[0] = 0.2f; c->reset_att_half[1] = 0.2f; c->reset_att_half[2] = 0.7f;
  for (int k = 0; k < 6; ++k) c->reset_vel_half[k] = 0.1f;
  c->gate_threshold = 0.35f;
  for (int k = 0; k < 3; ++k) c->gate_noise_pos[k] = 0.1f;
  c->add_gate_noise = 1;
  c->level_up_threshold = 3;
  c->level_down_threshold = 2;
  c->noise_curriculum = 1;
  c->noise_enhance_threshold = 4;
  c->noise_decay_threshold = 3;
  c->noise_enhance = 0.02f;
  c->noise_decay = 0.03f;
  c->obs_noise = 1;
  c->obs_lin_vel_noise = 0.03f;
  c->obs_att_noise = 0.05f;
  c->w_progress = 1.0f;
  c->w_body_rate = -0.1f;
  c->w_action_rate = -0.05f;
  c->w_collision = -100.0f;
  c->w_perception = 0.1f;
  c->w_success = 20.0f;
  c->w_bad_pose = -30.0f;
  c->collider_half[0] = 0.707f * 0.09f;
  c->collider_half[1] = 0.707f * 0.09f;
  c->collider_half[2] = 0.5f * 0.05f;
  c->collision_count_threshold = 0;
  c->out_of_bound[0] = 0.0f; c->out_of_bound[1] = 10.0f;
  c->term_contact = 1;
  c->term_bad_pose = 1;
  c->dr_rotor = 0;  // config C5 turns it on
  c->rotor_scale_range[0] = 0.9f; c->rotor_scale_range[1] = 1.1f;
  return GR_OK;
}

int gr_create(const gr_config* cfg, gr_ctx** out) {
  if (!cfg || !out) return GR_ERR_ARG;
  *out = nullptr;
  const gr_config& g = *cfg;
  if (g.num_envs <= 0 || g.num_types <= 0 || g.num_types > GR_MAX_TYPES || g.num_levels <= 0 ||
      g.num_levels > 255 || g.max_gates <= 0 || g.max_gates > 255 || g.decimation <= 0 ||
      (g.action_lag != 0 && g.action_lag != 1) || g.max_episode_length <= 0 || !(g.mass > 0.0f) ||
      (g.integrator != GR_INTEGRATOR_DD_EXPLICIT && g.integrator != GR_INTEGRATOR_SEMI_IMPLICIT) ||
      g.max_init_level < 0)  // (fewer envs than terrain columns is valid: IL's floor(i / (N / cols)) skips columns)
    return GR_ERR_ARG;
  gr_ctx* c = new (std::nothrow) gr_ctx();
  if (!c) return GR_ERR_STATE;
  c->cfg = g;
  derive(c);
  *out = c;
  return GR_OK;
}

int gr_destroy(gr_ctx* c) {
  if (!c) return GR_ERR_ARG;
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->table) (void)hipFree(c->table);
  if (c->kc_dev) (void)hipFree(c->kc_dev);
  if (c->blk_dev) (void)hipFree(c->blk_dev);
  if (c->status_dev) (void)hipFree(c->status_dev);
  if (c->cam_dev) (void)hipFree(c->cam_dev);
  if (c->res.stage) (void)hipFree(c->res.stage);
  if (c->res.live) (void)hipFree(c->res.live);
  delete c;
  return GR_OK;
}

const char* gr_last_error(const gr_ctx* c) {
  if (!c) return "null context";
  // a copy per calling thread, taken under the lock: gr_terrain_stage may set the message on the builder thread
  thread_local std::string copy;
  std::lock_guard<std::mutex> lk(const_cast<gr_ctx*>(c)->err_mu);
  copy = c->err;
  return copy.c_str();
}

int64_t gr_terrain_epoch(const gr_ctx* c) { return c ? c->terrain_epoch : GR_ERR_ARG; }

int gr_num_blocks(const gr_ctx* c) { return c ? (c->cfg.num_envs + GR_BLOCK - 1) / GR_BLOCK : GR_ERR_ARG; }
int gr_num_log_rows(const gr_ctx* c) { return c ? gr_num_blocks(c) * GR_LOG_ROWS_PER_BLOCK : GR_ERR_ARG; }

int gr_log_finalize(gr_ctx* c, const float* rows, const float* prev, float* out, void* stream) {
  if (!c || !rows || !out) return GR_ERR_ARG;
  hipError_t e = gr::launch_log_finalize(rows, gr_num_log_rows(c), prev, out, c->cfg.episode_length_s,
                                         (float)c->cfg.num_envs, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_log_finalize");
}

int gr_bytes_per_env_step(const gr_ctx* c, int64_t* rd, int64_t* wr) {
  if (!c || !rd || !wr) return GR_ERR_ARG;
  // the obstacle hint plane (obstacle tracks) is read and written like a motor plane
  const int motor = (c->cfg.use_motor_model ? 1 : 0) + (c->obst.records ? 1 : 0);
  // read: planes POSQ..PAR3 (14 x 16 B) [+ MOTOR] [+ ROTOR], int plane 16 B, action 16 B
  *rd = (14 + motor + (c->cfg.dr_rotor ? 1 : 0)) * 16 + 16 + 16;
  // written: POSQ..LAG, EP0, EP1 (8 x 16 B) [+ MOTOR], int plane, obs policy+critic (2 x 64 B),
  // aux 4, reward 4, terminated 1, time_out 1, dones 8.  RST0/RST1 (only on reset) not counted.
  *wr = (8 + motor) * 16 + 16 + 128 + 4 + 4 + 1 + 1 + 8;
  // the observation sink, when bound: policy + critic rows again (2 x 16 values)
  if (c->args.sink_policy) *wr += 2 * 16 * (c->args.sink_dtype == GR_DTYPE_BF16 ? 2 : 4);
  return GR_OK;
}

// track records [ntr][GR_TRACK_FLOATS] (host copy): finite heights, 2 <= gates <= max_gates, start gate in range
static int check_track_records(gr_ctx* c, const float* h, const char* who) {
  const gr_config& g = c->cfg;
  const int ntr = g.num_types * g.num_levels;
  for (int t = 0; t < ntr; ++t) {
    const float* r = &h[(size_t)t * GR_TRACK_FLOATS];
    const int start = (int)r[2], ng = (int)r[3];
    if (!(std::isfinite(r[0]) && std::isfinite(r[1])) || ng < 2 || ng > g.max_gates || start < 0 || start >= ng ||
        (float)start != r[2] || (float)ng != r[3])
      return fail(c, GR_ERR_ARG, std::string(who) + ": invalid track record " + std::to_string(t));
  }
  return GR_OK;
}

// pack the device gate table + track records into the context's table (stream-ordered; allocated once)
static int pack_tracks(gr_ctx* c, const float* gates, const float* tracks, hipStream_t s, const char* who) {
  const gr_config& g = c->cfg;
  const int ntr = g.num_types * g.num_levels;
  const size_t stride = (size_t)c->kc.track_stride;
  hipError_t e = hipSuccess;
  if (!c->table) {
    e = hipMalloc(&c->table, (size_t)ntr * stride * sizeof(float));
    if (e != hipSuccess) return hip_fail(c, e, "hipMalloc (track table)");
  }
  const size_t gb = (size_t)g.max_gates * GR_GATE_FLOATS * sizeof(float);
  e = hipMemcpy2DAsync(c->table, stride * sizeof(float), gates, gb, gb, ntr, hipMemcpyDeviceToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpy2DAsync(c->table + (size_t)g.max_gates * GR_GATE_FLOATS, stride * sizeof(float), tracks,
                         GR_TRACK_FLOATS * sizeof(float), GR_TRACK_FLOATS * sizeof(float), ntr,
                         hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return hip_fail(c, e, who);
  c->args.table = c->table;
  c->have_tracks = true;
  return GR_OK;
}

int gr_bind_tracks(gr_ctx* c, const float* gates, const float* tracks) {
  if (!c || !gates || !tracks) return fail(c, GR_ERR_ARG, "gr_bind_tracks: null pointer");
  const int ntr = c->cfg.num_types * c->cfg.num_levels;
  std::vector<float> h((size_t)ntr * GR_TRACK_FLOATS);
  hipError_t e = hipMemcpy(h.data(), tracks, h.size() * sizeof(float), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(c, e, "gr_bind_tracks: copy track records");
  int rc = check_track_records(c, h.data(), "gr_bind_tracks");
  if (rc != GR_OK) return rc;
  rc = pack_tracks(c, gates, tracks, nullptr, "gr_bind_tracks: pack");
  if (rc != GR_OK) return rc;
  e = hipDeviceSynchronize();
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_bind_tracks: sync");
}

// obstacle index arrays (host copies: counts [ntr], grid_f / grid_i [ntr][4], cells [num_cells][2]) against the sizes
static int check_obstacles(gr_ctx* c, const gr_obstacles* o, const int32_t* cnt, const float* gf, const int32_t* gi,
                           const int32_t* cells, const char* who) {
  const int ntr = c->cfg.num_types * c->cfg.num_levels;
  for (int t = 0; t < ntr; ++t) {
    const int nx = gi[4 * t], ny = gi[4 * t + 1], first = gi[4 * t + 2];
    if (cnt[t] < 0 || cnt[t] > o->max_obstacles || nx < 0 || ny < 0 || first < 0 ||
        (long)first + (long)nx * ny > o->num_cells)
      return fail(c, GR_ERR_ARG, std::string(who) + ": invalid count / grid of track " + std::to_string(t));
  }
  for (int k = 0; k < o->num_cells; ++k)
    if (cells[2 * k] < 0 || cells[2 * k + 1] < 0 || (long)cells[2 * k] + cells[2 * k + 1] > o->num_items)
      return fail(c, GR_ERR_ARG, std::string(who) + ": cell " + std::to_string(k) + " out of the item range");
  // one cell size and margin for all tracks (the per-env hints carry only the grown cell's corner)
  for (int t = 0; t < ntr; ++t)
    if (!(gf[4 * t + 2] > 0.0f) || !(gf[4 * t + 3] >= 0.0f) || gf[4 * t + 2] != gf[2] || gf[4 * t + 3] != gf[3])
      return fail(c, GR_ERR_ARG, std::string(who) + ": every track needs the same 1/cell > 0 and margin >= 0");
  return GR_OK;
}

static int check_obstacle_arrays(gr_ctx* c, const gr_obstacles* o, const char* who) {
  if (!o->records || !o->counts || !o->grid_f || !o->grid_i || !o->cells || !o->items || o->max_obstacles <= 0 ||
      o->num_cells <= 0 || o->num_items <= 0)
    return fail(c, GR_ERR_ARG, std::string(who) + ": null array or empty size");
  if (!aligned16(o->records) || !aligned16(o->grid_f) || !aligned16(o->grid_i) || !aligned16(o->items) ||
      (reinterpret_cast<uintptr_t>(o->cells) & 7u))
    return fail(c, GR_ERR_ARG, std::string(who) + ": records / grids / items must be 16-byte aligned, cells 8-byte");
  return GR_OK;
}

static void unbind_obstacles(gr_ctx* c) {
  std::memset(&c->obst, 0, sizeof(c->obst));
  c->args.obst_grid_f = nullptr;
  c->args.obst_grid_i = nullptr;
  c->args.obst_cells = nullptr;
  c->args.obst_items = nullptr;
}

// bind validated obstacle arrays and clear the per-env hints (they refer to the previous table) on stream s
static int attach_obstacles(gr_ctx* c, const gr_obstacles* o, float inv_cell, float margin_cells, hipStream_t s,
                            const char* who) {
  const float cell = 1.0f / inv_cell, margin = margin_cells * cell;
  c->args.h.obst_span = cell + 2.0f * margin;
  if (c->have_buf) {
    hipError_t e = hipMemsetAsync(c->buf.state + (size_t)GR_P_OHINT * c->cfg.num_envs * 4, 0,
                                  (size_t)c->cfg.num_envs * 16, s);
    if (e != hipSuccess) return hip_fail(c, e, who);
  }
  c->obst = *o;
  c->args.obst_grid_f = reinterpret_cast<const float4*>(o->grid_f);
  c->args.obst_grid_i = reinterpret_cast<const int4*>(o->grid_i);
  c->args.obst_cells = reinterpret_cast<const int2*>(o->cells);
  c->args.obst_items = reinterpret_cast<const float4*>(o->items);
  return GR_OK;
}

int gr_bind_obstacles(gr_ctx* c, const gr_obstacles* o) {
  if (!c) return GR_ERR_ARG;
  if (!o) {
    unbind_obstacles(c);
    return GR_OK;
  }
  int rc = check_obstacle_arrays(c, o, "gr_bind_obstacles");
  if (rc != GR_OK) return rc;
  const int ntr = c->cfg.num_types * c->cfg.num_levels;
  std::vector<int32_t> cnt(ntr), gi((size_t)ntr * 4), cells((size_t)o->num_cells * 2);
  std::vector<float> gf((size_t)ntr * 4);
  hipError_t e = hipMemcpy(cnt.data(), o->counts, cnt.size() * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(gf.data(), o->grid_f, gf.size() * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(gi.data(), o->grid_i, gi.size() * 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(cells.data(), o->cells, cells.size() * 4, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(c, e, "gr_bind_obstacles: copy index arrays");
  rc = check_obstacles(c, o, cnt.data(), gf.data(), gi.data(), cells.data(), "gr_bind_obstacles");
  if (rc != GR_OK) return rc;
  rc = attach_obstacles(c, o, gf[2], gf[3], nullptr, "gr_bind_obstacles: clear hints");
  if (rc != GR_OK) return rc;
  e = hipDeviceSynchronize();
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_bind_obstacles: sync");
}

int gr_swap_terrain(gr_ctx* c, const float* gates, const float* tracks, const float* tracks_host,
                    const gr_obstacles* obst, const gr_obstacles* obst_host, void* stream) {
  if (!c || !gates || !tracks || !tracks_host) return fail(c, GR_ERR_ARG, "gr_swap_terrain: null pointer");
  int rc = check_track_records(c, tracks_host, "gr_swap_terrain");
  if (rc != GR_OK) return rc;
  if (obst) {
    if (!obst_host || !obst_host->counts || !obst_host->grid_f || !obst_host->grid_i || !obst_host->cells)
      return fail(c, GR_ERR_ARG, "gr_swap_terrain: obstacles need their host index arrays");
    rc = check_obstacle_arrays(c, obst, "gr_swap_terrain");
    if (rc != GR_OK) return rc;
    if (obst_host->num_cells != obst->num_cells || obst_host->num_items != obst->num_items ||
        obst_host->max_obstacles != obst->max_obstacles)
      return fail(c, GR_ERR_ARG, "gr_swap_terrain: host and device obstacle sizes differ");
    rc = check_obstacles(c, obst, obst_host->counts, obst_host->grid_f, obst_host->grid_i, obst_host->cells,
                         "gr_swap_terrain");
    if (rc != GR_OK) return rc;
  }
  const hipStream_t s = (hipStream_t)stream;
  rc = pack_tracks(c, gates, tracks, s, "gr_swap_terrain: pack");
  if (rc != GR_OK) return rc;
  if (!obst) {
    unbind_obstacles(c);
    return GR_OK;
  }
  return attach_obstacles(c, obst, obst_host->grid_f[2], obst_host->grid_f[3], s, "gr_swap_terrain: clear hints");
}

static size_t up4(size_t n) { return (n + 3) & ~(size_t)3; }

// the resident live arrays as the kernels' terrain (reserve; again at every commit, after any gr_bind_* call)
static void bind_resident(gr_ctx* c) {
  gr_ctx::Resident& r = c->res;
  c->args.table = c->table;
  if (!r.live) {
    unbind_obstacles(c);
    return;
  }
  gr_obstacles o;
  o.records = r.live;
  o.counts = reinterpret_cast<const int32_t*>(r.live + r.o_cnt);
  o.grid_f = r.live + r.o_gf;
  o.grid_i = reinterpret_cast<const int32_t*>(r.live + r.o_gi);
  o.cells = reinterpret_cast<const int32_t*>(r.live + r.o_cells);
  o.items = r.live + r.o_items;
  o.max_obstacles = r.cap_obst;
  o.num_cells = r.cap_cells;
  o.num_items = r.cap_items;
  o.reserved = 0;
  c->obst = o;
  c->args.obst_grid_f = reinterpret_cast<const float4*>(o.grid_f);
  c->args.obst_grid_i = reinterpret_cast<const int4*>(o.grid_i);
  c->args.obst_cells = reinterpret_cast<const int2*>(o.cells);
  c->args.obst_items = reinterpret_cast<const float4*>(o.items);
}

int gr_terrain_reserve(gr_ctx* c, int32_t max_obstacles, int32_t max_cells, int32_t max_items) {
  if (!c) return GR_ERR_ARG;
  if (max_obstacles < 0 || (max_obstacles > 0 && (max_cells <= 0 || max_items <= 0)))
    return fail(c, GR_ERR_ARG, "gr_terrain_reserve: capacities");
  int rc = ensure_dev(c, "gr_terrain_reserve");
  if (rc != GR_OK) return rc;
  const gr_config& g = c->cfg;
  const size_t ntr = (size_t)g.num_types * g.num_levels;
  hipError_t e = hipDeviceSynchronize();  // (a reallocation: nothing may still read the old arrays)
  if (e != hipSuccess) return hip_fail(c, e, "gr_terrain_reserve: sync");
  gr_ctx::Resident& r = c->res;
  if (r.stage) (void)hipFree(r.stage);
  if (r.live) (void)hipFree(r.live);
  r = gr_ctx::Resident();
  r.cap_obst = max_obstacles;
  r.cap_cells = max_obstacles > 0 ? max_cells : 0;
  r.cap_items = max_obstacles > 0 ? max_items : 0;
  if (max_obstacles > 0) {
    r.o_cnt = ntr * (size_t)max_obstacles * GR_OBST_FLOATS;
    r.o_gf = r.o_cnt + up4(ntr);
    r.o_gi = r.o_gf + 4 * ntr;
    r.o_cells = r.o_gi + 4 * ntr;
    r.o_items = r.o_cells + up4(2 * (size_t)max_cells);
    r.obst_floats = r.o_items + (size_t)max_items * GR_OBST_FLOATS;
  }
  r.off_tracks = ntr * (size_t)g.max_gates * GR_GATE_FLOATS;
  r.off_obst = r.off_tracks + ntr * GR_TRACK_FLOATS;
  r.off_hdr = r.off_obst + r.obst_floats;
  e = hipMalloc(&r.stage, (r.off_hdr + 4) * sizeof(float));
  if (e == hipSuccess && r.obst_floats) e = hipMalloc(&r.live, r.obst_floats * sizeof(float));
  if (e == hipSuccess && !c->table) e = hipMalloc(&c->table, ntr * (size_t)c->kc.track_stride * sizeof(float));
  if (e != hipSuccess) {
    if (r.stage) (void)hipFree(r.stage);
    if (r.live) (void)hipFree(r.live);
    r = gr_ctx::Resident();
    return hip_fail(c, e, "gr_terrain_reserve: hipMalloc");
  }
  r.on = true;
  ++c->terrain_epoch;
  bind_resident(c);  // (the contents arrive with the first commit)
  c->have_tracks = false;  // until the first commit
  return GR_OK;
}

int gr_terrain_stage(gr_ctx* c, const float* gates_h, const float* tracks_h, const gr_obstacles* o, void* stream) {
  if (!c || !gates_h || !tracks_h) return fail(c, GR_ERR_ARG, "gr_terrain_stage: null pointer");
  gr_ctx::Resident& r = c->res;
  if (!r.on) return fail(c, GR_ERR_STATE, "gr_terrain_stage: gr_terrain_reserve first");
  if ((o != nullptr) != (r.cap_obst > 0))
    return fail(c, GR_ERR_ARG, "gr_terrain_stage: obstacles given iff reserved with obstacles");
  int rc = check_track_records(c, tracks_h, "gr_terrain_stage");
  if (rc != GR_OK) return rc;
  const gr_config& g = c->cfg;
  const size_t ntr = (size_t)g.num_types * g.num_levels;
  if (o) {
    if (!o->records || !o->counts || !o->grid_f || !o->grid_i || !o->cells || !o->items || o->max_obstacles <= 0 ||
        o->num_cells <= 0 || o->num_items <= 0)
      return fail(c, GR_ERR_ARG, "gr_terrain_stage: null obstacle array or empty size");
    if (o->max_obstacles > r.cap_obst || o->num_cells > r.cap_cells || o->num_items > r.cap_items)
      return fail(c, GR_ERR_CAPACITY, "gr_terrain_stage: the generation (" + std::to_string(o->max_obstacles) +
                                          " obstacles per track, " + std::to_string(o->num_cells) + " cells, " +
                                          std::to_string(o->num_items) + " items) exceeds the reservation");
    rc = check_obstacles(c, o, o->counts, o->grid_f, o->grid_i, o->cells, "gr_terrain_stage");
    if (rc != GR_OK) return rc;
    if (r.span_set && (o->grid_f[2] != r.inv_cell || o->grid_f[3] != r.margin))
      return fail(c, GR_ERR_ARG, "gr_terrain_stage: the obstacle grid's cell / margin changed between generations");
  }
  const hipStream_t s = (hipStream_t)stream;
  float* st = r.stage;
  hipError_t e = hipMemcpyAsync(st, gates_h, r.off_tracks * sizeof(float), hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = hipMemcpyAsync(st + r.off_tracks, tracks_h, ntr * GR_TRACK_FLOATS * sizeof(float), hipMemcpyHostToDevice, s);
  if (o) {
    float* ob = st + r.off_obst;
    const size_t rec_b = (size_t)o->max_obstacles * GR_OBST_FLOATS * sizeof(float);
    if (e == hipSuccess)
      e = hipMemcpy2DAsync(ob, (size_t)r.cap_obst * GR_OBST_FLOATS * sizeof(float), o->records, rec_b, rec_b, ntr,
                           hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(ob + r.o_cnt, o->counts, ntr * 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(ob + r.o_gf, o->grid_f, ntr * 16, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(ob + r.o_gi, o->grid_i, ntr * 16, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(ob + r.o_cells, o->cells, (size_t)o->num_cells * 8, hipMemcpyHostToDevice, s);
    if (e == hipSuccess)
      e = hipMemcpyAsync(ob + r.o_items, o->items, (size_t)o->num_items * GR_OBST_FLOATS * sizeof(float),
                         hipMemcpyHostToDevice, s);
    // header: float4s of the obstacle block the commit copies (through the last staged item)
    r.hdr_host[0] = (int32_t)((r.o_items + (size_t)o->num_items * GR_OBST_FLOATS) / 4);
    if (e == hipSuccess) e = hipMemcpyAsync(st + r.off_hdr, r.hdr_host, 16, hipMemcpyHostToDevice, s);
    r.staged_inv_cell = o->grid_f[2];
    r.staged_margin = o->grid_f[3];
  }
  if (e != hipSuccess) return hip_fail(c, e, "gr_terrain_stage: upload");
  r.staged = true;
  return GR_OK;
}

int gr_terrain_commit(gr_ctx* c, void* stream) {
  if (!c) return GR_ERR_ARG;
  gr_ctx::Resident& r = c->res;
  if (!r.on || !r.staged) return fail(c, GR_ERR_STATE, "gr_terrain_commit: nothing staged");
  const gr_config& g = c->cfg;
  gr::TerrainCommitArgs a;
  std::memset(&a, 0, sizeof(a));
  a.s_gates = reinterpret_cast<const float4*>(r.stage);
  a.s_tracks = reinterpret_cast<const float4*>(r.stage + r.off_tracks);
  a.table = reinterpret_cast<float4*>(c->table);
  a.ntr = g.num_types * g.num_levels;
  a.g4 = g.max_gates * GR_GATE_FLOATS / 4;
  a.stride4 = c->kc.track_stride / 4;
  if (r.live) {
    a.s_obst = reinterpret_cast<const float4*>(r.stage + r.off_obst);
    a.l_obst = reinterpret_cast<float4*>(r.live);
    a.hdr = reinterpret_cast<const int*>(r.stage + r.off_hdr);
    a.max_obst4 = (long long)(r.obst_floats / 4);
    if (c->have_buf) {
      a.hints = reinterpret_cast<float4*>(c->buf.state) + (size_t)GR_P_OHINT * g.num_envs;
      a.n_hints = g.num_envs;
    }
  }
  hipError_t e = gr::launch_terrain_commit(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "gr_terrain_commit");
  if (r.live) {
    r.inv_cell = r.staged_inv_cell;
    r.margin = r.staged_margin;
    r.span_set = true;
    const float cell = 1.0f / r.inv_cell;
    c->args.h.obst_span = cell + 2.0f * (r.margin * cell);
  }
  bind_resident(c);
  c->have_tracks = true;
  return GR_OK;
}

int gr_bind_buffers(gr_ctx* c, const gr_buffers* b) {
  if (!c || !b) return fail(c, GR_ERR_ARG, "gr_bind_buffers: null pointer");
  const void* ptrs[] = {b->state,      b->istate,          b->obs_policy,   b->obs_critic,    b->obs_aux,
                        b->reward,     b->terminated,      b->time_out,     b->dones,         b->prev_obs_critic,
                        b->prev_obs_aux, b->prev_time_out, b->log_partial,  b->counters};
  if (b->counter_index != 0 && b->counter_index != 1)
    return fail(c, GR_ERR_ARG, "gr_bind_buffers: counter_index must be 0 or 1");
  if (!aligned16(b->log_partial)) return fail(c, GR_ERR_ARG, "gr_bind_buffers: log_partial must be 16-byte aligned");
  for (const void* p : ptrs)
    if (!p) return fail(c, GR_ERR_ARG, "gr_bind_buffers: null buffer");
  if (!aligned16(b->state) || !aligned16(b->istate) || !aligned16(b->obs_policy) || !aligned16(b->obs_critic) ||
      !aligned16(b->prev_obs_critic))
    return fail(c, GR_ERR_ARG, "gr_bind_buffers: state/obs buffers must be 16-byte aligned");
  c->buf = *b;
  c->args.buf = *b;
  c->have_buf = true;
  return GR_OK;
}

int gr_bind_obs_sink(gr_ctx* c, void* policy, void* critic, int dtype) {
  if (!c) return GR_ERR_ARG;
  if (!policy) {  // unbind
    c->args.sink_policy = c->args.sink_critic = nullptr;
    c->args.sink_dtype = GR_DTYPE_F32;
    return GR_OK;
  }
  if (!critic) return fail(c, GR_ERR_ARG, "gr_bind_obs_sink: critic sink is null");
  if (dtype != GR_DTYPE_F32 && dtype != GR_DTYPE_BF16) return fail(c, GR_ERR_ARG, "gr_bind_obs_sink: dtype");
  if (!aligned16(policy) || !aligned16(critic))
    return fail(c, GR_ERR_ARG, "gr_bind_obs_sink: sinks must be 16-byte aligned");
  c->args.sink_policy = policy;
  c->args.sink_critic = critic;
  c->args.sink_dtype = dtype;
  return GR_OK;
}

static int ready(gr_ctx* c, const char* what) {
  if (!c) return GR_ERR_ARG;
  if (!c->have_buf || !c->have_tracks)
    return fail(c, GR_ERR_STATE, std::string(what) + ": buffers and tracks must be bound first");
  return ensure_dev(c, what);
}

int gr_init(gr_ctx* c, void* stream) {
  int r = ready(c, "gr_init");
  if (r) return r;
  hipError_t e = gr::launch_init(c->args, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "gr_init");
  e = hipMemsetAsync(c->buf.counters, 0, 2 * sizeof(uint32_t), (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "gr_init: counters");
  return GR_OK;
}

int gr_reset(gr_ctx* c, const uint8_t* mask, void* stream) {
  int r = ready(c, "gr_reset");
  if (r) return r;
  hipError_t e = gr::launch_env(gr::KMODE_RESET, c->args, nullptr, mask, (hipStream_t)stream, nullptr, nullptr);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_reset");
}

int gr_step(gr_ctx* c, const float* actions, void* stream) {
  int r = ready(c, "gr_step");
  if (r) return r;
  if (!actions || !aligned16(actions)) return fail(c, GR_ERR_ARG, "gr_step: actions must be a 16-byte aligned [N][4] fp32 buffer");
  hipEvent_t t0 = nullptr, t1 = nullptr;
  if (c->timing && c->ev_next < GR_TIMING_RING) {
    t0 = c->ev[2 * c->ev_next];
    t1 = c->ev[2 * c->ev_next + 1];
    c->ev_next++;
  }
  hipError_t e = gr::launch_env(gr::KMODE_STEP, c->args, actions, nullptr, (hipStream_t)stream, t0, t1);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_step");
}

int gr_step_kernel_variant(const gr_ctx* c) { return c ? gr::step_variant(c->args) : GR_ERR_ARG; }

int gr_device_status(gr_ctx* c, uint32_t* status, int clear, void* stream) {
  if (!c || !status) return fail(c, GR_ERR_ARG, "gr_device_status: null argument");
  *status = 0;
  if (!c->status_dev) return GR_OK;  // no kernel has run
  hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned host = 0;
  hipError_t e = hipMemcpyAsync(&host, c->status_dev, sizeof(unsigned), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess && clear) e = hipMemsetAsync(c->status_dev, 0, sizeof(unsigned), s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(c, e, "gr_device_status");
  *status = host;
  return GR_OK;
}

int gr_test_inject_fault(gr_ctx* c, int fault) {
  if (!c) return GR_ERR_ARG;
  if (fault != GR_FAULT_NONE && fault != GR_FAULT_OBST_NO_SIGNAL)
    return fail(c, GR_ERR_ARG, "gr_test_inject_fault: unknown fault");
  c->args.h.test_fault = fault;
  return GR_OK;
}

int gr_test_camera_slots(gr_ctx* c, int32_t slots) {
  if (!c) return GR_ERR_ARG;
  if (slots < 0 || slots > GR_CAM_OBST_SLOTS_MAX) return fail(c, GR_ERR_ARG, "gr_test_camera_slots: slots in [0, 64]");
  c->cam_test_slots = slots;
  return GR_OK;
}

int gr_set_timing(gr_ctx* c, int enable) {
  if (!c) return GR_ERR_ARG;
  if (enable && c->ev.empty()) {
    c->ev.resize(2 * GR_TIMING_RING, nullptr);
    for (auto& e : c->ev) {
      hipError_t r = hipEventCreate(&e);
      if (r != hipSuccess) return hip_fail(c, r, "gr_set_timing: hipEventCreate");
    }
  }
  c->timing = enable != 0;
  c->ev_next = 0;
  return GR_OK;
}

int gr_read_timing(gr_ctx* c, double* total_ms, int64_t* launches) {
  if (!c || !total_ms || !launches) return GR_ERR_ARG;
  double tot = 0.0;
  for (int i = 0; i < c->ev_next; ++i) {
    hipError_t r = hipEventSynchronize(c->ev[2 * i + 1]);
    if (r != hipSuccess) return hip_fail(c, r, "gr_read_timing: sync");
    float ms = 0.0f;
    r = hipEventElapsedTime(&ms, c->ev[2 * i], c->ev[2 * i + 1]);
    if (r != hipSuccess) return hip_fail(c, r, "gr_read_timing: elapsed");
    tot += ms;
  }
  *total_ms = tot;
  *launches = c->ev_next;
  c->ev_next = 0;
  return GR_OK;
}

int gr_observe(gr_ctx* c, void* stream) {
  int r = ready(c, "gr_observe");
  if (r) return r;
  hipError_t e = gr::launch_env(gr::KMODE_OBSERVE, c->args, nullptr, nullptr, (hipStream_t)stream, nullptr, nullptr);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_observe");
}

int gr_camera_config_default(gr_camera_config* k) {
  if (!k) return GR_ERR_ARG;
  std::memset(k, 0, sizeof(*k));
  // racing_ctbr_env.py:77-95 (the intrinsics are python doubles there)
  k->width = 96;
  k->height = 72;
  k->fx = (float)(388.963 / (640.0 / 96.0));
  k->cx = (float)(317.04 / (640.0 / 96.0));
  k->fy = (float)(388.963 / (480.0 / 72.0));
  k->cy = (float)(241.99 / (480.0 / 72.0));
  k->offset_pos[0] = 0.01f;
  k->offset_rot[0] = 0.991f;
  k->offset_rot[2] = -0.131f;
  k->max_distance = 10.0f;
  k->update_period = 0.04f;  // racing_ctbr_env.py:390-391
  k->noise_std = 0.02f;      // observation.py:84-85
  k->add_noise = 1;
  k->obs_scale = 10.0f;      // observation.py:88-92
  return GR_OK;
}

size_t gr_camera_config_size(void) { return sizeof(gr_camera_config); }

int gr_enable_camera(gr_ctx* c, const gr_camera_config* k) {
  if (!c || !k) return fail(c, GR_ERR_ARG, "gr_enable_camera: null pointer");
  const float* r = k->offset_rot;
  const float qn = r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3];
  if (k->width <= 0 || k->width > GR_CAM_MAX_W || k->width % 4 != 0 || k->height <= 0 || k->height > GR_CAM_MAX_H)
    return fail(c, GR_ERR_ARG, "gr_enable_camera: width must be a multiple of 4 in [4, 256], height in [1, 256]");
  if (!(k->fx > 0.0f) || !(k->fy > 0.0f) || !std::isfinite(k->cx) || !std::isfinite(k->cy) || !(qn > 0.0f) ||
      !(k->max_distance > 0.0f) || !(k->obs_scale > 0.0f) || !(k->update_period >= 0.0f) || !(k->noise_std >= 0.0f))
    return fail(c, GR_ERR_ARG, "gr_enable_camera: invalid intrinsics / offset / range / noise");
  if (c->cfg.max_gates > GR_CAM_MAX_GATES)
    return fail(c, GR_ERR_ARG, "gr_enable_camera: max_gates > 64 (one lane per gate)");
  gr_cam_derive(k, c->cfg.step_dt, &c->cam_k);
  if (c->cam_dev) {
    (void)hipFree(c->cam_dev);
    c->cam_dev = nullptr;
  }
  c->cam_enabled = true;
  return GR_OK;
}

int gr_bind_camera_buffers(gr_ctx* c, const gr_camera_buffers* b) {
  if (!c || !b) return fail(c, GR_ERR_ARG, "gr_bind_camera_buffers: null pointer");
  if (!b->depth || !b->age || !b->obs_policy || !b->obs_critic)
    return fail(c, GR_ERR_ARG, "gr_bind_camera_buffers: null buffer");
  if (!aligned16(b->depth) || !aligned16(b->obs_policy) || !aligned16(b->obs_critic) ||
      (reinterpret_cast<uintptr_t>(b->age) & 3u))
    return fail(c, GR_ERR_ARG, "gr_bind_camera_buffers: depth / obs rows must be 16-byte aligned");
  c->cam_buf = *b;
  c->have_cam_buf = true;
  return GR_OK;
}

int gr_camera_render(gr_ctx* c, int mode, const uint8_t* mask, void* stream) {
  int r = ready(c, "gr_camera_render");
  if (r) return r;
  if (!c->cam_enabled || !c->have_cam_buf)
    return fail(c, GR_ERR_STATE, "gr_camera_render: gr_enable_camera and gr_bind_camera_buffers first");
  if (mode != GR_CAM_STEP && mode != GR_CAM_RESET && mode != GR_CAM_OBSERVE)
    return fail(c, GR_ERR_ARG, "gr_camera_render: unknown mode");
  if (!c->cam_dev) {
    hipError_t e = hipMalloc(&c->cam_dev, sizeof(gr_cam_const));
    if (e == hipSuccess) e = hipMemcpy(c->cam_dev, &c->cam_k, sizeof(gr_cam_const), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(c, e, "gr_camera_render: camera constants");
  }
  gr::CamArgs a;
  std::memset(&a, 0, sizeof(a));
  a.cc = c->cam_dev;
  a.state = c->buf.state;
  a.istate = c->buf.istate;
  a.obs_p16 = c->buf.obs_policy;
  a.obs_c16 = c->buf.obs_critic;
  a.terminated = c->buf.terminated;
  a.time_out = c->buf.time_out;
  a.mask = mode == GR_CAM_RESET ? mask : nullptr;
  a.counters = c->buf.counters;
  a.counter_index = c->buf.counter_index;
  a.table = c->table;
  a.obst = c->obst.records;
  a.obst_counts = c->obst.counts;
  a.max_obst = c->obst.records ? c->obst.max_obstacles : 0;
  a.track_stride = c->kc.track_stride;
  a.num_levels = c->cfg.num_levels;
  a.max_gates = c->cfg.max_gates;
  a.num_envs = c->cfg.num_envs;
  a.env_id_offset = c->cfg.env_id_offset;
  a.mode = mode;
  a.width = c->cam_k.width;
  a.height = c->cam_k.height;
  a.seed_lo = c->cfg.seed_lo;
  a.seed_hi = c->cfg.seed_hi;
  a.depth = c->cam_buf.depth;
  a.age = c->cam_buf.age;
  a.out_p = c->cam_buf.obs_policy;
  a.out_c = c->cam_buf.obs_critic;
  a.obst_slots = c->cam_test_slots;
  hipError_t e = gr::launch_camera(a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_camera_render");
}

int gr_camera_bytes_per_env(const gr_ctx* c, int64_t* render_bytes, int64_t* reuse_bytes) {
  if (!c || !render_bytes || !reuse_bytes) return GR_ERR_ARG;
  if (!c->cam_enabled) return GR_ERR_STATE;
  const int64_t img = (int64_t)c->cam_k.npix * 4, rows = 2 * (16 * 4 + img);
  // both: state obs read (2 x 64), obs rows written, flags (2), age read + write (8)
  const int64_t common = 2 * 64 + rows + 2 + 8;
  *render_bytes = common + img + 2 * 16 + 16;  // depth written; pose planes + istate read
  *reuse_bytes = common + img;                 // depth read
  return GR_OK;
}

int gr_policy_forward(const gr_policy_args* a, void* stream) {
  if (!a || a->num_envs <= 0 || (a->hidden != 128 && a->hidden != 256) ||
      (a->activation != GR_POLICY_ACT_LRELU && a->activation != GR_POLICY_ACT_ELU) ||
      (a->precision != GR_POLICY_BF16 && a->precision != GR_POLICY_FP32))
    return GR_ERR_ARG;
  // net[1].obs == NULL: actor only (rollouts without a value estimate: play, the env-only rate)
  const int nets = a->net[1].obs ? 2 : 1;
  for (int k = 0; k < nets; ++k) {
    const gr_policy_net& n = a->net[k];
    if (!n.obs || !n.w1 || !n.b1 || !n.w2 || !n.b2 || !n.w3 || !n.b3 || !n.out || n.num_obs <= 0 || n.num_obs > 32 ||
        n.num_obs % 4 != 0 || !aligned16(n.obs) ||
        n.num_out <= 0 || n.num_out > 4 || (k == 1 && n.num_out != 1))
      return GR_ERR_ARG;
    if (!aligned16(n.w1) || !aligned16(n.w2) || !aligned16(n.w3)) return GR_ERR_ARG;
  }
  if (!a->std || !a->actions || !a->log_prob || !a->counters || (a->counter_index != 0 && a->counter_index != 1))
    return GR_ERR_ARG;
  const hipError_t e = a->precision == GR_POLICY_FP32 ? gr::launch_policy_f32(*a, (hipStream_t)stream)
                                                       : gr::launch_policy(*a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

static bool bn_shape_ok(int64_t m, int32_t c) { return m >= 1 && (c == 4 || c == 8 || c == 16 || c == 32 || c == 64); }

int64_t gr_bn_scratch_doubles(int64_t m, int32_t c) {
  return bn_shape_ok(m, c) ? (int64_t)gr::bn_scratch_doubles(m, c) : (int64_t)GR_ERR_ARG;
}

int gr_bn_act_forward(const float* x, int64_t m, int32_t c, const float* w, const float* b, float eps, int32_t act,
                      float slope, float* y, float* stats, double* part, void* stream) {
  if (!bn_shape_ok(m, c) || !x || !w || !b || !y || !stats || !part || !aligned16(x) || !aligned16(y) ||
      !aligned16(w) || !aligned16(b) || !aligned16(stats) || (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU))
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_bn_forward(x, m, c, w, b, eps, act, slope, y, stats, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_bn_running_update(float* running_mean, float* running_var, int64_t* num_batches, const float* stats, int32_t c,
                         float keep, float momentum, int32_t uses, int32_t count, void* stream) {
  if (!running_mean || !running_var || !stats || c < 1 || c > 4096 || uses < 1 || count < 0 || (count && !num_batches))
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_bn_running_update(running_mean, running_var, reinterpret_cast<long long*>(num_batches),
                                                    stats, c, keep, momentum, uses, count, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_bn_act_backward(const float* x, const float* gy, int64_t m, int32_t c, const float* w, const float* b,
                       const float* stats, int32_t act, float slope, float* gx, float* gw, float* gb, double* part,
                       void* stream) {
  if (!bn_shape_ok(m, c) || !x || !gy || !w || !b || !stats || !gx || !gw || !gb || !part || !aligned16(x) ||
      !aligned16(gy) || !aligned16(gx) || !aligned16(w) || !aligned16(b) || !aligned16(stats) ||
      (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU))
    return GR_ERR_ARG;
  const hipError_t e =
      gr::launch_bn_backward(x, gy, m, c, w, b, stats, act, slope, gx, gw, gb, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

static bool stem1_args_ok(const float* obs, int32_t nimg, const int16_t* pix, int32_t na, int32_t nb,
                          const float* conv_w, int32_t c, const float* bn_w, const float* bn_b) {
  return obs && pix && conv_w && bn_w && bn_b && nimg >= 1 && na >= 1 && nb >= 0 && na + nb <= 1024 &&
         (int64_t)nimg * (na + nb) < (int64_t)1 << 31 && bn_shape_ok(1, c) && aligned16(bn_w) && aligned16(bn_b);
}
static gr::Stem1 stem1_of(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                          int32_t nb, const float* conv_w, int32_t c, int64_t rows_out) {
  gr::Stem1 s;
  s.obs = obs; s.ld = ld; s.off = off; s.nimg = nimg; s.na = na; s.nbt = nb;
  s.rows = reinterpret_cast<const long long*>(rows);
  s.pix = reinterpret_cast<const short*>(pix); s.w = conv_w; s.c = c; s.rows_out = rows_out;
  return s;
}
static bool stem1_rows_ok(int32_t nimg, int32_t na, int32_t nb, int64_t rows_out) {
  return rows_out >= 1 && rows_out <= (int64_t)nimg * (na + nb);
}

int64_t gr_stem1_scratch_doubles(int32_t nimg, int32_t rows_per_img, int32_t c) {
  if (nimg < 1 || rows_per_img < 1 || !bn_shape_ok(1, c)) return GR_ERR_ARG;
  return gr::stem1_scratch_doubles(nimg, rows_per_img, c);
}

int gr_stem1_forward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                     int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b, float eps,
                     int32_t act, float slope, float* y, int64_t y_rows, float* stats, double* part, void* stream) {
  if (!stem1_args_ok(obs, nimg, pix, na, nb, conv_w, c, bn_w, bn_b) || !y || !stats || !part || !aligned16(y) ||
      !aligned16(stats) || (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU) ||
      !stem1_rows_ok(nimg, na, nb, y_rows))
    return GR_ERR_ARG;
  const gr::Stem1 s = stem1_of(obs, ld, off, rows, nimg, pix, na, nb, conv_w, c, y_rows);
  const hipError_t e = gr::launch_stem1_forward(s, bn_w, bn_b, eps, act, slope, y, stats, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_stem1_backward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                      int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                      const float* stats, int32_t act, float slope, const float* gy, int64_t gy_rows, float* g_conv_w,
                      float* g_bn_w, float* g_bn_b, double* part, void* stream) {
  if (!stem1_args_ok(obs, nimg, pix, na, nb, conv_w, c, bn_w, bn_b) || !stats || !gy || !g_conv_w || !g_bn_w ||
      !g_bn_b || !part || !aligned16(gy) || !aligned16(stats) || (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU) ||
      !stem1_rows_ok(nimg, na, nb, gy_rows))
    return GR_ERR_ARG;
  const gr::Stem1 s = stem1_of(obs, ld, off, rows, nimg, pix, na, nb, conv_w, c, gy_rows);
  const hipError_t e = gr::launch_stem1_backward(s, bn_w, bn_b, stats, act, slope, gy, g_conv_w, g_bn_w, g_bn_b, part,
                                                 (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_tsgemm(const float* a, int64_t lda, const float* b, int32_t b_nk, float* c, int64_t ldc, int64_t m, int32_t k,
              int32_t n, void* stream) {
  if (!a || !b || !c || m < 0 || !gr::tsgemm_covered(k, n, b_nk != 0) || lda < k || ldc < n || ((uintptr_t)a & 3) ||
      m * (lda > ldc ? lda : ldc) >= ((int64_t)1 << 40))
    return GR_ERR_ARG;
  if (m == 0) return GR_OK;
  const hipError_t e = gr::launch_tsgemm(a, (long long)lda, b, b_nk != 0, c, (long long)ldc, (long long)m, k, n,
                                         nullptr, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

static bool bnact_of(int32_t bn_c, const float* stats, const float* bn_w, const float* bn_b, int32_t act, float slope,
                     gr::BnAct* p) {
  if (!stats || !bn_w || !bn_b || !bn_shape_ok(1, bn_c) || (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU))
    return false;
  p->stats = stats; p->w = bn_w; p->b = bn_b; p->c = bn_c; p->act = act; p->slope = slope;
  return true;
}

int gr_tsgemm_bnact(const float* z, int64_t lda, const float* b, float* c, int64_t ldc, int64_t m, int32_t k, int32_t n,
                    int32_t bn_c, const float* stats, const float* bn_w, const float* bn_b, int32_t act, float slope,
                    void* stream) {
  gr::BnAct p;
  if (!z || !b || !c || m < 0 || k != 128 || n != 64 || lda < k || ldc < n || ((uintptr_t)z & 3) || bn_c != 32 ||
      !bnact_of(bn_c, stats, bn_w, bn_b, act, slope, &p) || m * (lda > ldc ? lda : ldc) >= ((int64_t)1 << 40))
    return GR_ERR_ARG;
  if (m == 0) return GR_OK;
  const hipError_t e = gr::launch_tsgemm(z, (long long)lda, b, true, c, (long long)ldc, (long long)m, k, n, &p,
                                         (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_bn_stats(const float* x, int64_t m, int32_t c, float eps, float* stats, double* part, void* stream) {
  if (!bn_shape_ok(m, c) || !x || !stats || !part || !aligned16(x) || !aligned16(stats)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_bn_stats(x, m, c, eps, stats, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int64_t gr_patch_wgrad_floats(int64_t m, int32_t n, int32_t k) {
  if (m < 1) return GR_ERR_ARG;
  const int blocks = gr::patch_wgrad_blocks(m, n, k);
  return blocks ? (int64_t)blocks * n * k : GR_ERR_ARG;
}

int gr_patch_wgrad(const float* x, int64_t ld, const float* gy, int64_t m, int32_t n, int32_t k, float* part,
                   float* gw, void* stream) {
  if (!x || !gy || !part || !gw || m < 1 || gr::patch_wgrad_blocks(m, n, k) == 0 || ld < k || !aligned16(gy) ||
      ((uintptr_t)x & 3) || m * ld >= ((int64_t)1 << 40))
    return GR_ERR_ARG;
  const hipError_t e =
      gr::launch_patch_wgrad(x, (long long)ld, gy, (long long)m, n, k, part, gw, nullptr, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_patch_wgrad_bnact(const float* z, int64_t ld, const float* gy, int64_t m, int32_t n, int32_t k, float* part,
                         float* gw, int32_t bn_c, const float* stats, const float* bn_w, const float* bn_b, int32_t act,
                         float slope, void* stream) {
  gr::BnAct p;
  if (!z || !gy || !part || !gw || m < 1 || n % 64 || gr::patch_wgrad_blocks(m, n, k) == 0 || ld < k ||
      !aligned16(gy) || ((uintptr_t)z & 3) || bn_c % 8 || 128 % bn_c || !bnact_of(bn_c, stats, bn_w, bn_b, act, slope, &p) ||
      m * ld >= ((int64_t)1 << 40))
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_patch_wgrad(z, (long long)ld, gy, (long long)m, n, k, part, gw, &p,
                                              (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_stem12_forward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                      int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b, float eps,
                      int32_t act, float slope, const float* w2f, int32_t n2, float* y, float* z2, float* stats,
                      double* moments, double* part, void* stream) {
  if (!stem1_args_ok(obs, nimg, pix, na, nb, conv_w, c, bn_w, bn_b) || c != 16 || !w2f || !z2 || !stats ||
      !part || !aligned16(w2f) || (y && !aligned16(y)) || !aligned16(z2) || !aligned16(stats) ||
      (reinterpret_cast<uintptr_t>(moments) & 7u) ||
      (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU) || n2 < 1 || na != 9 * n2 ||
      (int64_t)nimg * n2 * 32 >= (int64_t)1 << 31)
    return GR_ERR_ARG;
  const gr::Stem1 s = stem1_of(obs, ld, off, rows, nimg, pix, na, nb, conv_w, c, (int64_t)nimg * na);
  const hipError_t e = gr::launch_stem12_forward(s, bn_w, bn_b, eps, act, slope, w2f, n2, y, z2, stats, moments,
                                                 part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_stem12_backward(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix, int32_t na,
                       int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                       const float* stats, int32_t act, float slope, const float* gz2, int32_t n2, const float* w2t,
                       float* g_conv_w, float* g_bn_w, float* g_bn_b, double* part, void* stream) {
  if (!stem1_args_ok(obs, nimg, pix, na, nb, conv_w, c, bn_w, bn_b) || c != 16 || !stats || !gz2 || !w2t ||
      !g_conv_w || !g_bn_w || !g_bn_b || !part || !aligned16(gz2) || !aligned16(w2t) || !aligned16(stats) ||
      (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU) || n2 < 1 || na != 9 * n2 ||
      (int64_t)nimg * n2 * 32 >= (int64_t)1 << 31)
    return GR_ERR_ARG;
  const gr::Stem1 s = stem1_of(obs, ld, off, rows, nimg, pix, na, nb, conv_w, c, (int64_t)nimg * na);
  const hipError_t e = gr::launch_stem12_backward(s, bn_w, bn_b, stats, act, slope, gz2, n2, w2t, g_conv_w, g_bn_w,
                                                  g_bn_b, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int64_t gr_stem12_backward_w2_scratch_doubles(int32_t nimg) {
  return nimg < 1 ? GR_ERR_ARG : (int64_t)gr::stem12w_scratch_doubles(nimg);
}

int gr_stem12_backward_w2(const float* obs, int64_t ld, int64_t off, const int64_t* rows, int32_t nimg, const int16_t* pix,
                          int32_t na, int32_t nb, const float* conv_w, int32_t c, const float* bn_w, const float* bn_b,
                          const float* stats, const double* moments, int32_t act, float slope, const float* gz2,
                          int32_t n2, const float* w2t, float* g_conv_w, float* g_bn_w, float* g_bn_b, float* g_w2,
                          double* part, void* stream) {
  if (!stem1_args_ok(obs, nimg, pix, na, nb, conv_w, c, bn_w, bn_b) || c != 16 || !stats || !gz2 || !w2t ||
      !g_conv_w || !g_bn_w || !g_bn_b || !g_w2 || !part || !aligned16(gz2) || !aligned16(w2t) || !aligned16(stats) ||
      (reinterpret_cast<uintptr_t>(moments) & 7u) ||
      (act != GR_POLICY_ACT_LRELU && act != GR_POLICY_ACT_ELU) || !gr::stem12w_covers(n2) || na != 9 * n2 ||
      (int64_t)nimg * n2 * 32 >= (int64_t)1 << 31)
    return GR_ERR_ARG;
  const gr::Stem1 s = stem1_of(obs, ld, off, rows, nimg, pix, na, nb, conv_w, c, (int64_t)nimg * na);
  const hipError_t e = gr::launch_stem12_backward_w2(s, bn_w, bn_b, stats, moments, act, slope, gz2, n2, w2t, g_conv_w,
                                                     g_bn_w, g_bn_b, g_w2, part, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_column_sum_partials(int64_t rows) { return rows < 0 ? GR_ERR_ARG : gr::column_sum_blocks(rows); }

int gr_column_sum(const void* x, int dtype, int64_t rows, int32_t cols, float* partial, float* out, void* stream) {
  if (!x || !partial || !out || rows < 0 || cols <= 0 || (dtype != GR_DTYPE_F32 && dtype != GR_DTYPE_BF16))
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_column_sum(x, dtype, (long long)rows, cols, partial, out, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int64_t gr_head_partials(int64_t rows, int32_t k, int32_t h) {
  if (rows < 0 || k < 1 || k > 8 || h < 4 || h > 256 || h % 4) return GR_ERR_ARG;
  return (int64_t)gr::head_partial_rows(rows) * ((k * h + k + h + 3) & ~3);
}



int gr_head_forward(const float* z, int64_t rows, int32_t h, const float* w, const float* b, int32_t k, float slope,
                    float* y, void* stream) {
  if (!z || !w || !b || !y || rows < 0 || k < 1 || k > 8 || h < 4 || h > 256 || h % 4 || !aligned16(z))
    return GR_ERR_ARG;
  if (rows == 0) return GR_OK;
  const hipError_t e = gr::launch_head_forward(z, (long long)rows, h, w, b, k, slope, y, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_head_backward(const float* z, const float* gy, int64_t rows, int32_t h, const float* w, int32_t k, float slope,
                     float* gz, float* partial, float* sums, void* stream) {
  if (!z || !gy || !w || !gz || !partial || !sums || rows <= 0 || k < 1 || k > 8 || h < 4 || h > 256 || h % 4 ||
      !aligned16(z) || !aligned16(gz) || !aligned16(partial))
    return GR_ERR_ARG;
  const hipError_t e =
      gr::launch_head_backward(z, gy, (long long)rows, h, w, k, slope, gz, partial, sums, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

static bool in_args_ok(const float* x, int64_t rows, int32_t d, int32_t ldx, int32_t h) {
  return x && rows > 0 && d >= 4 && d <= 32 && d % 4 == 0 && ldx >= d && ldx % 4 == 0 && h >= 4 && h <= 256 &&
         h % 4 == 0 && aligned16(x);
}

int64_t gr_mlp_in_partials(int64_t rows, int32_t d, int32_t h) {
  if (rows < 0 || d < 4 || d > 32 || d % 4 || h < 4 || h > 256 || h % 4) return GR_ERR_ARG;
  return (int64_t)gr::in_partial_rows(rows) * (h * d + h);
}

int gr_mlp_in_forward(const float* x, int64_t rows, int32_t d, int32_t ldx, const float* w, const float* b, int32_t h,
                      float slope, float* y, void* stream) {
  if (!in_args_ok(x, rows, d, ldx, h) || !w || !b || !y || !aligned16(y)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_in_forward(x, (long long)rows, d, ldx, w, b, h, slope, y, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_mlp_in_backward(const float* gh, const float* hv, const float* x, int64_t rows, int32_t d, int32_t ldx,
                       int32_t h, float slope, float* partial, float* sums, void* stream) {
  if (!in_args_ok(x, rows, d, ldx, h) || !gh || !hv || !partial || !sums || !aligned16(gh) || !aligned16(hv) ||
      !aligned16(partial))
    return GR_ERR_ARG;
  const hipError_t e =
      gr::launch_in_backward(gh, hv, x, (long long)rows, d, ldx, h, slope, partial, sums, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

size_t gr_mlp_args_size(void) { return sizeof(gr_mlp_args); }

int64_t gr_mlp_h1mask_words(int64_t rows, int32_t hidden) {
  if (rows < 0 || (hidden != 128 && hidden != 256)) return GR_ERR_ARG;
  return (rows + 15) / 16 * (hidden / 16) * 4;
}

int64_t gr_mlp_partials(int64_t rows, int32_t hidden, int32_t nets) {
  if (rows < 0 || (hidden != 128 && hidden != 256) || nets < 1 || nets > 2) return GR_ERR_ARG;
  return gr::mlp_partial_floats(rows, hidden, nets, 32, 4);
}

// shapes and alignment of gr_mlp_args; `bwd` also checks the backward's buffers
static bool mlp_args_ok(const gr_mlp_args* a, bool bwd) {
  if (!a || a->rows <= 0 || a->nets < 1 || a->nets > 2 || (a->hidden != 128 && a->hidden != 256)) return false;
  for (int i = 0; i < a->nets; ++i) {
    const gr_mlp_net& n = a->net[i];
    // the kernels index rows and element offsets in 32 bits (gr_mlp.hip): rows * max(H, ldx) < 2^31 (GR_MLP_MAX_ELEMS)
    if (n.ldx > 0 && a->rows > (int64_t)GR_MLP_MAX_ELEMS / (n.ldx > a->hidden ? n.ldx : a->hidden)) return false;
    if (!n.x || !n.w1 || !n.b1 || !n.w2 || !n.b2 || !n.w3 || !n.b3 || !n.h1 || !n.z2 || n.d < 4 || n.d > 32 ||
        n.d % 4 || n.k < 1 || n.k > 4 || n.ldx < n.d || n.ldx % 4 || !aligned16(n.x) || !aligned16(n.w1) ||
        !aligned16(n.w2) || !aligned16(n.w3) || !aligned16(n.b1) || !aligned16(n.b2) || !aligned16(n.h1) ||
        !aligned16(n.z2))
      return false;
    if (!bwd && !n.y) return false;
    if (n.h1mask && !aligned16(n.h1mask)) return false;
    if (bwd && (!n.gy || !n.gz2 || !n.grads || !aligned16(n.gz2))) return false;
  }
  return !bwd || (a->partial && aligned16(a->partial));
}

int gr_mlp_forward(const gr_mlp_args* a, void* stream) {
  if (!mlp_args_ok(a, false)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_mlp_forward(*a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_mlp_backward(const gr_mlp_args* a, void* stream) {
  if (!mlp_args_ok(a, true)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_mlp_backward(*a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_adam_prepare(gr_adam_segment* t, int32_t nseg, int32_t* nblocks) {
  if (!t || !nblocks || nseg < 1 || nseg > GR_ADAM_MAX_SEGMENTS) return GR_ERR_ARG;
  int64_t nb = 0;
  for (int s = 0; s < nseg; ++s) {
    gr_adam_segment& g = t[s];
    if (!g.param || !g.grad || !g.exp_avg || !g.exp_avg_sq || g.numel <= 0 || g.step_slot < 0) return GR_ERR_ARG;
    for (int r = 0; r < s; ++r)
      if (t[r].step_slot == g.step_slot) return GR_ERR_ARG;  // one step counter per segment
    g.block_start = (int32_t)nb;
    nb += (g.numel + GR_ADAM_BLOCK - 1) / GR_ADAM_BLOCK;
    if (nb > 0x7fffffff) return GR_ERR_ARG;
  }
  *nblocks = (int32_t)nb;
  return GR_OK;
}

static bool adam_args_ok(const gr_adam_args* a) {
  return a && a->nseg >= 1 && a->nseg <= GR_ADAM_MAX_SEGMENTS && a->nblocks >= 1 && a->seg && a->step && a->coef &&
         a->part;
}

int gr_adam_clip(const gr_adam_args* a, float max_norm, float* norm_out, void* stream) {
  if (!adam_args_ok(a) || !(max_norm > 0.0f)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_adam_clip(*a, max_norm, norm_out, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_adam_step(const gr_adam_args* a, void* stream) {
  if (!adam_args_ok(a)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_adam_step(*a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_adam_clip_step(const gr_adam_args* a, float max_norm, float* norm_out, const float* kl, float* lr,
                      double desired_kl, double lr_min, double lr_max, void* stream) {
  if (!adam_args_ok(a) || !(max_norm > 0.0f)) return GR_ERR_ARG;
  if (kl && (!lr || lr != a->lr_ptr || !(desired_kl > 0.0) || !(lr_min > 0.0) || !(lr_max >= lr_min)))
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_adam_clip_step(*a, max_norm, norm_out, kl, kl ? lr : nullptr,
                                                 (float)(desired_kl * 2.0), (float)(desired_kl / 2.0), (float)lr_min,
                                                 (float)lr_max, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

static bool dones_bytes_ok(int b) { return b == 1 || b == 4 || b == 8; }

int gr_store_transition(const gr_transition_args* a, void* stream) {
  if (!a || a->n < 0 || a->k < 1 || a->k > 8 || !dones_bytes_ok(a->dones_bytes)) return GR_ERR_ARG;
  if (a->n == 0) return GR_OK;
  if (!a->reward || !a->dones || !a->value || !a->action || !a->logp || !a->mu || !a->sigma || !a->out_reward ||
      !a->out_dones || !a->out_action || !a->out_value || !a->out_logp || !a->out_mu || !a->out_sigma)
    return GR_ERR_ARG;
  if (a->ld_value < 0 || a->ld_logp < 0 || a->ld_action < 0 || a->ld_mu < 0 || a->ld_sigma < 0) return GR_ERR_ARG;
  const hipError_t e = gr::launch_store_transition(*a, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_episode_accumulate(int64_t n, const float* reward, const void* dones, int32_t dones_bytes, float* cur_rew,
                          float* cur_len, float* fin_rew, float* fin_len, uint8_t* fin_done, void* stream) {
  if (n < 0 || !dones_bytes_ok(dones_bytes)) return GR_ERR_ARG;
  if (n == 0) return GR_OK;
  if (!reward || !dones || !cur_rew || !cur_len || !fin_rew || !fin_len || !fin_done) return GR_ERR_ARG;
  const hipError_t e = gr::launch_episode_accumulate(n, reward, dones, dones_bytes, cur_rew, cur_len, fin_rew,
                                                     fin_len, fin_done, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_l2c2_mix(const float* obs, const float* next_obs, const float* w, int64_t rows, int32_t cols, float* out,
                void* stream) {
  if (!obs || !next_obs || !w || !out || rows < 0 || cols <= 0 || cols % 4 || !aligned16(obs) || !aligned16(next_obs) ||
      !aligned16(out))
    return GR_ERR_ARG;
  if (rows == 0) return GR_OK;
  const hipError_t e = gr::launch_l2c2_mix(obs, next_obs, cols, nullptr, nullptr, w, (long long)rows, cols, out,
                                           (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_l2c2_mix_rows(const float* obs, const float* next_obs, int64_t ld, const int64_t* rows_obs,
                     const int64_t* rows_next, const float* w, int64_t rows, int32_t cols, float* out, void* stream) {
  if (!obs || !next_obs || !rows_obs || !rows_next || !w || !out || rows < 0 || cols <= 0 || cols % 4 || ld < cols ||
      ld % 4 || !aligned16(obs) || !aligned16(next_obs) || !aligned16(out))
    return GR_ERR_ARG;
  if (rows == 0) return GR_OK;
  const hipError_t e = gr::launch_l2c2_mix(obs, next_obs, ld, reinterpret_cast<const long long*>(rows_obs),
                                           reinterpret_cast<const long long*>(rows_next), w, (long long)rows, cols, out,
                                           (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_gae(int64_t n, int32_t t_steps, float gamma, float lam, const float* rewards, const uint8_t* dones,
           const float* values, const float* last_values, int64_t ld_last, float* returns, float* advantages,
           void* stream) {
  if (n < 0 || t_steps < 1 || ld_last < 0) return GR_ERR_ARG;
  if (n == 0) return GR_OK;
  if (!rewards || !dones || !values || !last_values || !returns || !advantages) return GR_ERR_ARG;
  const hipError_t e = gr::launch_gae(n, t_steps, gamma, lam, rewards, dones, values, last_values, ld_last, returns,
                                      advantages, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int64_t gr_ppo_loss_partials(int64_t rows) {
  if (rows < 0) return GR_ERR_ARG;
  return (int64_t)gr::ppo_loss_blocks(rows) * 8;
}

static bool loss_args_ok(const gr_ppo_loss_args* a) {
  return a && a->rows > 0 && a->k >= 1 && a->k <= 8 && a->mu && a->std && a->value && a->act && a->logp_old &&
         a->adv && a->value_old && a->ret && a->mu_old && a->sig_old && a->ld_mu >= a->k && a->ld_act >= a->k &&
         a->ld_mu_old >= a->k && a->ld_sig_old >= a->k && a->ld_value >= 1 && a->ld_logp_old >= 1 && a->ld_adv >= 1 &&
         a->ld_value_old >= 1 && a->ld_ret >= 1;
}

int gr_ppo_loss_forward(const gr_ppo_loss_args* a, float* partial, float* sums, void* stream) {
  if (!loss_args_ok(a) || !partial || !sums) return GR_ERR_ARG;
  const hipError_t e = gr::launch_ppo_loss_forward(*a, partial, sums, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_ppo_loss_backward(const gr_ppo_loss_args* a, const float* g, float* dmu, float* dvalue, float* partial,
                         float* dstd, void* stream) {
  if (!loss_args_ok(a) || !g || !dmu || !dvalue || !partial || !dstd) return GR_ERR_ARG;
  const hipError_t e = gr::launch_ppo_loss_backward(*a, g, 1, 1.0f, dmu, dvalue, partial, dstd, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_ppo_loss_forward_loss(const gr_ppo_loss_args* a, float* partial, float* sums, float value_coef, float* loss,
                             float* stats, float* acc, float* kl_out, void* stream) {
  if (!loss_args_ok(a) || !partial || !sums || !loss || !stats) return GR_ERR_ARG;
  const hipError_t e = gr::launch_ppo_loss_forward_loss(*a, partial, sums, value_coef, loss, stats, acc, kl_out,
                                                        (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_ppo_loss_backward_loss(const gr_ppo_loss_args* a, const float* g_loss, float value_coef, float* dmu,
                              float* dvalue, float* partial, float* dstd, void* stream) {
  if (!loss_args_ok(a) || !g_loss || !dmu || !dvalue || !partial || !dstd) return GR_ERR_ARG;
  const hipError_t e = gr::launch_ppo_loss_backward(*a, g_loss, 0, value_coef, dmu, dvalue, partial, dstd,
                                                    (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_ppo_loss_forward_backward(const gr_ppo_loss_args* a, const float* g_loss, float value_coef, float* partial,
                                 float* sums, float* loss, float* stats, float* acc, float* kl_out, float* dmu,
                                 float* dvalue, float* dpartial, float* dstd, void* stream) {
  if (!loss_args_ok(a) || !g_loss || !partial || !sums || !loss || !stats || !dmu || !dvalue || !dpartial || !dstd ||
      partial == dpartial)
    return GR_ERR_ARG;
  const hipError_t e = gr::launch_ppo_loss_forward_backward(*a, g_loss, value_coef, partial, sums, loss, stats, acc,
                                                            kl_out, dmu, dvalue, dpartial, dstd, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_adaptive_lr(const float* kl, float* lr, double desired_kl, double lr_min, double lr_max, void* stream) {
  if (!kl || !lr || !(desired_kl > 0.0) || !(lr_min > 0.0) || !(lr_max >= lr_min)) return GR_ERR_ARG;
  const hipError_t e = gr::launch_adaptive_lr(kl, lr, (float)(desired_kl * 2.0), (float)(desired_kl / 2.0),
                                              (float)lr_min, (float)lr_max, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : GR_ERR_HIP;
}

int gr_test_dynamics(gr_ctx* c, int n, int mode, const float* si, const float* ab, const float* cmd, const float* ci,
                     const float* par, const float* drag, float* so, float* co, float* xo, void* stream) {
  if (!c || n <= 0 || !si || !ab || !cmd || !ci || !par || !drag || !so || !co || !xo) return GR_ERR_ARG;
  if (int r = ensure_dev(c, "gr_test_dynamics")) return r;
  hipError_t e = gr::launch_test_dynamics(c->args, n, mode, si, ab, cmd, ci, par, drag, so, co, xo, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_test_dynamics");
}

int gr_test_math(gr_ctx* c, int fn, int n, const float* x, const float* y, float* out, void* stream) {
  if (!c || n <= 0 || !x || !y || !out) return GR_ERR_ARG;
  hipError_t e = gr::launch_test_math(fn, n, x, y, out, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_test_math");
}

int gr_test_philox(gr_ctx* c, int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t* out4, void* stream) {
  if (!c || n <= 0 || !out4) return GR_ERR_ARG;
  hipError_t e = gr::launch_test_philox(n, c0, c1, c2, c3, c->cfg.seed_lo, c->cfg.seed_hi, out4, (hipStream_t)stream);
  return e == hipSuccess ? GR_OK : hip_fail(c, e, "gr_test_philox");
}

int gr_debug_read_stamps(uint64_t* host, int n) {
  if (!host || n <= 0) return GR_ERR_ARG;
  hipError_t e = gr::read_stamps(reinterpret_cast<unsigned long long*>(host), n);
  return e == hipSuccess ? GR_OK : (e == hipErrorNotSupported ? GR_ERR_STATE : GR_ERR_HIP);
}

int gr_debug_read_policy_stamps(uint64_t* host, int n) {
  if (!host || n <= 0) return GR_ERR_ARG;
  hipError_t e = gr::read_policy_stamps(reinterpret_cast<unsigned long long*>(host), n);
  return e == hipSuccess ? GR_OK : (e == hipErrorNotSupported ? GR_ERR_STATE : GR_ERR_HIP);
}

}  // extern "C"
