// gr_kernels.h — kernel argument block and launchers (internal to libgr.so).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/gr.h"

#ifndef GR_BLOCK
#define GR_BLOCK 256  // envs per step workgroup (three roles x GR_BLOCK / 64 waves)
#endif
#define GR_MAX_TYPES 64
#define GR_LOG_ROWS_PER_BLOCK (GR_BLOCK / 64)  // log rows per workgroup (one per physics wave of the step kernel)
// step kernel handovers + store staging + obstacle hand-over (3 rows + ready flags) in LDS
#define GR_XCH_BYTES ((5 + 6 + 8 + 3) * GR_BLOCK * 16 + 16)
#define GR_LDS_MAX (160 * 1024)                 // LDS a gfx950 workgroup may allocate
#define GR_STAMP_WAVES 8192  // diagnostic stamps (GR_STAMPS builds only)
#define GR_STAMP_SLOTS 16

struct gr_cam_const;  // gr_camera.h

namespace gr {

enum { KMODE_STEP = 0, KMODE_RESET = 1, KMODE_OBSERVE = 2 };

// Per-context constants: the config and everything derived from it once on the
// host.  Lives in device memory and is read through a __restrict__ kernel
// argument, so the compiler emits scalar loads next to each use instead of
// hoisting ~150 kernarg dwords into SGPRs at entry (which spilled into VGPR lanes).
struct KConst {
  gr_config cfg;
  int track_stride;    // floats per track: max_gates*GR_GATE_FLOATS + GR_TRACK_FLOATS
  int lds_bytes;       // dynamic LDS per workgroup (0: read the table from global memory)
  int type_start[GR_MAX_TYPES + 1];
  float thrust_lo, thrust_hi;  // 4 * f(omega_min/max), controller_diff.py:96-99
  float lat_reach;             // > max |lattice offset|: ground-test cull radius
  float w[7];                  // reward weights in RewardsCfg order
  // motor model (controller_diff.py:140-144, thrust_controller_diff.py)
  float B[4][4], Bi[4][4];
  float motor_fmax, motor_c;
  float tm_k2, tm_k1, tm_k0, tm_k1sq, tm_4k2, tm_inv2k2, tm_negk1;
};

// Constants every wave needs before its first loads / RNG draws: passed by value
// (one kernarg fetch at entry) instead of through the KConst pointer chain.
struct KHot {
  int num_envs, num_levels, max_gates, track_stride;
  int env_id_offset, use_motor_model, obs_noise, lds_tab_vec;  // lds_tab_vec: float4 of LDS table (0: global)
  uint32_t seed_lo, seed_hi;
  float obs_lin_vel_noise, obs_att_noise;
  float obst_span;  // obstacle grid: cell + 2 margin (m), the side of a hinted grown cell
  int dr_rotor;     // per-env rotor constants (GR_P_ROTOR)
  int integrator;   // GR_INTEGRATOR_* (the launch picks the lean step kernel for the explicit integrator)
  int test_fault;   // gr_test_inject_fault (0 in production)
};

// Passed by value (kernarg): per-binding pointers + the constants pointer.
struct KArgs {
  const KConst* kc;      // device copy (set from the kernel's __restrict__ argument)
  gr_buffers buf;
  const float* table;    // packed track table [T*L][track_stride]
  const int* blk_types;  // per workgroup: first | last terrain type << 16 (host-derived)
  // obstacles (gr_bind_obstacles; null: none): per-track xy grid, cells of record copies
  const float4* obst_grid_f;  // [T*L]: x0, y0, 1/cell, cell
  const int4* obst_grid_i;    // [T*L]: nx, ny, first cell, 0
  const int2* obst_cells;     // [C]: first item, count
  const float4* obst_items;   // [I][GR_OBST_FLOATS / 4]
  // observation sink (gr_bind_obs_sink; null: none): the policy / critic rows again, in sink_dtype
  void* sink_policy;
  void* sink_critic;
  int sink_dtype;
  unsigned* status;  // device status word (GR_STATUS_* bits, OR-ed by the kernels; gr_device_status)
  KHot h;
};

// Depth camera (gr_camera.hip): everything by value except the derived constants.
struct CamArgs {
  const ::gr_cam_const* cc;  // device copy
  const float* state;
  const int32_t* istate;
  const float* obs_p16;  // this call's state observations [N][16]
  const float* obs_c16;
  const uint8_t* terminated;
  const uint8_t* time_out;
  const uint8_t* mask;  // GR_CAM_RESET only (nullptr: all)
  const uint32_t* counters;
  int counter_index;
  const float* table;  // packed track table
  const float* obst;   // obstacle records [T*L][max_obst][GR_OBST_FLOATS] (null: none)
  const int32_t* obst_counts;  // [T*L]
  int max_obst;
  int track_stride, num_levels, max_gates, num_envs, env_id_offset, mode, width, height;
  int obst_slots;  // obstacle slots per wave in LDS (launch_camera sets it; > 0 on entry: a test's request)
  uint32_t seed_lo, seed_hi;
  float* depth;
  int32_t* age;
  float* out_p;
  float* out_c;
};
hipError_t launch_camera(const CamArgs& a, hipStream_t s);
hipError_t launch_policy(const gr_policy_args& a, hipStream_t s);  // gr_policy.hip
hipError_t launch_policy_f32(const gr_policy_args& a, hipStream_t s);  // gr_policy_f32.hip
int bn_scratch_doubles(long long m, int c);                                                // gr_bn.hip
// the stem's first block from the image (gr_bn.hip): image b at obs + b * ld + off; rows nimg x na from
// table a, then nimg x nbt from table b; pix [(na + nbt) * 9]; conv weight w [c][9]
struct Stem1 {
  const float* obs;
  long long ld, off;
  const long long* rows;  // image b is row rows[b] of obs (a mini-batch read through its permutation), or b if null
  int nimg, na, nbt;
  const short* pix;
  const float* w;
  int c;
  long long rows_out;  // rows of y / gy that exist: the forward stores rows [0, rows_out), the backward reads the
                       // gradient of those rows and takes the rest (cells no later layer reads) as zero
};
long long stem1_scratch_doubles(int nimg, int rows_per_img, int c);
hipError_t launch_stem1_forward(const Stem1& s, const float* bw, const float* bb, float eps, int act, float slope,
                                float* y, float* stats, double* part, hipStream_t st);
hipError_t launch_stem1_backward(const Stem1& s, const float* bw, const float* bb, const float* stats, int act,
                                 float slope, const float* gy, float* gconv, float* gbw, float* gbb, double* part,
                                 hipStream_t st);
// the first block's forward with conv2 (16 -> 32, 3x3 / 3) fused into its apply pass: y1 and z2 (gr_bn.hip stem12f_kernel)
hipError_t launch_stem12_forward(const Stem1& s, const float* bw, const float* bb, float eps, int act, float slope,
                                 const float* w2f, int n2, float* y, float* z2, float* stats, double* moments,
                                 double* part, hipStream_t st);
// ... and with conv2's weight gradient gw2 [32][144] too (position-major waves, y1 recomputed: gr_bn.hip stem12w_kernel;
// n2 <= 80), so the forward needs to store no y1
long long stem12w_scratch_doubles(int nimg);
bool stem12w_covers(int n2);
hipError_t launch_stem12_backward_w2(const Stem1& s, const float* bw, const float* bb, const float* stats,
                                     const double* moments, int act, float slope, const float* gz2, int n2,
                                     const float* w2t, float* gconv, float* gbw, float* gbb, float* gw2, double* part,
                                     hipStream_t st);
// the same backward with conv2's input gradient formed inside the passes (C = 16, na = 9 n2; gr_bn.hip stem12b_kernel)
hipError_t launch_stem12_backward(const Stem1& s, const float* bw, const float* bb, const float* stats, int act,
                                  float slope, const float* gz2, int n2, const float* w2t, float* gconv, float* gbw,
                                  float* gbb, double* part, hipStream_t st);
hipError_t launch_bn_running_update(float* rm, float* rv, long long* nbt, const float* stats, int c, float keep,
                                    float momentum, int uses, int count, hipStream_t s);
hipError_t launch_bn_forward(const float* x, long long m, int c, const float* w, const float* b, float eps, int act,
                             float slope, float* y, float* stats, double* part, hipStream_t s);
hipError_t launch_bn_backward(const float* x, const float* gy, long long m, int c, const float* w, const float* b,
                              const float* stats, int act, float slope, float* gx, float* gw, float* gb, double* part,
                              hipStream_t s);
int column_sum_blocks(long long m);                                                                       // gr_update.hip
int patch_wgrad_blocks(long long m, int n, int k);  // gr_update.hip: gw[n][k] = gy^T x (0: (n, k) not covered)
// a BatchNorm (batch statistics) + activation applied to a patch GEMM's input as it is loaded (gr_update.hip)
struct BnAct {
  const float* stats;  // [4][c]: mean, invstd, biased var, unbiased var (gr_bn_act_forward's)
  const float* w;
  const float* b;
  int c, act;
  float slope;
};
bool tsgemm_covered(int k, int n, bool b_nk);  // gr_update.hip: C[m][n] = A[m][k] B[k][n], B in registers
hipError_t launch_tsgemm(const float* a, long long lda, const float* bm, bool b_nk, float* c, long long ldc,
                         long long m, int k, int n, const BnAct* bna, hipStream_t s);
hipError_t launch_patch_wgrad(const float* x, long long ld, const float* gy, long long m, int n, int k, float* part,
                              float* gw, const BnAct* bna, hipStream_t s);
hipError_t launch_bn_stats(const float* x, long long m, int c, float eps, float* stats, double* part, hipStream_t s);
hipError_t launch_column_sum(const void* x, int dtype, long long m, int n, float* part, float* out, hipStream_t s);
int head_partial_rows(long long m);                                                                      // gr_update.hip
int in_partial_rows(long long m);                                                                        // gr_update.hip
hipError_t launch_l2c2_mix(const float* o, const float* nx, long long ld, const long long* ra, const long long* rb,
                           const float* w, long long rows, int cols, float* out, hipStream_t s);  // gr_rollout.hip
hipError_t launch_head_forward(const float* z, long long m, int h, const float* w, const float* b, int k, float slope,
                               float* y, hipStream_t s);
hipError_t launch_head_backward(const float* z, const float* gy, long long m, int h, const float* w, int k,
                                float slope, float* gz, float* part, float* sums, hipStream_t s);
hipError_t launch_in_forward(const float* x, long long m, int d, int ldx, const float* w, const float* b, int h,
                             float slope, float* y, hipStream_t s);
hipError_t launch_adam_clip(const gr_adam_args& a, float max_norm, float* norm_out, hipStream_t s);
hipError_t launch_adam_step(const gr_adam_args& a, hipStream_t s);
hipError_t launch_adam_clip_step(const gr_adam_args& a, float max_norm, float* norm_out, const float* kl, float* lr,
                                 float hi, float lo, float lr_min, float lr_max, hipStream_t s);
hipError_t launch_store_transition(const gr_transition_args& a, hipStream_t s);  // gr_rollout.hip
hipError_t launch_episode_accumulate(long long n, const float* reward, const void* dones, int dones_bytes,
                                     float* cur_rew, float* cur_len, float* fin_rew, float* fin_len,
                                     uint8_t* fin_done, hipStream_t s);
hipError_t launch_gae(long long n, int t_steps, float gamma, float lam, const float* rewards, const uint8_t* dones,
                      const float* values, const float* last_values, long long ld_last, float* returns,
                      float* advantages, hipStream_t s);
int ppo_loss_blocks(long long rows);
hipError_t launch_ppo_loss_forward(const gr_ppo_loss_args& a, float* part, float* sums, hipStream_t s);
hipError_t launch_ppo_loss_forward_loss(const gr_ppo_loss_args& a, float* part, float* sums, float value_coef,
                                        float* loss, float* stats, float* acc, float* kl_out, hipStream_t s);
hipError_t launch_ppo_loss_forward_backward(const gr_ppo_loss_args& a, const float* g, float value_coef, float* part,
                                            float* sums, float* loss, float* stats, float* acc, float* kl_out,
                                            float* dmu, float* dvalue, float* dpart, float* dstd, hipStream_t s);
hipError_t launch_ppo_loss_backward(const gr_ppo_loss_args& a, const float* g, int gv_index, float gv_coef, float* dmu,
                                    float* dvalue, float* part, float* dstd, hipStream_t s);
hipError_t launch_adaptive_lr(const float* kl, float* lr, float hi, float lo, float lr_min, float lr_max,
                              hipStream_t s);
// gr_mlp.hip: the update's whole-network MLP kernels
// gr_terrain.hip: gr_terrain_commit (staged terrain -> live, gate table packed, obstacle hints cleared)
struct TerrainCommitArgs {
  const float4* s_gates;   // staged [ntr][g4]
  const float4* s_tracks;  // staged [ntr] track records
  float4* table;           // packed [ntr][stride4]
  int ntr, g4, stride4;
  const float4* s_obst;    // staged obstacle block (null: obstacle-free tracks)
  float4* l_obst;          // live obstacle block
  const int* hdr;          // staged header: [0] = float4s of the block to copy
  long long max_obst4;     // float4s of the block (capacity)
  float4* hints;           // GR_P_OHINT plane (null: buffers not bound)
  int n_hints;
};
hipError_t launch_terrain_commit(const TerrainCommitArgs& a, hipStream_t s);
hipError_t launch_mlp_forward(const gr_mlp_args& a, hipStream_t s);
hipError_t launch_mlp_backward(const gr_mlp_args& a, hipStream_t s);
int64_t mlp_partial_floats(long long rows, int hidden, int nets, int max_d, int max_k);
hipError_t launch_in_backward(const float* gh, const float* hv, const float* x, long long m, int d, int ldx, int h,
                              float slope, float* part, float* sums, hipStream_t s);
// Camera launch (camera_kernel, gr_camera.hip).  Dynamic LDS: the normal table and the ray tables (workgroup), then
// per wave its gate slots, one 64-bit gate mask per 8x32 tile, on obstacle tracks its obstacle slots (the first
// `slots` obstacles in view; any further ones are set up again per tile from their records), their windows' pixel
// rectangles (one packed word per slot) and tile masks, and an 8-row staging band.  Every part a multiple of 4 floats.
#define GR_CAM_GATE_SLOT 36     // floats per gate slot in LDS (GR_CAM_SLOT of gr_camera.h)
#define GR_CAM_OSLOT 16         // floats per obstacle slot in LDS: slot floats 0-15 (frame, primitive, kind)
#define GR_CAM_OBST_SLOTS_MAX 64  // (64-bit tile masks)
#define GR_CAM_OBST_SLOTS 56    // obstacle slots per wave (obstacles in view per env: p99 41, max 53 over 1 024 envs)
#define CAM_WAVES 4             // waves per workgroup
#define CAM_LDS_PER_CU 163840
// (the normal table of the image noise, gr_normal_table.h: 4 floats per entry)
#define CAM_NORMAL_FLOATS (4 * 320)
__host__ __device__ inline size_t camera_tile_mask_floats(int width, int height) {
  return (2 * (size_t)((height + 7) / 8) * ((width + 31) / 32) + 3) & ~(size_t)3;
}
// obstacle slots + their pixel rectangles + their tile masks
__host__ __device__ inline size_t camera_obst_floats(int width, int height, int slots) {
  return slots > 0 ? (size_t)slots * GR_CAM_OSLOT + (((size_t)slots + 3) & ~(size_t)3) +
                         camera_tile_mask_floats(width, height)
                   : 0;
}
__host__ __device__ inline size_t camera_wave_floats(int width, int height, int max_gates, int slots) {
  return (size_t)max_gates * GR_CAM_GATE_SLOT + camera_tile_mask_floats(width, height) +
         camera_obst_floats(width, height, slots) + 8 * (size_t)width;
}
inline size_t camera_lds_bytes(int width, int height, int max_gates, int waves, int slots) {
  const size_t wpad = (size_t)((width + 3) & ~3), hpad = (size_t)((height + 3) & ~3);
  return 4 * (CAM_NORMAL_FLOATS + wpad + hpad + (size_t)waves * camera_wave_floats(width, height, max_gates, slots));
}
struct CamLaunch {
  int waves, slots;
  size_t lds;
};
// 4-wave workgroups; on obstacle tracks GR_CAM_OBST_SLOTS slots per wave, or slots_req > 0 (tests: the path for
// obstacles beyond the slots).  (Two 10-wave workgroups per CU with 43 slots, for 5 waves per SIMD, measured 1.68 ->
// 1.93 ms per obstacle re-render: the second workgroup's waves do not fit beside the first's at 96 VGPRs, r6za)
inline CamLaunch camera_launch_config(int width, int height, int max_gates, bool obst, int slots_req) {
  const int slots = obst ? (slots_req > 0 ? slots_req : GR_CAM_OBST_SLOTS) : 0;
  return {CAM_WAVES, slots, camera_lds_bytes(width, height, max_gates, CAM_WAVES, slots)};
}

// which step_kernel instantiation gr_step launches for these arguments (GR_STEP_* of gr.h)
int step_variant(const KArgs& a);
hipError_t launch_env(int mode, const KArgs& a, const float* actions, const uint8_t* mask, hipStream_t s,
                      hipEvent_t t0, hipEvent_t t1);
hipError_t launch_init(const KArgs& a, hipStream_t s);
hipError_t launch_log_finalize(const float* rows, int nrows, const float* prev, float* out, float ep_len_s,
                               float num_envs, hipStream_t s);
hipError_t launch_test_dynamics(const KArgs& a, int n, int mode, const float* si, const float* ab, const float* cmd,
                                const float* ci, const float* par, const float* drag, float* so, float* co, float* xo,
                                hipStream_t s);
hipError_t launch_test_math(int fn, int n, const float* x, const float* y, float* out, hipStream_t s);
hipError_t read_stamps(unsigned long long* host, int n);
hipError_t read_policy_stamps(unsigned long long* host, int n);  // gr_policy.hip
hipError_t allow_large_lds();  // lift the default dynamic-LDS cap of the env kernels
hipError_t launch_test_philox(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                              uint32_t* out, hipStream_t s);

}  // namespace gr
