// gr_policy.hip — rollout inference of the rsl_rl ActorCritic on MFMA (gfx950, bf16 in / fp32 accumulate).
//
// Reference: PPO.act (standalone/rsl_rl/ext/algorithms/ppo.py:71-85) calls ActorCritic.act (sample from
// Normal(actor(obs), std)), .evaluate (critic(critic_obs)) and .get_actions_log_prob; the MLPs are
// Linear -> act -> Linear -> act -> Linear with two hidden layers of H units (rsl_rl_ppo_cfg.py:15-41:
// [256, 256] per BASELINE; (128, 128) in the reference's state cfg), LeakyReLU(0.01) or ELU.
//
// One launch does both networks for all envs: blockIdx.y 0 = actor (+ Gaussian sampling and the log
// prob), 1 = critic.  A workgroup = 8 waves x 64 envs.  The hidden activations never leave registers:
// every layer is computed transposed, Y^T = W X^T, with W as the MFMA A operand and the activations as
// the B operand, so the fp32 accumulator tile of one layer (hidden unit on the register row, env on the
// lane column) becomes the next layer's B fragment by a bf16 pack in place (the k order inside a
// 32-wide k step is permuted; the host packs W in that same order, see rsl_rl/fused_inference.py).
// All weights (152 KB bf16 at H = 256) are staged once per workgroup in LDS, and every A fragment read
// from LDS feeds the four 16-env column tiles of a wave.
#include <hip/hip_runtime.h>

#include "../../include/gr.h"
#include "gr_kernels.h"
#include "gr_math.h"
#include "gr_rng.h"

namespace gr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#ifndef POL_WAVES
#define POL_WAVES 8  // waves per workgroup (two per SIMD: 256 registers per wave for 2 column tiles, no spills)
#endif
#ifndef POL_COLS
#define POL_COLS 2  // 16-env column tiles per wave: each LDS A fragment feeds POL_COLS MFMAs
#endif
#ifndef POL_BLOCKS_PER_NET
#define POL_BLOCKS_PER_NET 128  // 256 CUs on MI355X: one workgroup per CU for the two networks
#endif
#ifndef POL_TG
#define POL_TG 2  // layer-2 output row tiles per group: TG x COLS independent accumulator chains
#endif
#ifndef POL_PF
#define POL_PF 1  // k steps of A-fragment prefetch (register ring of POL_PF + 1 fragments per row tile)
#endif
#define POL_RING_IDX (s % (PF + 1))
#ifndef POL_PIPE
#define POL_PIPE 0  // 1: drain group g (activation, pack, layer 3) under group g + 1's first MFMAs
#endif
#ifndef POL_SB
#define POL_SB 1  // scheduling barriers around each k step's MFMAs
#endif
#ifndef POL_STAGGER
#define POL_STAGGER 0  // s_sleep units (64 cycles) by which waves 4-7 (the SIMD partners of 0-3) start late
#endif
#ifndef POL_PRIO
#define POL_PRIO 0  // 1: s_setprio 1 for waves 4-7
#endif
#define POL_ENVS_PER_WAVE (16 * POL_COLS)
static_assert(POL_COLS == 1 || POL_COLS == 2 || POL_COLS == 4, "the epilogue maps a wave's 16 C envs x 4 rows onto 64 lanes");

// -DGR_STAMPS (diagnostic build only, scripts/stamps.py policy): lane 0 of every wave records s_memtime at
// phase boundaries (0 entry, 1 weights staged, then per env tile k < 3: 2 + 4k layer 1, 3 + 4k layers 2 + 3,
// 4 + 4k epilogue stored; 14 / 15 s_memrealtime at entry / exit).  The product build compiles these away.
#ifdef GR_STAMPS
#define POL_STAMP_WAVES 4096
__device__ unsigned long long g_pol_stamps[POL_STAMP_WAVES * 16];
#define PSTAMP(k, fn)                                                                              \
  do {                                                                                            \
    unsigned long long t_ = fn();                                                                 \
    const unsigned w_ = (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); \
    if ((threadIdx.x & 63) == 0 && w_ < POL_STAMP_WAVES && (k) < 16) g_pol_stamps[w_ * 16 + (k)] = t_; \
  } while (0)
#else
#define PSTAMP(k, fn)
#endif

template <int ACT>
__device__ __forceinline__ float pol_act(float x) {
  // LeakyReLU (torch default slope 0.01) or ELU (alpha 1); compile-time, so the layer loops stay straight-line
  // ELU's exp(x) - 1 on the hardware exp2 (absolute error ~1e-7, far below the bf16 rounding that follows)
  if constexpr (ACT == GR_POLICY_ACT_ELU) return x > 0.0f ? x : __builtin_amdgcn_exp2f(x * 1.44269504f) - 1.0f;
  return fmaxf(x, 0.01f * x);  // = LeakyReLU(0.01) for every finite x: two VALU ops
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& lo, const f32x4& hi) {
  bf16x8 r;
  r[0] = (__bf16)lo[0]; r[1] = (__bf16)lo[1]; r[2] = (__bf16)lo[2]; r[3] = (__bf16)lo[3];
  r[4] = (__bf16)hi[0]; r[5] = (__bf16)hi[1]; r[6] = (__bf16)hi[2]; r[7] = (__bf16)hi[3];
  return r;
}

// the bias of an accumulator tile's rows (hidden units row0 + 4 (lane >> 4) + r), from LDS: the MFMA chain
// starts from it, so no add is needed afterwards
__device__ __forceinline__ f32x4 bias4(const float* b, int row0, int lane) {
  return *reinterpret_cast<const f32x4*>(b + row0 + 4 * (lane >> 4));
}
template <int ACT>
__device__ __forceinline__ void act4(f32x4& v) {
  if constexpr (ACT == GR_POLICY_ACT_LRELU) {
    // LeakyReLU(y) = 0.505 y + 0.495 |y|.  Layers 1 and 2 arrive pre-scaled by GR_POLICY_LRELU_PRESCALE
    // (v = 0.505 y, the host scales W and b), so the activation is ONE v_fma_f32 with an |.| source
    // modifier per element: v + (0.99 / 1.01) |v| (y for y > 0, 0.01 y below).  (max(y, 0.01 y) took a
    // packed multiply and a max; packed f32 VALU beside MFMAs costs more than its issue slot.)
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = __builtin_fmaf(__builtin_fabsf(v[r]), 0.980198019f, v[r]);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = pol_act<ACT>(v[r]);
  }
}

// Per workgroup (one network, 8 waves x 64 envs): all weight fragments staged in LDS once
// (W1 [T][64], W2 [T][S][64], W3 [S][64] bf16x8 = 152 KB at H = 256).  Per wave, layer 2 runs in pairs
// of output row tiles; each pair's activations are packed into one k step of layer 3 and consumed at
// once, so only layer 1's fragments (h1) and the running layer-3 accumulators stay live.
template <int H, int ACT>
__global__ __launch_bounds__(POL_WAVES * 64) void policy_kernel(gr_policy_args pa) {
  constexpr int T = H / 16;  // 16-row tiles of a hidden layer
  constexpr int S = H / 32;  // 32-wide k steps over a hidden layer
  constexpr int C = POL_COLS;
  const gr_policy_net& net = pa.net[blockIdx.y];
  PSTAMP(14, __builtin_amdgcn_s_memrealtime);
  PSTAMP(0, __builtin_amdgcn_s_memtime);
  extern __shared__ bf16x8 wl[];
  bf16x8* w1s = wl;                  // [T][64]
  bf16x8* w2s = wl + T * 64;         // [T][S][64]
  bf16x8* w3s = w2s + T * S * 64;    // [S][64]
  float* b1s = reinterpret_cast<float*>(w3s + S * 64);  // [H]
  float* b2s = b1s + H;                                 // [H]
  {
    const bf16x8* __restrict__ g1 = reinterpret_cast<const bf16x8*>(net.w1);
    const bf16x8* __restrict__ g2 = reinterpret_cast<const bf16x8*>(net.w2);
    const bf16x8* __restrict__ g3 = reinterpret_cast<const bf16x8*>(net.w3);
    // all of a thread's fragments loaded before any is written: one L2 round trip, not one per fragment
    constexpr int NV = T * 64 + T * S * 64 + S * 64, PER = (NV + POL_WAVES * 64 - 1) / (POL_WAVES * 64);
    bf16x8 st[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + q * POL_WAVES * 64;
      const bf16x8* src = i < T * 64 ? g1 + i : i < T * 64 + T * S * 64 ? g2 + (i - T * 64) : g3 + (i - T * 64 - T * S * 64);
      if (i < NV) st[q] = *src;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int i = threadIdx.x + q * POL_WAVES * 64;
      if (i < NV) wl[i] = st[q];  // w1s, w2s, w3s are contiguous
    }
    for (int i = threadIdx.x; i < H; i += POL_WAVES * 64) {
      b1s[i] = net.b1[i];
      b2s[i] = net.b2[i];
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int n = pa.num_envs, D = net.num_obs;
  const uint32_t cnt = pa.counters[pa.counter_index];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) pa.counters[pa.counter_index ^ 1] = cnt + 1u;
  __syncthreads();  // weights staged
  // persistent over env tiles: the weights are staged once per workgroup.  Layer-1 B fragments: obs^T,
  // lane l holds obs[env0 + 16c + (l & 15)][8 (l >> 4) + j] (k < D, else 0), from two unconditional
  // float4 loads per lane and column tile (rows clamped into range, num_obs % 4 == 0).  The next tile's
  // loads are issued before this tile's MLP, so their latency hides behind it.
  const int envs_per_block = POL_WAVES * POL_ENVS_PER_WAVE, stride = gridDim.x * envs_per_block;
  const int k0 = 8 * (lane >> 4), kc = k0 < D ? k0 : 0;
  float4 ld[C][2];
  auto load_obs = [&](int base) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int env = base + wave * POL_ENVS_PER_WAVE + 16 * c + (lane & 15);
      env = env < n ? env : n - 1;
      const float4* row = reinterpret_cast<const float4*>(net.obs + (size_t)env * D + kc);
      ld[c][0] = row[0];
      ld[c][1] = k0 + 4 < D ? row[1] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  };
  // Epilogue lane map: a wave's 16 C envs x 4 output rows on its 64 lanes.  Lane L takes env e = L % (16 C)
  // of the wave and the RPL = C rows RPL p .. RPL p + RPL - 1 (p = L / (16 C)).  Per-row sampling constants
  // (actor): std, 1 / (2 var), -log(std) - log(sqrt(2 pi)).
  constexpr int RPL = C;
  const int p = lane / (16 * C), e_w = lane % (16 * C);
  float sdv[RPL], i2v[RPL], lpc[RPL];
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    const int r = RPL * p + q;
    sdv[q] = blockIdx.y == 0 && r < net.num_out ? pa.std[r] : 1.0f;
    i2v[q] = 1.0f / (2.0f * sdv[q] * sdv[q]);
    lpc[q] = -logf(sdv[q]) - 0.91893853320467274f;
  }
  load_obs(blockIdx.x * envs_per_block);
  PSTAMP(1, __builtin_amdgcn_s_memtime);
  int tile_k = 0;
  (void)tile_k;  // (stamp slot index, GR_STAMPS builds)
#if POL_PRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#if POL_STAGGER
  if (wave >= 4) __builtin_amdgcn_s_sleep(POL_STAGGER);
#endif
  for (int base = blockIdx.x * envs_per_block; base < n; base += stride) {
  const int env0 = base + wave * POL_ENVS_PER_WAVE;
  bf16x8 xb[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float v[8] = {ld[c][0].x, ld[c][0].y, ld[c][0].z, ld[c][0].w, ld[c][1].x, ld[c][1].y, ld[c][1].z, ld[c][1].w};
#pragma unroll
    for (int j = 0; j < 8; ++j) xb[c][j] = (__bf16)(k0 + j < D ? v[j] : 0.0f);
  }
  if (base + stride < n) load_obs(base + stride);
  // ---- layer 1: h1^T = act(W1 x^T + b1), two row tiles at a time = one k step of layer 2
  bf16x8 h1[S][C];
#pragma unroll
  for (int t = 0; t < T; t += 2) {
    const bf16x8 a0 = w1s[t * 64 + lane], a1 = w1s[(t + 1) * 64 + lane];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      f32x4 y0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, xb[c], bias4(b1s, 16 * t, lane), 0, 0, 0);
      f32x4 y1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, xb[c], bias4(b1s, 16 * t + 16, lane), 0, 0, 0);
      act4<ACT>(y0);
      act4<ACT>(y1);
      h1[t / 2][c] = pack8(y0, y1);
    }
  }
  PSTAMP(2 + 4 * tile_k, __builtin_amdgcn_s_memtime);
  // ---- layer 2 (pairs of row tiles) fused with layer 3: out^T += W3[:, k step t/2] act(W2 h1^T + b2)
  f32x4 o[C];
#pragma unroll
  for (int c = 0; c < C; ++c) o[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  constexpr int TG = POL_TG;  // row tiles per group (even): TG x C independent accumulator chains
  // activation + bf16 pack + layer-3 k step of a finished group's accumulators
  auto drain = [&](f32x4 (&g)[TG][C], int t0) {
#pragma unroll
    for (int u = 0; u < TG; u += 2) {
      const bf16x8 a3 = w3s[((t0 + u) / 2) * 64 + lane];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        act4<ACT>(g[u][c]);
        act4<ACT>(g[u + 1][c]);
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3, pack8(g[u][c], g[u + 1][c]), o[c], 0, 0, 0);
      }
    }
  };
#if POL_PIPE
  f32x4 pend[TG][C];  // the previous group: drained right after the first k step of the next one is issued
#endif
#pragma unroll
  for (int t = 0; t < T; t += TG) {
    f32x4 acc[TG][C];
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const f32x4 b = bias4(b2s, 16 * (t + u), lane);
#pragma unroll
      for (int c = 0; c < C; ++c) acc[u][c] = b;
    }
    // A fragments in a register ring POL_PF k steps deep: the reads of k step s + POL_PF are issued before the
    // MFMAs of step s (the scheduling barriers keep the compiler from folding them back into read -> wait -> MFMA)
    constexpr int PF = POL_PF;
    bf16x8 ring[PF + 1][TG];
#pragma unroll
    for (int s = 0; s < PF && s < S; ++s)
#pragma unroll
      for (int u = 0; u < TG; ++u) ring[s][u] = w2s[((t + u) * S + s) * 64 + lane];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s + PF < S) {
#pragma unroll
        for (int u = 0; u < TG; ++u) ring[(s + PF) % (PF + 1)][u] = w2s[((t + u) * S + s + PF) * 64 + lane];
      }
#if POL_SB
      __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
      for (int u = 0; u < TG; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c)
          acc[u][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ring[POL_RING_IDX][u], h1[s][c], acc[u][c], 0, 0, 0);
#if POL_SB
      __builtin_amdgcn_sched_barrier(0);
#endif
#if POL_PIPE
      if (s == 0 && t > 0) drain(pend, t - TG);
#endif
    }
#if POL_PIPE
#pragma unroll
    for (int u = 0; u < TG; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) pend[u][c] = acc[u][c];
#else
    drain(acc, t);
#endif
  }
#if POL_PIPE
  drain(pend, T - TG);
#endif
  PSTAMP(3 + 4 * tile_k, __builtin_amdgcn_s_memtime);
  // Epilogue on all 64 lanes (lane map above): the accumulator lane e & 15 of column tile e >> 4 holds
  // output rows 0-3 of env e.
  const int nout = net.num_out, src = e_w & 15, ct = e_w >> 4;
  const int env = env0 + e_w;
  if (blockIdx.y == 1) {  // critic: the value (row 0)
    float v = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float t = __shfl(o[c][0], src, 64);
      v = ct == c ? t : v;
    }
    if (p == 0 && env < n) net.out[env] = v + net.b3[0];
    PSTAMP(4 + 4 * tile_k, __builtin_amdgcn_s_memtime);
    ++tile_k;
    continue;
  }
  float y[RPL];
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    float v = 0.0f;
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int pp = 0; pp < 4 / RPL; ++pp) {
        const float t = __shfl(o[c][RPL * pp + q], src, 64);
        v = ct == c && p == pp ? t : v;
      }
    const int r = RPL * p + q;
    y[q] = v + (r < nout ? net.b3[r] : 0.0f);
  }
  // actor: Normal(mean, std) sample and its log prob summed over the actions (torch Normal.log_prob:
  // -(x - mu)^2 / (2 var) - log(std) - log(sqrt(2 pi))).  One Philox block per env: rows 0, 1 from Box-Muller
  // on words (x, y), rows 2, 3 on (z, w); the lanes of an env draw the same block.  Box-Muller on the
  // hardware log2 / sin / cos / sqrt (v_sin / v_cos take revolutions: u2 in [0, 1) is the angle / 2 pi).
  const gr_u32x4 w = gr_philox4x32_10((uint32_t)(pa.env_id_offset + env), cnt, GR_TAG_POLICY, 0u, pa.seed_lo,
                                      pa.seed_hi);
  float z[RPL];
#pragma unroll
  for (int b = 0; b < (RPL + 1) / 2; ++b) {
    const int pair = (RPL * p) / 2 + b;  // 0: rows 0, 1; 1: rows 2, 3
    const float u1 = gr_u01_open0(pair ? w.z : w.x), u2 = gr_u01(pair ? w.w : w.y);
    const float rad = __builtin_amdgcn_sqrtf(-1.38629436f * __builtin_amdgcn_logf(u1));  // -2 ln u1
    const float zc = rad * __builtin_amdgcn_cosf(u2), zs = rad * __builtin_amdgcn_sinf(u2);
    if (RPL == 1) {
      z[0] = (p & 1) ? zs : zc;
    } else {
      z[2 * b] = zc;
      z[2 * b + 1] = zs;
    }
  }
  float act[RPL], lp = 0.0f;
#pragma unroll
  for (int q = 0; q < RPL; ++q) {
    act[q] = y[q] + sdv[q] * z[q];
    const float dlt = act[q] - y[q];
    if (RPL * p + q < nout) lp += lpc[q] - dlt * dlt * i2v[q];
  }
#pragma unroll
  for (int m = 16 * C; m < 64; m *= 2) lp += __shfl_xor(lp, m, 64);
  if (env < n) {
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
      const int r = RPL * p + q;
      if (r < nout) {
        net.out[(size_t)env * nout + r] = y[q];
        pa.actions[(size_t)env * nout + r] = act[q];
      }
    }
    if (p == 0) pa.log_prob[env] = lp;
  }
  PSTAMP(4 + 4 * tile_k, __builtin_amdgcn_s_memtime);
  ++tile_k;
  }  // env tiles
  PSTAMP(15, __builtin_amdgcn_s_memrealtime);
}

template <int H, int ACT>
static hipError_t launch_policy_t(const gr_policy_args& a, dim3 grid, size_t lds, hipStream_t s) {
  static bool lds_attr = false;  // up to 152 KB of dynamic LDS: above the default cap, set once
  if (!lds_attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&policy_kernel<H, ACT>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    lds_attr = true;
  }
  hipLaunchKernelGGL((policy_kernel<H, ACT>), grid, dim3(POL_WAVES * 64), lds, s, a);
  return hipGetLastError();
}

hipError_t read_policy_stamps(unsigned long long* host, int n) {
#ifdef GR_STAMPS
  if (n > POL_STAMP_WAVES * 16) n = POL_STAMP_WAVES * 16;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pol_stamps), (size_t)n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost);
#else
  (void)host;
  (void)n;
  return hipErrorNotSupported;
#endif
}

hipError_t launch_policy(const gr_policy_args& a, hipStream_t s) {
  const int envs_per_block = POL_WAVES * POL_ENVS_PER_WAVE;
  const int tiles = (a.num_envs + envs_per_block - 1) / envs_per_block;
  // one workgroup per CU (the weights fill its LDS), half of the CUs per network (all of them, actor only)
  const int nets = a.net[1].obs ? 2 : 1, per_net = POL_BLOCKS_PER_NET * (3 - nets);
  const dim3 grid(tiles < per_net ? tiles : per_net, nets);
  const size_t lds =
      ((size_t)a.hidden / 16 + (size_t)a.hidden * a.hidden / 512 + (size_t)a.hidden / 32) * 64 * 16 + 2 * 4 * (size_t)a.hidden;
  const bool elu = a.activation == GR_POLICY_ACT_ELU;
  if (a.hidden == 256)
    return elu ? launch_policy_t<256, GR_POLICY_ACT_ELU>(a, grid, lds, s)
               : launch_policy_t<256, GR_POLICY_ACT_LRELU>(a, grid, lds, s);
  return elu ? launch_policy_t<128, GR_POLICY_ACT_ELU>(a, grid, lds, s)
             : launch_policy_t<128, GR_POLICY_ACT_LRELU>(a, grid, lds, s);
}

}  // namespace gr
