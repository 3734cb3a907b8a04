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
#define POL_ENVS_PER_WAVE (16 * POL_COLS)

template <int ACT>
__device__ __forceinline__ float pol_act(float x) {
  // LeakyReLU (torch default slope 0.01) or ELU (alpha 1); compile-time, so the layer loops stay straight-line
  if constexpr (ACT == GR_POLICY_ACT_ELU) return x > 0.0f ? x : expm1f(x);
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
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = pol_act<ACT>(v[r]);
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
#ifndef POL_ABL_NOSTAGE
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
#endif
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
  // persistent over env tiles: the weights are staged once per workgroup
  const int envs_per_block = POL_WAVES * POL_ENVS_PER_WAVE;
  for (int base = blockIdx.x * envs_per_block; base < n; base += gridDim.x * envs_per_block) {
  const int env0 = base + wave * POL_ENVS_PER_WAVE;
  // layer-1 B fragments: obs^T, lane l holds obs[env0 + 16c + (l & 15)][8 (l >> 4) + j] (k < D, else 0).
  // Two unconditional float4 loads per lane and column tile (rows clamped into range, num_obs % 4 == 0),
  // all issued before the first is used.
  bf16x8 xb[C];
  {
    float4 ld[C][2];
    const int k0 = 8 * (lane >> 4);
    const int kc = k0 < D ? k0 : 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int env = env0 + 16 * c + (lane & 15);
      env = env < n ? env : n - 1;
      const float4* row = reinterpret_cast<const float4*>(net.obs + (size_t)env * D + kc);
      ld[c][0] = row[0];
      ld[c][1] = k0 + 4 < D ? row[1] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float v[8] = {ld[c][0].x, ld[c][0].y, ld[c][0].z, ld[c][0].w, ld[c][1].x, ld[c][1].y, ld[c][1].z, ld[c][1].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) xb[c][j] = (__bf16)(k0 + j < D ? v[j] : 0.0f);
    }
  }
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
  // ---- layer 2 (pairs of row tiles) fused with layer 3: out^T += W3[:, k step t/2] act(W2 h1^T + b2)
  f32x4 o[C];
#pragma unroll
  for (int c = 0; c < C; ++c) o[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  constexpr int TG = POL_TG;  // row tiles per group (even): TG x C independent accumulator chains
#pragma unroll
  for (int t = 0; t < T; t += TG) {
    f32x4 acc[TG][C];
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const f32x4 b = bias4(b2s, 16 * (t + u), lane);
#pragma unroll
      for (int c = 0; c < C; ++c) acc[u][c] = b;
    }
    // A fragments double-buffered in registers: the reads of k step s + 1 are issued before the MFMAs of
    // step s (the scheduling barriers keep the compiler from folding them back into read -> wait -> MFMA)
    bf16x8 acur[TG], anxt[TG];
#pragma unroll
    for (int u = 0; u < TG; ++u) acur[u] = w2s[((t + u) * S) * 64 + lane];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      if (s + 1 < S) {
#pragma unroll
        for (int u = 0; u < TG; ++u) anxt[u] = w2s[((t + u) * S + s + 1) * 64 + lane];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < TG; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c)
          acc[u][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(acur[u], h1[s][c], acc[u][c], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (s + 1 < S) {
#pragma unroll
        for (int u = 0; u < TG; ++u) acur[u] = anxt[u];
      }
    }
#pragma unroll
    for (int u = 0; u < TG; u += 2) {
      const bf16x8 a3 = w3s[((t + u) / 2) * 64 + lane];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        act4<ACT>(acc[u][c]);
        act4<ACT>(acc[u + 1][c]);
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a3, pack8(acc[u][c], acc[u + 1][c]), o[c], 0, 0, 0);
      }
    }
  }
  // Epilogue on all 64 lanes: lane L takes output row r = L >> 4 of env env0 + 16c + (L & 15) from lane L & 15
  // (which holds rows 0-3 in its accumulator registers).
  const int nout = net.num_out, r = lane >> 4, l16 = lane & 15;
  const float br = r < nout ? net.b3[r] : 0.0f;
  const float sd = blockIdx.y == 0 && r < nout ? pa.std[r] : 1.0f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float v0 = __shfl(o[c][0], l16, 64), v1 = __shfl(o[c][1], l16, 64);
    const float v2 = __shfl(o[c][2], l16, 64), v3 = __shfl(o[c][3], l16, 64);
    const float y = (r == 0 ? v0 : r == 1 ? v1 : r == 2 ? v2 : v3) + br;
    const int env = env0 + 16 * c + l16;
    const bool live = env < n && r < nout;
    if (blockIdx.y == 1) {  // critic: the value
      if (live) net.out[env] = y;
      continue;
    }
    // actor: Normal(mean, std) sample and its log prob summed over the actions (torch Normal.log_prob:
    // -(x - mu)^2 / (2 var) - log(std) - log(sqrt(2 pi))).  The env's four lanes draw the same Philox block.
    const gr_u32x4 w = gr_philox4x32_10((uint32_t)(pa.env_id_offset + env), cnt, GR_TAG_POLICY, 0u, pa.seed_lo,
                                        pa.seed_hi);
    float z0, z1;
    gr_box_muller(r < 2 ? w.x : w.z, r < 2 ? w.y : w.w, &z0, &z1);
    const float eps = (r & 1) ? z1 : z0;
    const float a = y + sd * eps;
    const float dlt = a - y;
    float lp = r < nout ? -(dlt * dlt) / (2.0f * (sd * sd)) - logf(sd) - 0.91893853320467274f : 0.0f;
    lp += __shfl_xor(lp, 16, 64);
    lp += __shfl_xor(lp, 32, 64);
#ifdef POL_ABL_NOEPI
    if (live && a == 12345.0f) {
#else
    if (live) {
#endif
      net.out[(size_t)env * nout + r] = y;
      pa.actions[(size_t)env * nout + r] = a;
      if (r == 0) pa.log_prob[env] = lp;
    }
  }
  }  // env tiles
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

hipError_t launch_policy(const gr_policy_args& a, hipStream_t s) {
  const int envs_per_block = POL_WAVES * POL_ENVS_PER_WAVE;
  const int tiles = (a.num_envs + envs_per_block - 1) / envs_per_block;
  // one workgroup per CU (the weights fill its LDS), half of the CUs per network
  const dim3 grid(tiles < POL_BLOCKS_PER_NET ? tiles : POL_BLOCKS_PER_NET, 2);
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
