// gr_policy_f32.hip — rollout inference of the rsl_rl ActorCritic at the reference's precision: fp32
// operands on v_mfma_f32_16x16x4_f32 (gfx950), every dot product an fp32 fmaf chain (no bf16, no xf32).
//
// Reference: PPO.act (standalone/rsl_rl/ext/algorithms/ppo.py:71-85) -> ActorCritic.act / evaluate /
// get_actions_log_prob on the fp32 MLPs num_obs -> H -> H -> num_out (rsl_rl_ppo_cfg.py:15-41).  Same
// outputs, sampling stream and call-counter contract as the bf16 kernel (gr_policy.hip), so the two are
// interchangeable behind gr_policy_forward (gr_policy_args.precision).
//
// Why a different layout from the bf16 kernel: fp32 W2 is 256 KB at H = 256 and does not fit the 160 KB
// LDS.  Instead every wave keeps ITS slice of W2 in registers for the whole launch:
//   - a workgroup = 8 waves (2 per SIMD), persistent over 16 C-env tiles; wave w owns hidden rows
//     [H/8 w, H/8 (w + 1)) of both hidden layers (H/128 16-row tiles);
//   - layer 1: wave w computes its h1 rows for the tile (A = W1 rows from registers, B = obs^T from
//     global) and stores them transposed into LDS ([env][H + 4] floats);
//   - layer 2: wave w computes its h2 rows; A = its W2 rows from registers (128 VGPRs at H = 256), B = all
//     of h1 from LDS as float4 reads (one ds_read_b128 = the B fragments of 4 k steps);
//   - layer 3: wave w's partial out = W3[:, its rows] h2 (MFMA on the accumulators in place), summed over
//     the 8 waves in LDS in a fixed order by the epilogue waves of the NEXT tile (one barrier per tile).
// The k order: the MFMA's lane l (g = l >> 4, j = l & 15) holds A[row j][k = g] and B[k = g][env j]; the
// C tile holds rows 4 g + r of column j in register r.  So k step 4 q + r of a layer is hidden unit
// (or input) 16 q + 4 g + r: register r of the previous layer's accumulator, register r of a float4 read
// of LDS, element r of a float4 load of a W row.  No host-side packing: W1, W2, W3 are the module's
// row-major fp32 weights.
#include <hip/hip_runtime.h>

#include "../../include/gr.h"
#include "gr_kernels.h"
#include "gr_rng.h"

namespace gr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define PF_WAVES 8  // 2 per SIMD: each holds 256 registers, its W2 slice uses 128 of them at H = 256
#ifndef PF_COLS
#define PF_COLS 4  // 16-env column tiles per workgroup tile (4: one barrier per 64 envs, 1-2 % faster than 2)
#endif
#ifndef PF_BLOCKS_PER_NET
#define PF_BLOCKS_PER_NET 128  // one workgroup per CU (the registers hold one), half the CUs per network
#endif
static_assert(PF_COLS >= 1 && PF_COLS <= PF_WAVES, "one epilogue wave per column tile");

template <int ACT>
__device__ __forceinline__ float act_f32(float x) {
  // torch: leaky_relu x > 0 ? x : x * slope; elu x > 0 ? x : expm1(x) (alpha = scale = 1)
  if constexpr (ACT == GR_POLICY_ACT_ELU) return x > 0.0f ? x : expm1f(x);
  return x > 0.0f ? x : x * 0.01f;
}

template <int ACT>
__device__ __forceinline__ void act4_f32(f32x4& v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = act_f32<ACT>(v[r]);
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// LDS of one workgroup (floats): h1 [2][E][H + 4], wave partials [2][PF_WAVES][E][4], b1 [H], b2 [H]
constexpr size_t policy_f32_lds_bytes(int h, int cols) {
  return 4 * ((size_t)2 * 16 * cols * (h + 4) + 2 * PF_WAVES * 16 * cols * 4 + 2 * h);
}

template <int H, int ACT, int Q1>
__global__ __launch_bounds__(PF_WAVES * 64) void policy_f32_kernel(gr_policy_args pa) {
  constexpr int C = PF_COLS, E = 16 * C;   // envs per workgroup tile
  constexpr int TW = H / (16 * PF_WAVES);  // 16-row tiles per wave and hidden layer
  constexpr int Q = H / 16;                // 16-unit groups of a hidden layer (4 k steps each)
  constexpr int HP = H + 4;                // h1 row stride: float4 reads of 16 envs hit 16 distinct bank quads
  static_assert(TW >= 1, "H >= 128");
  const gr_policy_net& net = pa.net[blockIdx.y];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int n = pa.num_envs, D = net.num_obs, nout = net.num_out;
  extern __shared__ float lds[];
  float* h1s = lds;                                  // [2][E][HP]
  float* parts = h1s + 2 * E * HP;                   // [2][PF_WAVES][E][4]
  float* b1s = parts + 2 * PF_WAVES * E * 4;         // [H]
  float* b2s = b1s + H;                              // [H]
  const float* __restrict__ W1 = static_cast<const float*>(net.w1);
  const float* __restrict__ W2 = static_cast<const float*>(net.w2);
  const float* __restrict__ W3 = static_cast<const float*>(net.w3);

  // ---- this wave's weights, in registers for the whole launch
  float w1r[TW][Q1][4], w2r[TW][4 * Q], w3r[TW][4];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = 16 * (wave * TW + t) + j;
#pragma unroll
    for (int q = 0; q < Q1; ++q) {
      const int k = 16 * q + 4 * g;
      const f32x4 v = k < D ? ld4(W1 + (size_t)row * D + k) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int r = 0; r < 4; ++r) w1r[t][q][r] = v[r];
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const f32x4 v = ld4(W2 + (size_t)row * H + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) w2r[t][4 * q + r] = v[r];
    }
    const f32x4 v3 = j < nout ? ld4(W3 + (size_t)j * H + 16 * (wave * TW + t) + 4 * g) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int r = 0; r < 4; ++r) w3r[t][r] = v3[r];
  }
  for (int i = threadIdx.x; i < H; i += PF_WAVES * 64) {
    b1s[i] = net.b1[i];
    b2s[i] = net.b2[i];
  }
  const uint32_t cnt = pa.counters[pa.counter_index];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) pa.counters[pa.counter_index ^ 1] = cnt + 1u;
  // epilogue constants: lane (g, j) takes output row g of env j of its column tile
  const bool actor = blockIdx.y == 0;
  const float sdv = actor && g < nout ? pa.std[g] : 1.0f;
  const float i2v = 1.0f / (2.0f * sdv * sdv), lpc = -logf(sdv) - 0.91893853320467274f;
  const float b3v = g < nout ? net.b3[g] : 0.0f;

  // layer-1 B fragments: lane (g, j) of column c holds obs[env 16 c + j][16 q + 4 g + r] in element r
  const int stride = gridDim.x * E;
  f32x4 xo[C][Q1];
  auto load_obs = [&](int base) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      int env = base + 16 * c + j;
      env = env < n ? env : n - 1;
#pragma unroll
      for (int q = 0; q < Q1; ++q) {
        const int k = 16 * q + 4 * g;
        xo[c][q] = k < D ? ld4(net.obs + (size_t)env * D + k) : (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
      }
    }
  };
  // the epilogue of tile kt (8-wave partial sums -> mean / value, sampling, log prob, stores): column tile
  // e is taken by wave (2 kt + e) mod 8, so the extra work rotates over the waves
  auto epilogue = [&](int kt, int base) {
    const int e = (wave - 2 * kt) & (PF_WAVES - 1);
    if (e >= C) return;
    const float* pp = parts + (size_t)(kt & 1) * PF_WAVES * E * 4 + (16 * e + j) * 4 + g;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < PF_WAVES; ++w) v += pp[w * E * 4];
    const int env = base + 16 * e + j;
    if (!actor) {
      if (g == 0 && env < n) net.out[env] = v + b3v;
      return;
    }
    const float y = v + b3v;
    // Normal(mean, std) sample, the bf16 kernel's stream: one Philox block per env, rows 0 / 1 from
    // Box-Muller on words (x, y), rows 2 / 3 on (z, w)
    const gr_u32x4 w = gr_philox4x32_10((uint32_t)(pa.env_id_offset + env), cnt, GR_TAG_POLICY, 0u, pa.seed_lo,
                                        pa.seed_hi);
    const float u1 = gr_u01_open0(g >> 1 ? w.z : w.x), u2 = gr_u01(g >> 1 ? w.w : w.y);
    const float rad = __builtin_amdgcn_sqrtf(-1.38629436f * __builtin_amdgcn_logf(u1));
    const float z = rad * ((g & 1) ? __builtin_amdgcn_sinf(u2) : __builtin_amdgcn_cosf(u2));
    const float a = y + sdv * z, dlt = a - y;
    float lp = g < nout ? lpc - dlt * dlt * i2v : 0.0f;
    lp += __shfl_xor(lp, 16, 64);
    lp += __shfl_xor(lp, 32, 64);
    if (env < n) {
      if (g < nout) {
        net.out[(size_t)env * nout + g] = y;
        pa.actions[(size_t)env * nout + g] = a;
      }
      if (g == 0) pa.log_prob[env] = lp;
    }
  };

  // ---- per tile: layer 1 -> LDS, layer 2 from LDS, layer 3 partial -> LDS; the epilogue of the previous tile
  // after the barrier.  (Interleaving the next tile's layer 1 into this tile's layer-2 stream was measured 2 %
  // slower, 169 -> 172 us; DESIGN 4e'.)
  auto layer1_store = [&](float* h1dst, f32x4 (&y)[TW][C]) {
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        act4_f32<ACT>(y[t][c]);
        *reinterpret_cast<f32x4*>(h1dst + (16 * c + j) * HP + 16 * (wave * TW + t) + 4 * g) = y[t][c];
      }
  };
  auto layer1_init = [&](f32x4 (&y)[TW][C]) {
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const f32x4 bb = ld4(b1s + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
      for (int c = 0; c < C; ++c) y[t][c] = bb;
    }
  };
  // k step kk (< 4 Q1) of layer 1 for every row tile and column
  auto layer1_step = [&](int kk, const f32x4 (&x)[C][Q1], f32x4 (&y)[TW][C]) {
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < C; ++c) y[t][c] = mfma4(w1r[t][kk >> 2][kk & 3], x[c][kk >> 2][kk & 3], y[t][c]);
  };
  // layer 2 of the tile in h1, layer 3 partial into parts[slot]
  auto layer23 = [&](const float* h1, int slot) {
    f32x4 acc[TW][C];
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const f32x4 bb = ld4(b2s + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
      for (int c = 0; c < C; ++c) acc[t][c] = bb;
    }
    f32x4 hb[2][C];
#pragma unroll
    for (int c = 0; c < C; ++c) hb[0][c] = ld4(h1 + (16 * c + j) * HP + 4 * g);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (q + 1 < Q) {
#pragma unroll
        for (int c = 0; c < C; ++c) hb[(q + 1) & 1][c] = ld4(h1 + (16 * c + j) * HP + 16 * (q + 1) + 4 * g);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int c = 0; c < C; ++c) acc[t][c] = mfma4(w2r[t][4 * q + r], hb[q & 1][c][r], acc[t][c]);
    }
    f32x4 o[C];
#pragma unroll
    for (int c = 0; c < C; ++c) o[c] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < C; ++c) {
        act4_f32<ACT>(acc[t][c]);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[c] = mfma4(w3r[t][r], acc[t][c][r], o[c]);
      }
    // rows 0-3 of the output tile live in lanes 0-15 (g = 0)
    if (g == 0) {
#pragma unroll
      for (int c = 0; c < C; ++c)
        *reinterpret_cast<f32x4*>(parts + ((size_t)(slot * PF_WAVES + wave) * E + 16 * c + j) * 4) = o[c];
    }
  };

  load_obs(blockIdx.x * E);
  __syncthreads();  // biases staged
  int kt = 0, prev_base = 0;
  for (int base = blockIdx.x * E; base < n; base += stride, ++kt) {
    float* h1 = h1s + (kt & 1) * E * HP;
    f32x4 x[C][Q1], y1[TW][C];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int q = 0; q < Q1; ++q) x[c][q] = xo[c][q];
    if (base + stride < n) load_obs(base + stride);
    // ---- layer 1: this wave's h1 rows for the tile -> LDS (transposed: [env][unit])
    layer1_init(y1);
#pragma unroll
    for (int kk = 0; kk < 4 * Q1; ++kk) layer1_step(kk, x, y1);
    layer1_store(h1, y1);
    __syncthreads();  // h1 of tile kt complete; the partials of tile kt - 1 complete
    if (kt > 0) epilogue(kt - 1, prev_base);
    layer23(h1, kt & 1);
    prev_base = base;
  }
  __syncthreads();
  if (kt > 0) epilogue(kt - 1, prev_base);
}

template <int H, int ACT, int Q1>
static hipError_t launch_policy_f32_t(const gr_policy_args& a, dim3 grid, hipStream_t s) {
  const size_t lds = policy_f32_lds_bytes(H, PF_COLS);
  static bool lds_attr = false;  // above the default 64 KB dynamic-LDS cap: set once
  if (!lds_attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&policy_f32_kernel<H, ACT, Q1>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    lds_attr = true;
  }
  hipLaunchKernelGGL((policy_f32_kernel<H, ACT, Q1>), grid, dim3(PF_WAVES * 64), lds, s, a);
  return hipGetLastError();
}

template <int H, int ACT>
static hipError_t launch_policy_f32_h(const gr_policy_args& a, dim3 grid, hipStream_t s) {
  // the layer-1 k depth: one 16-input group when both networks read <= 16 observations, else two
  const int d1 = a.net[1].obs ? a.net[1].num_obs : 0;
  const int d = a.net[0].num_obs > d1 ? a.net[0].num_obs : d1;
  return d <= 16 ? launch_policy_f32_t<H, ACT, 1>(a, grid, s) : launch_policy_f32_t<H, ACT, 2>(a, grid, s);
}

hipError_t launch_policy_f32(const gr_policy_args& a, hipStream_t s) {
  const int envs_per_block = 16 * PF_COLS;
  const int tiles = (a.num_envs + envs_per_block - 1) / envs_per_block;
  const int nets = a.net[1].obs ? 2 : 1, per_net = PF_BLOCKS_PER_NET * (3 - nets);  // actor only: every CU
  const dim3 grid(tiles < per_net ? tiles : per_net, nets);
  const bool elu = a.activation == GR_POLICY_ACT_ELU;
  if (a.hidden == 256)
    return elu ? launch_policy_f32_h<256, GR_POLICY_ACT_ELU>(a, grid, s) : launch_policy_f32_h<256, GR_POLICY_ACT_LRELU>(a, grid, s);
  return elu ? launch_policy_f32_h<128, GR_POLICY_ACT_ELU>(a, grid, s) : launch_policy_f32_h<128, GR_POLICY_ACT_LRELU>(a, grid, s);
}

}  // namespace gr
