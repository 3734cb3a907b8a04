// gr_bn.hip — training-mode BatchNorm fused with its activation, on channels-last rows [M][C] (gfx950).
//
// The vision stem (VisionActorCritic, standalone/rsl_rl/ext/modules/vision_actor_critic.py:43-144, here
// rsl_rl/vision_actor_critic.py) runs Conv -> BatchNorm2d -> LeakyReLU three times on [batch*H*W, C]
// matrices with millions of rows and C = 16 / 32 / 64.  PyTorch spends 13 full passes over each such
// matrix per forward + backward (statistics, transform, activation, activation backward, BN backward
// reduce and element passes) and saves both the BN output and the activation output.  Here:
//   forward:  one statistics pass (read x) + one apply pass (read x, write y = act(bn(x)));
//   backward: one reduce pass (read gy, x) + one element pass (read gy, x, write gx);
// the activation's derivative is recomputed from x, so only x is kept for the backward.
//
// Layout: a thread owns one float4 (4 channels) of a row per item and walks the rows with a stride that
// is a multiple of C / 4, so its channel group is fixed (C / 4 must be a power of two dividing 256: C in
// {4, 8, 16, 32, 64}).  Per-channel sums: fp32 per thread over its items, shifted by the channel's value in
// row 0 (no cancellation in E[x^2] - E[x]^2), then fp64 across the block and across blocks in a fixed
// order — deterministic, no atomics, graph-capturable.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/gr.h"
#include "gr_kernels.h"

namespace gr {

constexpr int BN_THREADS = 256;
#ifndef GR_BN_MAX_BLOCKS
#define GR_BN_MAX_BLOCKS 1024
#endif
constexpr int BN_MAX_BLOCKS = GR_BN_MAX_BLOCKS;  // blocks per pass (partial rows of the fixed-order reductions)

__host__ __device__ inline int bn_blocks(long long m, int c) {
  const long long q = m * (c / 4);
  long long b = (q + BN_THREADS * 8 - 1) / (BN_THREADS * 8);  // ~8 float4 per thread at least
  if (b < 1) b = 1;
  return (int)(b < BN_MAX_BLOCKS ? b : BN_MAX_BLOCKS);
}

template <int ACT>
__device__ __forceinline__ float bn_act(float z, float slope) {
  if constexpr (ACT == GR_POLICY_ACT_ELU) return z > 0.0f ? z : expm1f(z);
  return z > 0.0f ? z : z * slope;
}
// d act / d z, from z (torch's leaky_relu_backward tests the input; ELU's uses the output y = expm1(z))
template <int ACT>
__device__ __forceinline__ float bn_dact(float z, float slope) {
  if constexpr (ACT == GR_POLICY_ACT_ELU) return z > 0.0f ? 1.0f : expm1f(z) + 1.0f;
  return z > 0.0f ? 1.0f : slope;
}

__device__ __forceinline__ float4 ld4f(const float* p, long long q) { return reinterpret_cast<const float4*>(p)[q]; }
__device__ __forceinline__ float comp(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// block reduction of 8 per-thread sums (two quantities x 4 channels) over the threads of each channel group,
// in fp64, then one row of partials per block: part[block][2][C]
__device__ void bn_block_partials(const float a[8], int c, double* part) {
  __shared__ double red[BN_THREADS * 8];
  const int t = threadIdx.x, c4 = c / 4;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[k * BN_THREADS + t] = (double)a[k];
  __syncthreads();
  // thread (quantity s, channel ch) sums the threads t' with t' % c4 == ch / 4 in index order
  for (int j = t; j < 2 * c; j += BN_THREADS) {
    const int s = j / c, ch = j % c, g = ch / 4, k = ch % 4;
    double acc = 0.0;
    for (int u = g; u < BN_THREADS; u += c4) acc += red[(s * 4 + k) * BN_THREADS + u];
    part[(size_t)blockIdx.x * 2 * c + j] = acc;
  }
}

// ---- forward: shifted channel sums of x
__global__ __launch_bounds__(BN_THREADS) void bn_stats_partial(const float* __restrict__ x, long long m, int c,
                                                               double* __restrict__ part) {
  const int c4 = c / 4;
  const long long q0 = (long long)blockIdx.x * BN_THREADS + threadIdx.x, stride = (long long)gridDim.x * BN_THREADS;
  const long long nq = m * c4;
  const float4 sh = ld4f(x, threadIdx.x & (c4 - 1));  // row 0 of this thread's channel group
  float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (long long q = q0; q < nq; q += stride) {
    const float4 v = ld4f(x, q);
    const float d[4] = {v.x - sh.x, v.y - sh.y, v.z - sh.z, v.w - sh.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] += d[k];
      a[4 + k] += d[k] * d[k];
    }
  }
  bn_block_partials(a, c, part);
}

// sums over the blocks' partials of `npairs` quantities (part[block][npairs]), in a fixed order: thread
// (pair j, lane k) of the BN_FINAL_THREADS sums the partials b = k (mod T), T = BN_FINAL_THREADS / npairs
// threads per pair, 32 (then 8) loads in flight at a time (the partials come from L2 / HBM: one load at a time left
// a 1 024-block reduction latency-bound at ~70 us), then lane 0 of each pair adds the T lane sums in order.
// Thread index = k * npairs + j: consecutive threads read consecutive pairs of one partial row (coalesced; with
// j = t / T a wave's load touched 16 rows, and the final took ~30 us for 1 024 rows of 32 pairs)
constexpr int BN_FINAL_THREADS = 1024;
__device__ void bn_final_sums(const double* __restrict__ part, int npairs, int blocks, double* out, int stride = 0) {
  __shared__ double red[BN_FINAL_THREADS];
  if (stride == 0) stride = npairs;  // (the partial rows' length, when the pairs are a slice of a longer row)
  const int T = BN_FINAL_THREADS / npairs, j = threadIdx.x % npairs, k = threadIdx.x / npairs;
  double acc = 0.0;
  if (k < T) {
    int b = k;
    // 32 loads in flight: the partials were just written by blocks on every XCD, so each round trip is a
    // far-memory latency (8 at a time left the final at ~29 us for 1 024 partial rows, profiles/round05_*)
    for (; b + 31 * T < blocks; b += 32 * T) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = part[(size_t)(b + u * T) * stride + j];
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
    for (; b + 7 * T < blocks; b += 8 * T) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(b + u * T) * stride + j];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += v[u];
    }
    for (; b < blocks; b += T) acc += part[(size_t)b * stride + j];
    red[j * T + k] = acc;
  }
  __syncthreads();
  if (j < npairs && k == 0) {
    double s = 0.0;
    for (int u = 0; u < T; ++u) s += red[j * T + u];
    out[j] = s;
  }
  __syncthreads();
}

// stats[0][c] mean, [1][c] invstd = 1 / sqrt(var + eps), [2][c] biased var, [3][c] unbiased var
// shift[c]: the per-channel shift of the partial sums (row 0 of x)
__global__ __launch_bounds__(BN_FINAL_THREADS) void bn_stats_final(const float* __restrict__ shift, long long m, int c, int blocks,
                                                             float eps, const double* __restrict__ part,
                                                             float* __restrict__ stats) {
  __shared__ double sums[128];
  bn_final_sums(part, 2 * c, blocks, sums);
  const int ch = threadIdx.x;
  if (ch >= c) return;
  const double md = (double)m, d1 = sums[ch] / md;
  double var = sums[c + ch] / md - d1 * d1;
  var = var > 0.0 ? var : 0.0;
  const float varf = (float)var;
  stats[ch] = (float)((double)shift[ch] + d1);
  stats[c + ch] = 1.0f / sqrtf(varf + eps);
  stats[2 * c + ch] = varf;
  stats[3 * c + ch] = m > 1 ? (float)(var * md / (md - 1.0)) : varf;
}

// ---- forward: y = act((x - mean) * invstd * w + b)
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void bn_apply(const float* __restrict__ x, long long m, int c,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       const float* __restrict__ stats, float slope, float* __restrict__ y) {
  const int c4 = c / 4, g = threadIdx.x & (c4 - 1);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + c, g), wv = ld4f(w, g), bv = ld4f(b, g);
  const long long nq = m * c4, stride = (long long)gridDim.x * BN_THREADS;
  for (long long q = (long long)blockIdx.x * BN_THREADS + threadIdx.x; q < nq; q += stride) {
    const float4 v = ld4f(x, q);
    float4 o;
    o.x = bn_act<ACT>((v.x - mu.x) * is.x * wv.x + bv.x, slope);
    o.y = bn_act<ACT>((v.y - mu.y) * is.y * wv.y + bv.y, slope);
    o.z = bn_act<ACT>((v.z - mu.z) * is.z * wv.z + bv.z, slope);
    o.w = bn_act<ACT>((v.w - mu.w) * is.w * wv.w + bv.w, slope);
    reinterpret_cast<float4*>(y)[q] = o;
  }
}

// ---- backward: per channel sum(gz), sum(gz * xhat), gz = gy * act'(z)
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_partial(const float* __restrict__ x, const float* __restrict__ gy,
                                                             long long m, int c, const float* __restrict__ w,
                                                             const float* __restrict__ b, const float* __restrict__ stats,
                                                             float slope, double* __restrict__ part) {
  const int c4 = c / 4, g = threadIdx.x & (c4 - 1);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + c, g), wv = ld4f(w, g), bv = ld4f(b, g);
  const long long nq = m * c4, stride = (long long)gridDim.x * BN_THREADS;
  float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (long long q = (long long)blockIdx.x * BN_THREADS + threadIdx.x; q < nq; q += stride) {
    const float4 v = ld4f(x, q), dy = ld4f(gy, q);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (comp(v, k) - comp(mu, k)) * comp(is, k);
      const float gz = comp(dy, k) * bn_dact<ACT>(xh * comp(wv, k) + comp(bv, k), slope);
      a[k] += gz;
      a[4 + k] += gz * xh;
    }
  }
  bn_block_partials(a, c, part);
}

// sums[0][c] = sum gz (= grad bias), sums[1][c] = sum gz * xhat (= grad weight)
__global__ __launch_bounds__(BN_FINAL_THREADS) void bn_bwd_final(int c, int blocks, const double* __restrict__ part,
                                                           float* __restrict__ gw, float* __restrict__ gb,
                                                           float* __restrict__ sums) {
  __shared__ double tot[128];
  bn_final_sums(part, 2 * c, blocks, tot);
  const int ch = threadIdx.x;
  if (ch >= c) return;
  sums[ch] = (float)tot[ch];
  sums[c + ch] = (float)tot[c + ch];
  gb[ch] = (float)tot[ch];
  gw[ch] = (float)tot[c + ch];
}

// gx = (gz - sum(gz) / M - xhat * sum(gz xhat) / M) * invstd * w
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void bn_bwd_elemt(const float* __restrict__ x, const float* __restrict__ gy,
                                                           long long m, int c, const float* __restrict__ w,
                                                           const float* __restrict__ b, const float* __restrict__ stats,
                                                           const float* __restrict__ sums, float slope,
                                                           float* __restrict__ gx) {
  const int c4 = c / 4, g = threadIdx.x & (c4 - 1);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + c, g), wv = ld4f(w, g), bv = ld4f(b, g);
  const float inv_m = 1.0f / (float)m;
  const float4 s1 = ld4f(sums, g), s2 = ld4f(sums + c, g);
  const float mg[4] = {s1.x * inv_m, s1.y * inv_m, s1.z * inv_m, s1.w * inv_m};
  const float mgx[4] = {s2.x * inv_m, s2.y * inv_m, s2.z * inv_m, s2.w * inv_m};
  const long long nq = m * c4, stride = (long long)gridDim.x * BN_THREADS;
  for (long long q = (long long)blockIdx.x * BN_THREADS + threadIdx.x; q < nq; q += stride) {
    const float4 v = ld4f(x, q), dy = ld4f(gy, q);
    float o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = (comp(v, k) - comp(mu, k)) * comp(is, k);
      const float gz = comp(dy, k) * bn_dact<ACT>(xh * comp(wv, k) + comp(bv, k), slope);
      o[k] = (gz - mg[k] - xh * mgx[k]) * (comp(is, k) * comp(wv, k));
    }
    reinterpret_cast<float4*>(gx)[q] = make_float4(o[0], o[1], o[2], o[3]);
  }
}

int bn_scratch_doubles(long long m, int c) { return bn_blocks(m, c) * 2 * c + 2 * c; }

// the running-statistics update of `uses` training-mode forwards over the same rows (F.batch_norm's, as
// fused_bn._update_running made it with torch's ops: r = r * keep, then r + momentum * batch stat, per forward), and
// num_batches_tracked + count: one launch instead of five per BatchNorm and forward
__global__ void bn_running_update(float* __restrict__ rm, float* __restrict__ rv, long long* __restrict__ nbt,
                                  const float* __restrict__ stats, int c, float keep, float momentum, int uses,
                                  int count) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < c) {
    const float mean = stats[j], var = stats[3 * c + j];
    float a = rm[j], v = rv[j];
    for (int u = 0; u < uses; ++u) {
      a = __fmaf_rn(momentum, mean, a * keep);
      v = __fmaf_rn(momentum, var, v * keep);
    }
    rm[j] = a;
    rv[j] = v;
  }
  if (j == 0 && nbt) nbt[0] += count;
}

hipError_t launch_bn_running_update(float* rm, float* rv, long long* nbt, const float* stats, int c, float keep,
                                    float momentum, int uses, int count, hipStream_t s) {
  hipLaunchKernelGGL(bn_running_update, dim3((c + 63) / 64), dim3(64), 0, s, rm, rv, nbt, stats, c, keep, momentum,
                     uses, count);
  return hipGetLastError();
}

hipError_t launch_bn_forward(const float* x, long long m, int c, const float* w, const float* b, float eps, int act,
                             float slope, float* y, float* stats, double* part, hipStream_t s) {
  const int nb = bn_blocks(m, c);
  hipLaunchKernelGGL(bn_stats_partial, dim3(nb), dim3(BN_THREADS), 0, s, x, m, c, part);
  hipLaunchKernelGGL(bn_stats_final, dim3(1), dim3(BN_FINAL_THREADS), 0, s, x, m, c, nb, eps, part, stats);  // shift: row 0 of x
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(bn_apply<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, m, c, w, b, stats, slope, y);
  else
    hipLaunchKernelGGL(bn_apply<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, m, c, w, b, stats, slope, y);
  return hipGetLastError();
}

hipError_t launch_bn_stats(const float* x, long long m, int c, float eps, float* stats, double* part, hipStream_t s) {
  const int nb = bn_blocks(m, c);
  hipLaunchKernelGGL(bn_stats_partial, dim3(nb), dim3(BN_THREADS), 0, s, x, m, c, part);
  hipLaunchKernelGGL(bn_stats_final, dim3(1), dim3(BN_FINAL_THREADS), 0, s, x, m, c, nb, eps, part, stats);
  return hipGetLastError();
}

hipError_t launch_bn_backward(const float* x, const float* gy, long long m, int c, const float* w, const float* b,
                              const float* stats, int act, float slope, float* gx, float* gw, float* gb, double* part,
                              hipStream_t s) {
  const int nb = bn_blocks(m, c);
  // the two channel sums live after the partials in the same workspace (as floats)
  float* sums = reinterpret_cast<float*>(part + (size_t)nb * 2 * c);
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(bn_bwd_partial<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, gy, m, c, w, b, stats, slope, part);
  else
    hipLaunchKernelGGL(bn_bwd_partial<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, gy, m, c, w, b, stats, slope, part);
  hipLaunchKernelGGL(bn_bwd_final, dim3(1), dim3(BN_FINAL_THREADS), 0, s, c, nb, part, gw, gb, sums);
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(bn_bwd_elemt<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, gy, m, c, w, b, stats, sums, slope, gx);
  else
    hipLaunchKernelGGL(bn_bwd_elemt<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, s, x, gy, m, c, w, b, stats, sums, slope, gx);
  return hipGetLastError();
}

// ------------------------------------------------------------- the stem's first block from the image
// Conv2d(1, C, 3, stride 3, no bias) -> BatchNorm2d -> act of VisionActorCritic.stem_gemm, evaluated from
// the depth image itself: row r of the conv output is W1 . patch(r), patch(r) the 9 pixels of a 3 x 3 cell
// (pixel tables in the row order of stem_gemm: nimg x na rows of table a, then nimg x nb rows of table b, so
// conv2's input stays a view of y).  Neither the patch matrix nor the conv output is ever written: the
// statistics pass and the apply pass recompute the 36 FMAs of a thread's 4 channels, and so do the backward
// passes, which end in the conv weight's gradient (the image needs none) instead of writing gx.
constexpr int STEM_MAX_CELLS = 1024;  // na + nbt (768 at 72 x 96)

// image b's pixels: row rows[b] of obs when the batch is read through an index, else row b
__device__ __forceinline__ const float* stem_img(const Stem1& s, long long b) {
  return s.obs + (s.rows ? s.rows[b] : b) * s.ld + s.off;
}
__device__ __forceinline__ void stem_stage_table(const Stem1& s, short* tab) {
  for (int i = threadIdx.x; i < (s.na + s.nbt) * 9; i += BN_THREADS) tab[i] = s.pix[i];
  __syncthreads();
}
__device__ __forceinline__ void stem_pixels(const Stem1& s, const short* tab, unsigned r, float px[9]) {
  const unsigned ra = (unsigned)s.nimg * (unsigned)s.na;
  unsigned b, p;
  if (r < ra) {
    b = r / (unsigned)s.na;
    p = r - b * (unsigned)s.na;
  } else {
    const unsigned q = r - ra;
    b = q / (unsigned)s.nbt;
    p = (unsigned)s.na + (q - b * (unsigned)s.nbt);
  }
  const float* img = stem_img(s, b);
  const short* t = tab + p * 9;
#pragma unroll
  for (int k = 0; k < 9; ++k) px[k] = img[t[k]];
}
// the thread's 4 conv outputs (channels 4 g .. 4 g + 3), k-ordered fp32 FMA chains
__device__ __forceinline__ void stem_conv(const float w[4][9], const float px[9], float x[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float a = w[j][0] * px[0];
#pragma unroll
    for (int k = 1; k < 9; ++k) a = __builtin_fmaf(w[j][k], px[k], a);
    x[j] = a;
  }
}
__device__ __forceinline__ void stem_load_w(const Stem1& s, int g, float w[4][9]) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 9; ++k) w[j][k] = s.w[(4 * g + j) * 9 + k];
}

// forward statistics: shifted channel sums of the conv output; block 0 also writes the shift (row 0)
__global__ __launch_bounds__(BN_THREADS) void stem1_stats_partial(Stem1 s, double* __restrict__ part,
                                                                  float* __restrict__ shift) {
  __shared__ short tab[STEM_MAX_CELLS * 9];
  stem_stage_table(s, tab);
  const int c4 = s.c / 4, g = threadIdx.x & (c4 - 1);
  float w[4][9], px[9], sh[4], x[4];
  stem_load_w(s, g, w);
  stem_pixels(s, tab, 0u, px);
  stem_conv(w, px, sh);
  if (blockIdx.x == 0 && threadIdx.x < c4)
    for (int j = 0; j < 4; ++j) shift[4 * g + j] = sh[j];
  const unsigned m = (unsigned)s.nimg * (unsigned)(s.na + s.nbt);
  const unsigned step = gridDim.x * BN_THREADS / c4;
  float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (unsigned r = (blockIdx.x * BN_THREADS + threadIdx.x) / c4; r < m; r += step) {
    stem_pixels(s, tab, r, px);
    stem_conv(w, px, x);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float d = x[j] - sh[j];
      a[j] += d;
      a[4 + j] += d * d;
    }
  }
  bn_block_partials(a, s.c, part);
}

// forward apply: y[r][4 g + j] = act((x - mean) * invstd * w + b)
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void stem1_apply(Stem1 s, const float* __restrict__ bw, const float* __restrict__ bb,
                                                          const float* __restrict__ stats, float slope, float* __restrict__ y) {
  __shared__ short tab[STEM_MAX_CELLS * 9];
  stem_stage_table(s, tab);
  const int c4 = s.c / 4, g = threadIdx.x & (c4 - 1);
  float w[4][9], px[9], x[4];
  stem_load_w(s, g, w);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + s.c, g), wv = ld4f(bw, g), bv = ld4f(bb, g);
  const unsigned m = (unsigned)s.nimg * (unsigned)(s.na + s.nbt);
  const unsigned step = gridDim.x * BN_THREADS / c4;
  for (unsigned r = (blockIdx.x * BN_THREADS + threadIdx.x) / c4; r < m; r += step) {
    stem_pixels(s, tab, r, px);
    stem_conv(w, px, x);
    float4 o;
    o.x = bn_act<ACT>((x[0] - mu.x) * is.x * wv.x + bv.x, slope);
    o.y = bn_act<ACT>((x[1] - mu.y) * is.y * wv.y + bv.y, slope);
    o.z = bn_act<ACT>((x[2] - mu.z) * is.z * wv.z + bv.z, slope);
    o.w = bn_act<ACT>((x[3] - mu.w) * is.w * wv.w + bv.w, slope);
    if (r < s.rows_out) reinterpret_cast<float4*>(y)[(size_t)r * c4 + g] = o;
  }
}

// backward reduce: per channel sum(gz), sum(gz xhat)
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void stem1_bwd_partial(Stem1 s, const float* __restrict__ gy,
                                                                const float* __restrict__ bw, const float* __restrict__ bb,
                                                                const float* __restrict__ stats, float slope,
                                                                double* __restrict__ part) {
  __shared__ short tab[STEM_MAX_CELLS * 9];
  stem_stage_table(s, tab);
  const int c4 = s.c / 4, g = threadIdx.x & (c4 - 1);
  float w[4][9], px[9], x[4];
  stem_load_w(s, g, w);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + s.c, g), wv = ld4f(bw, g), bv = ld4f(bb, g);
  const unsigned m = (unsigned)s.nimg * (unsigned)(s.na + s.nbt);
  const unsigned step = gridDim.x * BN_THREADS / c4;
  float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
  for (unsigned r = (blockIdx.x * BN_THREADS + threadIdx.x) / c4; r < m; r += step) {
    stem_pixels(s, tab, r, px);
    stem_conv(w, px, x);
    const float4 dy = r < s.rows_out ? ld4f(gy, (long long)r * c4 + g) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (x[j] - comp(mu, j)) * comp(is, j);
      const float gz = comp(dy, j) * bn_dact<ACT>(xh * comp(wv, j) + comp(bv, j), slope);
      a[j] += gz;
      a[4 + j] += gz * xh;
    }
  }
  bn_block_partials(a, s.c, part);
}

// backward element + conv weight gradient: gx = (gz - sum gz / M - xhat sum gz xhat / M) invstd w (never
// written), gW[4 g + j][k] += gx_j px_k; per block [C][9] partials in fp64
template <int ACT>
__global__ __launch_bounds__(BN_THREADS) void stem1_bwd_wgrad(Stem1 s, const float* __restrict__ gy,
                                                              const float* __restrict__ bw, const float* __restrict__ bb,
                                                              const float* __restrict__ stats, const float* __restrict__ sums,
                                                              float slope, double* __restrict__ wpart) {
  __shared__ short tab[STEM_MAX_CELLS * 9];
  __shared__ float red[BN_THREADS * 36];
  stem_stage_table(s, tab);
  const int c4 = s.c / 4, g = threadIdx.x & (c4 - 1);
  float w[4][9], px[9], x[4], acc[4][9];
  stem_load_w(s, g, w);
  const float4 mu = ld4f(stats, g), is = ld4f(stats + s.c, g), wv = ld4f(bw, g), bv = ld4f(bb, g);
  const unsigned m = (unsigned)s.nimg * (unsigned)(s.na + s.nbt);
  const float inv_m = 1.0f / (float)m;
  const float4 s1 = ld4f(sums, g), s2 = ld4f(sums + s.c, g);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[j][k] = 0.0f;
  const unsigned step = gridDim.x * BN_THREADS / c4;
  for (unsigned r = (blockIdx.x * BN_THREADS + threadIdx.x) / c4; r < m; r += step) {
    stem_pixels(s, tab, r, px);
    stem_conv(w, px, x);
    const float4 dy = r < s.rows_out ? ld4f(gy, (long long)r * c4 + g) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float xh = (x[j] - comp(mu, j)) * comp(is, j);
      const float gz = comp(dy, j) * bn_dact<ACT>(xh * comp(wv, j) + comp(bv, j), slope);
      const float gx = (gz - comp(s1, j) * inv_m - xh * (comp(s2, j) * inv_m)) * (comp(is, j) * comp(wv, j));
#pragma unroll
      for (int k = 0; k < 9; ++k) acc[j][k] = __builtin_fmaf(gx, px[k], acc[j][k]);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 9; ++k) red[(j * 9 + k) * BN_THREADS + threadIdx.x] = acc[j][k];
  __syncthreads();
  // (channel 4 gg + j, k) sums the threads of group gg in index order
  for (int v = threadIdx.x; v < 9 * s.c; v += BN_THREADS) {
    const int ch = v / 9, k = v % 9, gg = ch / 4, j = ch % 4;
    double t = 0.0;
    for (int u = gg; u < BN_THREADS; u += c4) t += (double)red[(j * 9 + k) * BN_THREADS + u];
    wpart[(size_t)blockIdx.x * 9 * s.c + v] = t;
  }
}

__global__ __launch_bounds__(BN_FINAL_THREADS) void stem1_wgrad_final(int n, int blocks, const double* __restrict__ wpart,
                                                                      float* __restrict__ gw) {
  __shared__ double tot[1024];
  bn_final_sums(wpart, n, blocks, tot);
  for (int v = threadIdx.x; v < n; v += BN_FINAL_THREADS) gw[v] = (float)tot[v];
}

// ------------------------------------------------------------- the first block on fp32 MFMA (C = 16)
// The per-row kernels above spend four threads per row (one per 4 channels), each re-deriving the row's image
// and cell and gathering the same 9 pixels from global memory, plus 36 VALU FMAs; the four passes ran at
// 1.7-2.4x their HBM floors (profiles/round03_vision_update_kernel_stats.csv).  Here a workgroup takes whole
// images: it stages the image (27.6 KB at 72 x 96) in LDS with coalesced loads, and its four waves take the
// image's rows 16 at a time (tiles of table a, then of table b; every tile lies within one image and one table).
// The conv is three v_mfma_f32_16x16x4f32 (K = 9 padded to 12): lane l gathers pixels k = l/16, l/16 + 4 (and 8
// for l < 16) of row l % 16 from the LDS image — the A operand — against the weights W[l % 16][k] held as the B
// operand, and receives x[row 4 (l/16) + v][channel l % 16], v = 0..3.  The MFMA is a k-ordered fmaf chain from 0
// (padding adds exact zeros), so every x is bit-identical to stem_conv's.  The conv weight's gradient is a second
// product on the same tile, G[ch][k] += sum_rows gx[row][ch] px[row][k]: the lane's four gx (channel l % 16, rows
// 4 (l/16) + v) are exactly the A operands of four 16x16x4 MFMAs over the rows 4 kk + v, their B operands the
// tile's pixels read back from a per-wave LDS copy of the A operands.  Per-lane sums are fp32 within a tile and
// fp64 across tiles and in the fixed-order block reductions.  A pixel table reaching beyond SM_IMG_CAP floats
// (or beyond the row: ld - off) gathers from global memory instead (the same arithmetic).
typedef float sm4 __attribute__((ext_vector_type(4)));
constexpr int SM_IMG_CAP = 8192;  // image floats staged in LDS per workgroup
constexpr int SM_GRID = 512;      // workgroups: two per CU (LDS ~73 KB each), images strided over them
constexpr int SM_WAVES = 4;       // compute waves per workgroup; one more wave stages the next image (LDS-DMA)
constexpr int SM_THREADS = 64 * (SM_WAVES + 1);
// tiles per compute wave in flight together: 12 in the forward passes, 6 in the backward ones (which also hold
// the tiles' gradient rows); measured against 4 / 6 / 12 everywhere (gpurun_out/r4q)
template <int PASS>
constexpr int sm_tiles() { return PASS <= 1 ? 12 : 6; }
enum { SM_STATS = 0, SM_APPLY = 1, SM_BWDP = 2, SM_WGRAD = 3 };

struct SmArgs {
  const float* bw;     // BN weight / bias
  const float* bb;
  const float* stats;  // [4][16] (mean, invstd, ...)
  const float* sums;   // [2][16] sum gz, sum gz xhat (SM_WGRAD)
  const float* gy;     // [rows_out][16]
  float* y;            // [rows_out][16] (SM_APPLY)
  double* part;        // block partials
  float* shift;        // [16] (SM_STATS)
  float slope;
};

__device__ __forceinline__ sm4 sm_mfma(float a, float b, sm4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ sm4 sm_conv(const float px[3], const float wb[3]) {
  sm4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  acc = sm_mfma(px[0], wb[0], acc);
  acc = sm_mfma(px[1], wb[1], acc);
  return sm_mfma(px[2], wb[2], acc);
}
__device__ __forceinline__ unsigned sm_wave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// dynamic LDS: the pixel table (int16, padded to 16 B), then two image buffers of sm_img_floats (the cap rounded
// up to a DMA instruction's 256 floats; at least 1 024 each: the block reductions reuse them at the end)
__host__ __device__ inline size_t sm_tab_floats(int ncell) { return (size_t)((ncell * 9 + 7) & ~7) / 2; }
__host__ __device__ inline size_t sm_img_floats(int cap) { const size_t c = ((size_t)cap + 255) & ~(size_t)255; return c > 1024 ? c : 1024; }
__host__ __device__ inline size_t sm_lds_bytes(int ncell, int cap) { return 4 * (sm_tab_floats(ncell) + 2 * sm_img_floats(cap)); }

typedef __attribute__((address_space(3))) void sm_lds_void_t;
typedef __attribute__((address_space(1))) void sm_glob_void_t;
// the image's first `span` floats into the LDS buffer dst by LDS-DMA (global_load_lds), issued by one wave: per
// instruction lane l's 16 (or 4) bytes land at dst + o + 4 l (or + l); lanes past the span read the image's first
// bytes (in bounds) into the buffer's padding.  v4: the image rows are 16-B aligned and span % 4 == 0.
__device__ __forceinline__ void sm_dma_image(const float* g, float* dst, int span, bool v4) {
  const int lane = threadIdx.x & 63;
  if (v4) {
    for (int o = 0; o < span; o += 256) {
      const int i = o + 4 * lane;
      __builtin_amdgcn_global_load_lds((sm_glob_void_t*)(g + (i < span ? i : 0)), (sm_lds_void_t*)(dst + o), 16, 0, 0);
    }
  } else {
    for (int o = 0; o < span; o += 64) {
      const int i = o + lane;
      __builtin_amdgcn_global_load_lds((sm_glob_void_t*)(g + (i < span ? i : 0)), (sm_lds_void_t*)(dst + o), 4, 0, 0);
    }
  }
}

template <int PASS, int ACT, bool V4>
__global__ __launch_bounds__(SM_THREADS) void stem1i_kernel(Stem1 s, SmArgs q, int cap) {
  extern __shared__ float4 sm_dyn4[];
  __shared__ int s_span;
  __shared__ float pimg[SM_WAVES][16][17];  // SM_WGRAD: per wave, the tile's A operands [row][k] (+1: banks; one
                                            // buffer per wave: its LDS accesses complete in order)
  const int na = s.na, nbt = s.nbt, ncell = na + nbt;
  short* tab = reinterpret_cast<short*>(sm_dyn4);
  float* im0 = reinterpret_cast<float*>(sm_dyn4) + sm_tab_floats(ncell);
  float* im1 = im0 + sm_img_floats(cap);
  const unsigned l = threadIdx.x & 63, ch = l & 15, kq = l >> 4, w = sm_wave();
  const bool loader = w == SM_WAVES;  // (wave-uniform)
  if (threadIdx.x == 0) s_span = 0;
  __syncthreads();
  int mx = 0;
  for (int i = threadIdx.x; i < ncell * 9; i += SM_THREADS) {
    const short t = s.pix[i];
    tab[i] = t;
    mx = mx > (int)t + 1 ? mx : (int)t + 1;
  }
  atomicMax(&s_span, mx);
  __syncthreads();
  const int span = s_span;
  const bool staged = span <= cap;  // (block-uniform)
  const bool v4 = V4 && (span & 3) == 0;

  float wb[3];  // B operand of the conv: W[ch][k = kq + 4 c] (0 for k >= 9)
#pragma unroll
  for (int c = 0; c < 3; ++c) wb[c] = kq + 4 * c < 9 ? s.w[ch * 9 + kq + 4 * c] : 0.0f;
  float mu = 0.0f, is = 0.0f, wv = 0.0f, bv = 0.0f, mg = 0.0f, mgx = 0.0f, sh = 0.0f;
  const unsigned m = (unsigned)s.nimg * (unsigned)ncell, rows = (unsigned)s.rows_out, ra = (unsigned)s.nimg * (unsigned)na;
  if constexpr (PASS == SM_STATS) {
    // the shift: row 0 (image 0, cell 0) of this lane's channel, from global memory (lane ch holds row 0)
    const bool ok = (int)(l & 15) < ncell;
    const short* t0 = tab + (ok ? (int)(l & 15) : 0) * 9;
    const float* im_0 = stem_img(s, 0);
    const float v0 = im_0[t0[kq]], v1 = im_0[t0[kq + 4]], v2 = im_0[t0[8]];
    const float px[3] = {ok ? v0 : 0.0f, ok ? v1 : 0.0f, (ok && kq == 0) ? v2 : 0.0f};
    const sm4 x0 = sm_conv(px, wb);
    sh = __shfl(x0[0], (int)ch);
    if (blockIdx.x == 0 && threadIdx.x < 16) q.shift[ch] = sh;
  } else {
    mu = q.stats[ch];
    is = q.stats[16 + ch];
    wv = q.bw[ch];
    bv = q.bb[ch];
    if constexpr (PASS == SM_WGRAD) {
      const float inv_m = 1.0f / (float)m;
      mg = q.sums[ch] * inv_m;
      mgx = q.sums[16 + ch] * inv_m;
      if (!loader) pimg[w][l & 15][12 + kq] = 0.0f;  // k = 12 .. 15: zero B operands
    }
  }
  const float isw = is * wv;
  double a0 = 0.0, a1 = 0.0, g4[4] = {0.0, 0.0, 0.0, 0.0};
  const int ta = (na + 15) / 16, T = ta + (nbt + 15) / 16;
  constexpr int U = sm_tiles<PASS>();

  // images b = blockIdx.x + k gridDim.x: the loader wave stages image k + 1 into the other buffer (LDS-DMA) while
  // the compute waves run image k; the barrier at the end of each image drains the DMA (s_waitcnt vmcnt(0))
  const int nmine = s.nimg > (int)blockIdx.x ? (s.nimg - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (staged && loader && nmine > 0) sm_dma_image(stem_img(s, blockIdx.x), im0, span, v4);
  __syncthreads();
  for (int k = 0; k < nmine; ++k) {
    const int b = (int)blockIdx.x + k * (int)gridDim.x;
    const float* g = stem_img(s, b);
    const float* im = (k & 1) ? im1 : im0;
    if (loader) {
      if (staged && k + 1 < nmine) sm_dma_image(stem_img(s, b + (long long)gridDim.x), (k & 1) ? im0 : im1, span, v4);
    } else {
      // one instantiation per source, so the gathers stay ds_read (LDS) or global_load: a pointer chosen at run time
      // between the two became flat loads with full waits
      auto tiles = [&](auto from_lds) {
      for (int j0 = (int)w; j0 < T; j0 += SM_WAVES * U) {
        // U tiles j0 + SM_WAVES u at a time: their gathers (and gradient loads) issue before any is consumed
        int nvalid[U];
        unsigned r0[U];
        float px[U][3], gv[U][4];
        int po[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = j0 + SM_WAVES * u;
          int cell0;
          if (j < ta) {
            cell0 = 16 * j;
            nvalid[u] = na - cell0 < 16 ? na - cell0 : 16;
            r0[u] = (unsigned)b * (unsigned)na + (unsigned)cell0;
          } else if (j < T) {
            const int jj = 16 * (j - ta);
            cell0 = na + jj;
            nvalid[u] = nbt - jj < 16 ? nbt - jj : 16;
            r0[u] = ra + (unsigned)b * (unsigned)nbt + (unsigned)jj;
          } else {  // past the image's last tile
            cell0 = 0;
            nvalid[u] = 0;
            r0[u] = 0;
          }
          const bool ok = (int)(l & 15) < nvalid[u];
          const short* t = tab + (cell0 + (ok ? (int)(l & 15) : 0)) * 9;
          po[u][0] = t[kq];  // (all the tiles' table reads before any image read: one LDS wait, not one per tile)
          po[u][1] = t[kq + 4];
          po[u][2] = t[8];
          if constexpr (PASS == SM_BWDP || PASS == SM_WGRAD) {
            // gy of the lane's rows (0 past rows_out: those rows enter the statistics only)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const unsigned r = r0[u] + 4 * kq + v;
              const bool live = (int)(4 * kq + v) < nvalid[u] && r < rows;
              const float gl = q.gy[(size_t)(live ? r : 0u) * 16 + ch];
              gv[u][v] = live ? gl : 0.0f;
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float v0, v1, v2;
          if constexpr (decltype(from_lds)::value) {  // ds_read: the image in LDS
            v0 = im[po[u][0]];
            v1 = im[po[u][1]];
            v2 = im[po[u][2]];
          } else {
            v0 = g[po[u][0]];
            v1 = g[po[u][1]];
            v2 = g[po[u][2]];
          }
          // the A operand as loaded, no selects (a select let the compiler move the load under a branch, with a
          // wait per tile): k = 9 .. 11 meet zero weights (fma(p, 0, acc) = acc for finite p), and rows past the
          // tile's end (a clamped cell's pixels) give outputs every pass masks
          px[u][0] = v0;
          px[u][1] = v1;
          px[u][2] = v2;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const sm4 x = sm_conv(px[u], wb);
          if constexpr (PASS == SM_STATS) {
            float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const float d = (int)(4 * kq + v) < nvalid[u] ? x[v] - sh : 0.0f;
              s0 += d;
              s1 += d * d;
            }
            a0 += (double)s0;
            a1 += (double)s1;
          } else if constexpr (PASS == SM_APPLY) {
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const unsigned r = r0[u] + 4 * kq + v;
              if ((int)(4 * kq + v) < nvalid[u] && r < rows)
                q.y[(size_t)r * 16 + ch] = bn_act<ACT>((x[v] - mu) * is * wv + bv, q.slope);
            }
          } else {
            float gz[4], xh[4];
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              xh[v] = (x[v] - mu) * is;
              gz[v] = gv[u][v] * bn_dact<ACT>(xh[v] * wv + bv, q.slope);
            }
            if constexpr (PASS == SM_BWDP) {
              float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
              for (int v = 0; v < 4; ++v) {
                s0 += gz[v];
                s1 += gz[v] * xh[v];
              }
              a0 += (double)s0;
              a1 += (double)s1;
            } else {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
              // the B operand: the tile's pixels, 0 past its rows and for k >= 9
              const bool okc = (int)(l & 15) < nvalid[u] && (c < 2 || kq == 0);
              pimg[w][l & 15][kq + 4 * c] = okc ? px[u][c] : 0.0f;
            }
              sm4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
              for (int v = 0; v < 4; ++v) {
                // rows past the tile's end: their pixels (the B operand) are 0
                const float gx = (gz[v] - mg - xh[v] * mgx) * isw;
                acc = sm_mfma(gx, pimg[w][4 * kq + v][ch], acc);
              }
#pragma unroll
              for (int c = 0; c < 4; ++c) g4[c] += (double)acc[c];
            }
          }
        }
      }
      };
      if (staged)
        tiles(std::true_type{});
      else
        tiles(std::false_type{});
    }
    __syncthreads();  // image k read, image k + 1 staged
  }

  // fixed-order block reductions of the compute waves' sums through the (now free) image buffers
  double* red = reinterpret_cast<double*>(im0);
  if constexpr (PASS == SM_STATS || PASS == SM_BWDP) {
    // part[block][2][16]: per channel the waves in order, then l / 16 in order
    if (!loader) {
      red[threadIdx.x] = a0;
      red[BN_THREADS + threadIdx.x] = a1;
    }
    __syncthreads();
    if (threadIdx.x < 32) {
      const int qq = threadIdx.x >> 4, c = threadIdx.x & 15;
      double acc = 0.0;
      for (int ww = 0; ww < BN_THREADS / 64; ++ww)
        for (int k = 0; k < 4; ++k) acc += red[qq * BN_THREADS + ww * 64 + k * 16 + c];
      q.part[(size_t)blockIdx.x * 32 + threadIdx.x] = acc;
    }
  } else if constexpr (PASS == SM_WGRAD) {
    // lane l holds G[channel 4 (l / 16) + c][k = l % 16]; wpart[block][ch * 9 + k]: the waves' values in order
    if (!loader) {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[c * BN_THREADS + threadIdx.x] = g4[c];
    }
    __syncthreads();
    for (int v = threadIdx.x; v < 16 * 9; v += BN_THREADS) {
      const int c2 = v / 9, k = v % 9, lane = (c2 >> 2) * 16 + k, c = c2 & 3;
      double t = 0.0;
      for (int ww = 0; ww < BN_THREADS / 64; ++ww) t += red[c * BN_THREADS + ww * 64 + lane];
      q.part[(size_t)blockIdx.x * 144 + v] = t;
    }
  }
}

// ------------------------------------------------------------- the first block's backward fused with conv2's dgrad
// conv2 = Conv2d(16, 32, 3, stride 3) on the first block's output, whose rows come grouped as conv2's patches (cell
// 9 p + j of table a is position j of patch p).  Its input gradient gy1[cell 9 p + j][c] = sum_o gz2[p][o] W2[o][j, c]
// was a GEMM writing [rows, 144] (1.13 GB per 24 576-image mini-batch) that both backward passes then read back.
// Here the passes form it themselves: a tile is 16 patches at one position j, so
//   gy1 tile = gz2[16 patches][32] x W2[32][j, 16 channels]: eight v_mfma_f32_16x16x4f32, k step s of lane group g
//   taking o = 8 g + s (A: the lane's patch row of gz2, two float4; B: W2 re-laid as w2t[j][g][c][s], two float4),
// and the output fragment (patch 4 (l/16) + v, channel l % 16) is exactly the conv1 fragment of the same 16 cells
// (cells 9 (16 chunk + i) + j as the tile's rows).  Table b's cells (not under conv2) have gy1 = 0.
// One pass instead of two: the conv weight's gradient sum_r gx[r][ch] px[r][k], gx = (gz - mg - xhat mgx) isw with
// mg, mgx the batch means of gz and gz xhat, is isw (A1 - mg A2 - mgx A3) with A1 = sum gz px, A2 = sum px,
// A3 = sum xhat px, none of which needs mg or mgx: the pass accumulates them with the BN sums (12 MFMAs per tile on
// the pixels read back from LDS, as the weight-gradient pass did for gx) and stem12_final combines them in fp64.
// Per-lane sums are fp32 over one image's tiles, fp64 across images and in the block / final reductions (fp64 per
// tile, as the first block's own passes do, took ~50 fp64 conversions and adds per tile).
struct Sm12Args {
  const float* bw;
  const float* bb;
  const float* stats;
  const float* gz2;   // [nimg * n2][32]
  const float* w2t;   // [9][4][16][8]: W2[o = 8 g + s][j * 16 + c] at ((j * 4 + g) * 16 + c) * 8 + s
  double* part;       // [grid][32] BN sums (as SM_BWDP)
  double* wpart;      // [grid][3][144] A1, A2, A3 (channel 4 (l / 16) + c, tap l % 16 layout as SM_WGRAD's)
  float slope;
  int n2;             // conv2 patches per image (na = 9 n2)
};

template <int ACT, bool V4>
__global__ __launch_bounds__(SM_THREADS) void stem12b_kernel(Stem1 s, Sm12Args q, int cap) {
  extern __shared__ float4 sm_dyn4[];
  __shared__ int s_span;
  __shared__ float pimg[SM_WAVES][16][17];
  const int na = s.na, nbt = s.nbt, ncell = na + nbt, n2 = q.n2;
  short* tab = reinterpret_cast<short*>(sm_dyn4);
  float* im0 = reinterpret_cast<float*>(sm_dyn4) + sm_tab_floats(ncell);
  float* im1 = im0 + sm_img_floats(cap);
  const unsigned l = threadIdx.x & 63, ch = l & 15, kq = l >> 4, w = sm_wave();
  const bool loader = w == SM_WAVES;
  if (threadIdx.x == 0) s_span = 0;
  __syncthreads();
  int mx = 0;
  for (int i = threadIdx.x; i < ncell * 9; i += SM_THREADS) {
    const short t = s.pix[i];
    tab[i] = t;
    mx = mx > (int)t + 1 ? mx : (int)t + 1;
  }
  atomicMax(&s_span, mx);
  __syncthreads();
  const int span = s_span;
  const bool staged = span <= cap;
  const bool v4 = V4 && (span & 3) == 0;

  float wb[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) wb[c] = kq + 4 * c < 9 ? s.w[ch * 9 + kq + 4 * c] : 0.0f;
  const float mu = q.stats[ch], is = q.stats[16 + ch], wv = q.bw[ch], bv = q.bb[ch];
  if (!loader) pimg[w][l & 15][12 + kq] = 0.0f;  // k = 12 .. 15: zero B operands
  // A2 (the pixel sums, the same for every channel) on the VALU: this lane's row, taps kq, kq + 4, kq + 8
  double a0 = 0.0, a1 = 0.0, g1[4] = {0.0, 0.0, 0.0, 0.0}, g3[4] = {0.0, 0.0, 0.0, 0.0}, p2[3] = {0.0, 0.0, 0.0};
  const int nch = (n2 + 15) / 16, ta = 9 * nch;
  const int T = ta + (nbt + 15) / 16;
  constexpr int U = 3;

  const int nmine = s.nimg > (int)blockIdx.x ? (s.nimg - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (staged && loader && nmine > 0) sm_dma_image(stem_img(s, blockIdx.x), im0, span, v4);
  __syncthreads();
  for (int k = 0; k < nmine; ++k) {
    const int b = (int)blockIdx.x + k * (int)gridDim.x;
    const float* g = stem_img(s, b);
    const float* im = (k & 1) ? im1 : im0;
    if (loader) {
      if (staged && k + 1 < nmine) sm_dma_image(stem_img(s, b + (long long)gridDim.x), (k & 1) ? im0 : im1, span, v4);
    } else {
      // fp32 sums over this image's tiles (<= 15 per wave), folded into the fp64 accumulators once per image
      float f0 = 0.0f, f1 = 0.0f, fp2[3] = {0.0f, 0.0f, 0.0f};
      sm4 fg1 = {0.0f, 0.0f, 0.0f, 0.0f}, fg3 = {0.0f, 0.0f, 0.0f, 0.0f};
      auto tiles = [&](auto from_lds) {
      for (int j0 = (int)w; j0 < T; j0 += SM_WAVES * U) {
        int nvalid[U];
        bool conv2t[U];  // a table-a tile (gy1 from gz2); else table b (gy1 = 0)
        float px[U][3];
        int po[U][3];
        float4 za[U][2], wf[U][2];  // gz2 A fragments, W2 B fragments
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int t = j0 + SM_WAVES * u;
          int cell;
          conv2t[u] = t < ta;
          if (t < ta) {
            const int chunk = t / 9, jj = t - 9 * chunk;
            nvalid[u] = n2 - 16 * chunk < 16 ? n2 - 16 * chunk : 16;
            const int p = 16 * chunk + ((int)(l & 15) < nvalid[u] ? (int)(l & 15) : 0);
            cell = 9 * p + jj;
            const float4* zr = reinterpret_cast<const float4*>(q.gz2 + ((size_t)b * n2 + p) * 32 + 8 * kq);
            za[u][0] = zr[0];
            za[u][1] = zr[1];
            const float4* wr = reinterpret_cast<const float4*>(q.w2t + (size_t)((jj * 4 + (int)kq) * 16 + (int)ch) * 8);
            wf[u][0] = wr[0];
            wf[u][1] = wr[1];
          } else if (t < T) {
            const int jb = 16 * (t - ta);
            nvalid[u] = nbt - jb < 16 ? nbt - jb : 16;
            cell = na + jb + ((int)(l & 15) < nvalid[u] ? (int)(l & 15) : 0);
            za[u][0] = za[u][1] = wf[u][0] = wf[u][1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          } else {
            nvalid[u] = 0;
            cell = 0;
            za[u][0] = za[u][1] = wf[u][0] = wf[u][1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
          }
          const short* tt = tab + cell * 9;
          po[u][0] = tt[kq];
          po[u][1] = tt[kq + 4];
          po[u][2] = tt[8];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if constexpr (decltype(from_lds)::value) {
            px[u][0] = im[po[u][0]];
            px[u][1] = im[po[u][1]];
            px[u][2] = im[po[u][2]];
          } else {
            px[u][0] = g[po[u][0]];
            px[u][1] = g[po[u][1]];
            px[u][2] = g[po[u][2]];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const sm4 x = sm_conv(px[u], wb);
          // gy1 of the tile's rows (patches 4 kq + v, channel ch): k step s of lane group kq is o = 8 kq + s
          sm4 gyt = {0.0f, 0.0f, 0.0f, 0.0f};
          if (conv2t[u]) {  // (wave-uniform)
            const float a8[8] = {za[u][0].x, za[u][0].y, za[u][0].z, za[u][0].w, za[u][1].x, za[u][1].y, za[u][1].z, za[u][1].w};
            const float b8[8] = {wf[u][0].x, wf[u][0].y, wf[u][0].z, wf[u][0].w, wf[u][1].x, wf[u][1].y, wf[u][1].z, wf[u][1].w};
#pragma unroll
            for (int ss = 0; ss < 8; ++ss) gyt = sm_mfma(a8[ss], b8[ss], gyt);
          }
          float gz[4], xh[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const bool live = (int)(4 * kq + v) < nvalid[u];
            xh[v] = (x[v] - mu) * is;
            gz[v] = (live ? gyt[v] : 0.0f) * bn_dact<ACT>(xh[v] * wv + bv, q.slope);
          }
          float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const bool row = (int)(4 * kq + v) < nvalid[u];  // (xhat of a row past the tile's end: its pixels are 0)
            s0 += gz[v];
            s1 += row ? gz[v] * xh[v] : 0.0f;
          }
          f0 += s0;
          f1 += s1;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const bool okc = (int)(l & 15) < nvalid[u] && (c < 2 || kq == 0);
            const float pc = okc ? px[u][c] : 0.0f;
            pimg[w][l & 15][kq + 4 * c] = pc;
            fp2[c] += pc;
          }
          sm4 c1 = {0.0f, 0.0f, 0.0f, 0.0f}, c3 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const float pv = pimg[w][4 * kq + v][ch];
            c1 = sm_mfma(gz[v], pv, c1);
            c3 = sm_mfma(xh[v], pv, c3);
          }
          fg1 += c1;
          fg3 += c3;
        }
      }
      };
      if (staged)
        tiles(std::true_type{});
      else
        tiles(std::false_type{});
      a0 += (double)f0;
      a1 += (double)f1;
#pragma unroll
      for (int c = 0; c < 3; ++c) p2[c] += (double)fp2[c];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        g1[c] += (double)fg1[c];
        g3[c] += (double)fg3[c];
      }
    }
    __syncthreads();
  }

  // fixed-order block reductions through the (now free) image buffers (>= 2 x 1 024 floats: 4 x 256 doubles a round)
  double* red = reinterpret_cast<double*>(im0);
  if (!loader) {
    red[threadIdx.x] = a0;
    red[BN_THREADS + threadIdx.x] = a1;
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int qq = threadIdx.x >> 4, c = threadIdx.x & 15;
    double acc = 0.0;
    for (int ww = 0; ww < BN_THREADS / 64; ++ww)
      for (int k = 0; k < 4; ++k) acc += red[qq * BN_THREADS + ww * 64 + k * 16 + c];
    q.part[(size_t)blockIdx.x * 32 + threadIdx.x] = acc;
  }
#pragma unroll
  for (int a = 0; a < 3; a += 2) {
    __syncthreads();
    if (!loader) {
#pragma unroll
      for (int c = 0; c < 4; ++c) red[c * BN_THREADS + threadIdx.x] = a == 0 ? g1[c] : g3[c];
    }
    __syncthreads();
    for (int v = threadIdx.x; v < 16 * 9; v += BN_THREADS) {
      const int c2 = v / 9, k = v % 9, lane = (c2 >> 2) * 16 + k, c = c2 & 3;
      double t = 0.0;
      for (int ww = 0; ww < BN_THREADS / 64; ++ww) t += red[c * BN_THREADS + ww * 64 + lane];
      q.wpart[((size_t)blockIdx.x * 3 + a) * 144 + v] = t;
    }
  }
  // A2[k]: the lanes holding tap k (lane group k % 4, register k / 4) summed over rows and waves in a fixed order,
  // stored for every channel
  __syncthreads();
  if (!loader) {
#pragma unroll
    for (int c = 0; c < 3; ++c) red[c * BN_THREADS + threadIdx.x] = p2[c];
  }
  __syncthreads();
  for (int v = threadIdx.x; v < 16 * 9; v += BN_THREADS) {
    const int k = v % 9, c = k >> 2, g = k & 3;
    double t = 0.0;
    for (int ww = 0; ww < BN_THREADS / 64; ++ww)
      for (int i = 0; i < 16; ++i) t += red[c * BN_THREADS + ww * 64 + g * 16 + i];
    q.wpart[((size_t)blockIdx.x * 3 + 1) * 144 + v] = t;
  }
}

// gconv[ch][k] = isw (A1 - mg A2 - mgx A3), the A sums over the blocks in a fixed order, mg / mgx from the BN sums
__global__ __launch_bounds__(BN_FINAL_THREADS) void stem12_final(int blocks, const double* __restrict__ wpart,
                                                                const float* __restrict__ sums, const float* __restrict__ stats,
                                                                const float* __restrict__ bw, double m, float* __restrict__ gw) {
  __shared__ double tot[3 * 144];
  // the three sums one after the other (7 threads per column instead of 2 for all 432 at once)
  for (int a = 0; a < 3; ++a) bn_final_sums(wpart + a * 144, 144, blocks, tot + a * 144, 3 * 144);
  for (int v = threadIdx.x; v < 144; v += BN_FINAL_THREADS) {
    const int ch = v / 9;
    const double mg = (double)sums[ch] / m, mgx = (double)sums[16 + ch] / m;
    const double isw = (double)stats[16 + ch] * (double)bw[ch];
    gw[v] = (float)(isw * (tot[v] - mg * tot[144 + v] - mgx * tot[288 + v]));
  }
}

static void sm12_launch(const Stem1& s, const Sm12Args& q, int act, int grid, hipStream_t st) {
  long long room = s.ld - s.off;
  const int cap = (int)(room < 1 ? 1 : room < SM_IMG_CAP ? room : SM_IMG_CAP);
  const size_t lds = sm_lds_bytes(s.na + s.nbt, cap);
  const bool v4 = ((uintptr_t)(s.obs + s.off) & 15) == 0 && (s.ld & 3) == 0;
  if (act == GR_POLICY_ACT_ELU) {
    if (v4)
      hipLaunchKernelGGL((stem12b_kernel<GR_POLICY_ACT_ELU, true>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
    else
      hipLaunchKernelGGL((stem12b_kernel<GR_POLICY_ACT_ELU, false>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
  } else {
    if (v4)
      hipLaunchKernelGGL((stem12b_kernel<GR_POLICY_ACT_LRELU, true>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
    else
      hipLaunchKernelGGL((stem12b_kernel<GR_POLICY_ACT_LRELU, false>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
  }
}

template <int PASS>
static void sm_launch(const Stem1& s, const SmArgs& q, int act, int grid, hipStream_t st) {
  long long room = s.ld - s.off;
  const int cap = (int)(room < 1 ? 1 : room < SM_IMG_CAP ? room : SM_IMG_CAP);
  const size_t lds = sm_lds_bytes(s.na + s.nbt, cap);
  const bool v4 = ((uintptr_t)(s.obs + s.off) & 15) == 0 && (s.ld & 3) == 0;  // every image row 16-B aligned
  if (act == GR_POLICY_ACT_ELU) {
    if (v4)
      hipLaunchKernelGGL((stem1i_kernel<PASS, GR_POLICY_ACT_ELU, true>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
    else
      hipLaunchKernelGGL((stem1i_kernel<PASS, GR_POLICY_ACT_ELU, false>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
  } else {
    if (v4)
      hipLaunchKernelGGL((stem1i_kernel<PASS, GR_POLICY_ACT_LRELU, true>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
    else
      hipLaunchKernelGGL((stem1i_kernel<PASS, GR_POLICY_ACT_LRELU, false>), dim3(grid), dim3(SM_THREADS), lds, st, s, q, cap);
  }
}

static int stem_blocks(const Stem1& s) { return bn_blocks((long long)s.nimg * (s.na + s.nbt), s.c); }

// workspace (doubles): BN partials [nb][2c] | shift + sums (2c floats, as c doubles) | wgrad partials [nb][3][9c]
// (three sums per block for the fused conv2 backward, one for the first block's own)
long long stem1_scratch_doubles(int nimg, int rows_per_img, int c) {
  const long long nb = bn_blocks((long long)nimg * rows_per_img, c);
  return nb * 2 * c + 2 * c + nb * 27 * c;
}

// ------------------------------------------------------------- the first block's apply pass fused with conv2
// y1 = act(bn(conv1(image))) as SM_APPLY stores it, and conv2's output z2[p][o] = sum_{j, c} y1[9 p + j][c] W2[o][j, c]
// from the same registers (conv2's patch GEMM read y1 back from HBM: 1.13 GB per 24 576-image mini-batch).  conv1 runs
// transposed here, C[channel][cell] = W1 . pixels (A = the weights, B = the gathered pixels: the same k-ordered fmaf
// chain, so y1 is bit-identical to SM_APPLY's), so a lane holds one cell (a patch of the tile) and four channels
// 4 (l/16) + v: exactly conv2's A fragment with k step v of lane group g taking channel 4 g + v.  A wave owns whole
// 16-patch chunks (its nine positions j accumulate in its registers, in j order: deterministic), so the workgroup
// has SMF_WAVES = 5 compute waves (72 x 96: five chunks of 80 patches per image) and one loader wave.
constexpr int SMF_WAVES = 5;
constexpr int SMF_THREADS = 64 * (SMF_WAVES + 1);
struct Sm12fArgs {
  const float* bw;
  const float* bb;
  const float* stats;  // [4][16] (mean, invstd, ...)
  const float* w2f;    // [9][4][32][4]: W2[o][j * 16 + 4 g + v] at ((j * 4 + g) * 32 + o) * 4 + v
  float* y;            // [nimg * na][16]
  float* z2;           // [nimg * n2][32]
  float slope;
  int n2;
};

template <int ACT, bool V4>
__global__ __launch_bounds__(SMF_THREADS) void stem12f_kernel(Stem1 s, Sm12fArgs q, int cap) {
  extern __shared__ float4 sm_dyn4[];
  __shared__ int s_span;
  const int na = s.na, nbt = s.nbt, ncell = na + nbt, n2 = q.n2;
  short* tab = reinterpret_cast<short*>(sm_dyn4);
  float* im0 = reinterpret_cast<float*>(sm_dyn4) + sm_tab_floats(ncell);
  float* im1 = im0 + sm_img_floats(cap);
  const unsigned l = threadIdx.x & 63, lo = l & 15, kq = l >> 4, w = sm_wave();
  const bool loader = w == SMF_WAVES;
  if (threadIdx.x == 0) s_span = 0;
  __syncthreads();
  int mx = 0;
  for (int i = threadIdx.x; i < ncell * 9; i += SMF_THREADS) {
    const short t = s.pix[i];
    tab[i] = t;
    mx = mx > (int)t + 1 ? mx : (int)t + 1;
  }
  atomicMax(&s_span, mx);
  __syncthreads();
  const int span = s_span;
  const bool staged = span <= cap;
  const bool v4 = V4 && (span & 3) == 0;

  // conv1 as C[channel][cell]: A = W1[channel lo][k = kq + 4 c] (0 for k >= 9); the lane's output channels 4 kq + v
  float wa[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) wa[c] = kq + 4 * c < 9 ? s.w[lo * 9 + kq + 4 * c] : 0.0f;
  float mu[4], is[4], wv[4], bv[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int chn = 4 * (int)kq + v;
    mu[v] = q.stats[chn];
    is[v] = q.stats[16 + chn];
    wv[v] = q.bw[chn];
    bv[v] = q.bb[chn];
  }
  const unsigned rows = (unsigned)s.rows_out;
  const int nch = (n2 + 15) / 16;

  const int nmine = s.nimg > (int)blockIdx.x ? (s.nimg - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (staged && loader && nmine > 0) sm_dma_image(stem_img(s, blockIdx.x), im0, span, v4);
  __syncthreads();
  for (int k = 0; k < nmine; ++k) {
    const int b = (int)blockIdx.x + k * (int)gridDim.x;
    const float* g = stem_img(s, b);
    const float* im = (k & 1) ? im1 : im0;
    if (loader) {
      if (staged && k + 1 < nmine) sm_dma_image(stem_img(s, b + (long long)gridDim.x), (k & 1) ? im0 : im1, span, v4);
    } else {
      auto chunks = [&](auto from_lds) {
      for (int chunk = (int)w; chunk < nch; chunk += SMF_WAVES) {
        const int nvalid = n2 - 16 * chunk < 16 ? n2 - 16 * chunk : 16;
        const bool ok = (int)lo < nvalid;
        const int p = 16 * chunk + (ok ? (int)lo : 0);
        // the chunk's nine positions: table reads, then pixel gathers, all issued before any is consumed
        int po[9][3];
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) {
          const short* tt = tab + (9 * p + jj) * 9;
          po[jj][0] = tt[kq];
          po[jj][1] = tt[kq + 4];
          po[jj][2] = tt[8];
        }
        float px[9][3];
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) {
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            if constexpr (decltype(from_lds)::value)
              px[jj][c] = im[po[jj][c]];
            else
              px[jj][c] = g[po[jj][c]];
          }
        }
        sm4 z0 = {0.0f, 0.0f, 0.0f, 0.0f}, z1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int jj = 0; jj < 9; ++jj) {
          sm4 x = {0.0f, 0.0f, 0.0f, 0.0f};
          x = sm_mfma(wa[0], px[jj][0], x);
          x = sm_mfma(wa[1], px[jj][1], x);
          x = sm_mfma(wa[2], px[jj][2], x);
          float4 y4;
          float yv[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) yv[v] = bn_act<ACT>((x[v] - mu[v]) * is[v] * wv[v] + bv[v], q.slope);
          y4.x = yv[0]; y4.y = yv[1]; y4.z = yv[2]; y4.w = yv[3];
          const unsigned r = (unsigned)b * (unsigned)na + (unsigned)(9 * p + jj);
          if (q.y && ok && r < rows) reinterpret_cast<float4*>(q.y + (size_t)r * 16)[kq] = y4;  // (null: no backward)
          // conv2: B fragment W2[o][jj, 4 kq + v] for o = lo (z0) and 16 + lo (z1)
          const float4 b0 = reinterpret_cast<const float4*>(q.w2f)[(jj * 4 + (int)kq) * 32 + (int)lo];
          const float4 b1 = reinterpret_cast<const float4*>(q.w2f)[(jj * 4 + (int)kq) * 32 + 16 + (int)lo];
          z0 = sm_mfma(yv[0], b0.x, z0);
          z0 = sm_mfma(yv[1], b0.y, z0);
          z0 = sm_mfma(yv[2], b0.z, z0);
          z0 = sm_mfma(yv[3], b0.w, z0);
          z1 = sm_mfma(yv[0], b1.x, z1);
          z1 = sm_mfma(yv[1], b1.y, z1);
          z1 = sm_mfma(yv[2], b1.z, z1);
          z1 = sm_mfma(yv[3], b1.w, z1);
        }
        // lane (o = lo, kq) holds z2[patch 16 chunk + 4 kq + v][o] (z0) and [16 + o] (z1)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int pp = 4 * (int)kq + v;
          if (pp < nvalid) {
            float* zr = q.z2 + ((size_t)b * n2 + 16 * chunk + pp) * 32;
            zr[lo] = z0[v];
            zr[16 + lo] = z1[v];
          }
        }
      }
      };
      if (staged)
        chunks(std::true_type{});
      else
        chunks(std::false_type{});
    }
    __syncthreads();
  }
}

hipError_t stem12g_launch(const Stem1& s, const Sm12fArgs& f, int act, hipStream_t st);  // (below, with stem12w)
// (below): blocks written; mom (64 doubles, may be null): the pixel moments gr_stem12_backward_w2 takes A2 / A3 from,
// through mpart (grid x 64 + 9 doubles of workspace)
int stem_stats_launch(const Stem1& s, double* part, float* shift, hipStream_t st, double* mpart = nullptr,
                      double* mom = nullptr);

hipError_t launch_stem12_forward(const Stem1& s, const float* bw, const float* bb, float eps, int act, float slope,
                                 const float* w2f, int n2, float* y, float* z2, float* stats, double* moments,
                                 double* part, hipStream_t st) {
  const int nb = stem_blocks(s);
  float* shift = reinterpret_cast<float*>(part + (size_t)nb * 2 * s.c);
  const long long m = (long long)s.nimg * (s.na + s.nbt);
  const int grid = nb < SM_GRID ? nb : SM_GRID;
  // (the moment partials in the workspace's wgrad region, unused by a forward: nb x 27 c >= grid x 64 + 9)
  double* mpart = part + (size_t)nb * 2 * s.c + 2 * s.c;
  const int sgrid = stem_stats_launch(s, part, shift, st, mpart, moments);
  hipLaunchKernelGGL(bn_stats_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, shift, m, s.c, sgrid, eps, part, stats);
  long long room = s.ld - s.off;
  const int cap = (int)(room < 1 ? 1 : room < SM_IMG_CAP ? room : SM_IMG_CAP);
  const size_t lds = sm_lds_bytes(s.na + s.nbt, cap);
  const bool v4 = ((uintptr_t)(s.obs + s.off) & 15) == 0 && (s.ld & 3) == 0;
  Sm12fArgs f{bw, bb, stats, w2f, y, z2, slope, n2};
  // no y1 to store (the backward recomputes it, or no backward): the position-grouped kernel (stem12g_kernel)
  if (!y && n2 <= 80) return stem12g_launch(s, f, act, st);
  if (act == GR_POLICY_ACT_ELU) {
    if (v4)
      hipLaunchKernelGGL((stem12f_kernel<GR_POLICY_ACT_ELU, true>), dim3(grid), dim3(SMF_THREADS), lds, st, s, f, cap);
    else
      hipLaunchKernelGGL((stem12f_kernel<GR_POLICY_ACT_ELU, false>), dim3(grid), dim3(SMF_THREADS), lds, st, s, f, cap);
  } else {
    if (v4)
      hipLaunchKernelGGL((stem12f_kernel<GR_POLICY_ACT_LRELU, true>), dim3(grid), dim3(SMF_THREADS), lds, st, s, f, cap);
    else
      hipLaunchKernelGGL((stem12f_kernel<GR_POLICY_ACT_LRELU, false>), dim3(grid), dim3(SMF_THREADS), lds, st, s, f, cap);
  }
  return hipGetLastError();
}

hipError_t launch_stem1_forward(const Stem1& s, const float* bw, const float* bb, float eps, int act, float slope,
                                float* y, float* stats, double* part, hipStream_t st) {
  const int nb = stem_blocks(s);
  float* shift = reinterpret_cast<float*>(part + (size_t)nb * 2 * s.c);
  const long long m = (long long)s.nimg * (s.na + s.nbt);
  if (s.c == 16) {  // the reference's stem: the MFMA kernels, whole images per workgroup
    const int grid = nb < SM_GRID ? nb : SM_GRID;
    SmArgs q{bw, bb, stats, nullptr, nullptr, y, part, shift, slope};
    const int sgrid = stem_stats_launch(s, part, shift, st);
    hipLaunchKernelGGL(bn_stats_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, shift, m, s.c, sgrid, eps, part, stats);
    sm_launch<SM_APPLY>(s, q, act, grid, st);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(stem1_stats_partial, dim3(nb), dim3(BN_THREADS), 0, st, s, part, shift);
  hipLaunchKernelGGL(bn_stats_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, shift, m, s.c, nb, eps, part, stats);
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(stem1_apply<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, bw, bb, stats, slope, y);
  else
    hipLaunchKernelGGL(stem1_apply<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, bw, bb, stats, slope, y);
  return hipGetLastError();
}

hipError_t launch_stem1_backward(const Stem1& s, const float* bw, const float* bb, const float* stats, int act,
                                 float slope, const float* gy, float* gconv, float* gbw, float* gbb, double* part,
                                 hipStream_t st) {
  const int nb = stem_blocks(s);
  float* sums = reinterpret_cast<float*>(part + (size_t)nb * 2 * s.c);
  double* wpart = part + (size_t)nb * 2 * s.c + 2 * s.c;
  if (s.c == 16) {
    const int grid = nb < SM_GRID ? nb : SM_GRID;
    SmArgs q{bw, bb, stats, sums, gy, nullptr, part, nullptr, slope};
    sm_launch<SM_BWDP>(s, q, act, grid, st);
    hipLaunchKernelGGL(bn_bwd_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, s.c, grid, part, gbw, gbb, sums);
    q.part = wpart;
    sm_launch<SM_WGRAD>(s, q, act, grid, st);
    hipLaunchKernelGGL(stem1_wgrad_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, 9 * s.c, grid, wpart, gconv);
    return hipGetLastError();
  }
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(stem1_bwd_partial<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, gy, bw, bb, stats, slope, part);
  else
    hipLaunchKernelGGL(stem1_bwd_partial<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, gy, bw, bb, stats, slope, part);
  hipLaunchKernelGGL(bn_bwd_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, s.c, nb, part, gbw, gbb, sums);
  if (act == GR_POLICY_ACT_ELU)
    hipLaunchKernelGGL(stem1_bwd_wgrad<GR_POLICY_ACT_ELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, gy, bw, bb, stats, sums, slope, wpart);
  else
    hipLaunchKernelGGL(stem1_bwd_wgrad<GR_POLICY_ACT_LRELU>, dim3(nb), dim3(BN_THREADS), 0, st, s, gy, bw, bb, stats, sums, slope, wpart);
  hipLaunchKernelGGL(stem1_wgrad_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, 9 * s.c, nb, wpart, gconv);
  return hipGetLastError();
}

hipError_t launch_stem12_backward(const Stem1& s, const float* bw, const float* bb, const float* stats, int act,
                                  float slope, const float* gz2, int n2, const float* w2t, float* gconv, float* gbw,
                                  float* gbb, double* part, hipStream_t st) {
  const int nb = stem_blocks(s);
  float* sums = reinterpret_cast<float*>(part + (size_t)nb * 2 * s.c);
  double* wpart = part + (size_t)nb * 2 * s.c + 2 * s.c;
  const int grid = nb < SM_GRID ? nb : SM_GRID;
  Sm12Args q{bw, bb, stats, gz2, w2t, part, wpart, slope, n2};
  sm12_launch(s, q, act, grid, st);
  hipLaunchKernelGGL(bn_bwd_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, s.c, grid, part, gbw, gbb, sums);
  hipLaunchKernelGGL(stem12_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, grid, wpart, sums, stats, bw,
                     (double)s.nimg * (double)(s.na + s.nbt), gconv);
  return hipGetLastError();
}


// ------------------------------------------------------------- the first block's backward with conv2's dgrad AND wgrad
// stem12b_kernel above forms conv2's input gradient inside the first block's backward, but conv2's weight gradient
// gW2[o][j, c] = sum_p gz2[p][o] y1[9 p + j][c] was a separate pass (gr_patch_wgrad) over a y1 [nimg * na][16] that
// the forward had to write: 1.13 GB written + 1.13 GB read back per 24 576-image mini-batch, plus that pass's launch.
// Here the backward recomputes y1 = act(bn(conv1)) from the registers it already holds (the same expression as the
// forward's, so the same bits) and contracts it with gz2 on MFMA, and the forward stores no y1.
//
// Work split: position-major.  Wave w (8 per workgroup, 2 per SIMD) owns conv2 position j = w: its tiles are the
// image's 16-patch chunks at that position (the rows 9 p + j of patches p = 16 c .. 16 c + 15), so the wave holds
// conv2's weight fragments of ONE position and the conv2 weight-gradient accumulators of one position (plus
// position 8's, whose chunks go to waves 0 .. nch - 1; table b's tiles to the others).  The tile list of a wave is
// the same for every image, so every pixel offset it gathers is computed once, before the image loop (no table reads
// or index arithmetic per tile).  All eight waves share the staging of the next image and its gz2 rows (LDS-DMA);
// gz2's rows sit in LDS with their 16-float halves swapped on every second row group (the G2 operand reads of four
// row groups hit two bank halves instead of one).
//
// Per table-a tile (lane l = 16 g + i; A operands by row i, C rows 4 g + v):
//   x   = conv1 of patches 16 c + i at position j        3 MFMA (A = pixels, B = W1: as sm_conv, bit-identical x)
//   gy1 = gz2[patch][0..31] x W2[0..31][j, ch]            8 MFMA (k step s of group g: o = 8 g + s)
//   gz = gy1 act'(z), y1 = act(z), z = xhat w + b         VALU (rows past n2: 0)
//   A1 += gz^T px, A3 += xhat^T px                         8 MFMA (B = the tile's pixels gathered a second time in
//                                                                the B layout: rows 4 g + v, tap i)
//   G2[ch][o] += y1^T gz2                                  8 MFMA (B = gz2[patch 4 g + v][o = i, 16 + i] from LDS)
// 27 MFMA per tile.  Table-b tiles (cells under no conv2 patch: gz = 0) add only to A3 and A2.  Sums: fp32 within an
// image, fp64 across images and in the fixed-order block / final reductions; deterministic.
constexpr int SW_WAVES = 8;
constexpr int SW_THREADS = 64 * SW_WAVES;
constexpr int SW_MAX_CHUNKS = 5;  // conv2 patches per image <= 80 (72 x 96: exactly 80): offsets held in registers
constexpr int SW_GRID = 256;      // one workgroup per CU (~200 VGPRs: two waves per SIMD)
constexpr int SW_G2 = 9 * 16 * 32;  // conv2 weight-gradient partials per block: [position][channel][o]

struct Sw12Args {
  const float* bw;
  const float* bb;
  const float* stats;
  const float* gz2;  // [nimg * n2][32]
  const float* w2t;  // [9][4][16][8] (as Sm12Args)
  double* part;      // [grid][32] BN sums
  double* wpart;     // [grid][3][144] A1, A2, A3 (stem12_final's layout)
  double* g2part;    // [grid][9][16][32]
  float slope;
  int n2;
  const double* mom;  // the forward's pixel moments (stem_moments_final), or null: A2 / A3 summed here
};

// an image buffer: the staged floats (a DMA instruction's 256 rounded up) + 4 (a zero float, 16-byte aligned stride)
__host__ __device__ inline int sw_img_stride(int cap) { return (int)sm_img_floats(cap) + 4; }
// a gz2 buffer: 16 rows per chunk (rows n2 .. 16 nch zero), at least the DMA's 256-float granularity
__host__ __device__ inline int sw_gz_stride(int n2) {
  const int rows = (n2 + 15) / 16 * 16 * 32, dma = (n2 * 32 + 255) & ~255;
  return rows > dma ? rows : dma;
}
__host__ __device__ inline size_t sw_lds_bytes(int n2, int cap) {
  const size_t b = 4 * (2 * (size_t)sw_img_stride(cap) + 2 * (size_t)sw_gz_stride(n2));
  return b < 8 * 8 * SW_THREADS ? 8 * 8 * SW_THREADS : b;  // (the end's reductions: 8 doubles per thread)
}
// LDS float of gz2[row r][o]: the two 16-float halves of rows with r & 4 swapped
__device__ __forceinline__ int sw_gz_at(int r, int o) { return r * 32 + (o ^ ((r & 4) << 2)); }

// the image's first `span` floats into dst by LDS-DMA, the instructions shared by the eight waves
__device__ __forceinline__ void sw_dma_image(const float* g, float* dst, int span, bool v4, int w) {
  const int lane = threadIdx.x & 63;
  if (v4) {
    for (int o = 256 * w; o < span; o += 256 * SW_WAVES) {
      const int i = o + 4 * lane;
      __builtin_amdgcn_global_load_lds((sm_glob_void_t*)(g + (i < span ? i : 0)), (sm_lds_void_t*)(dst + o), 16, 0, 0);
    }
  } else {
    for (int o = 64 * w; o < span; o += 64 * SW_WAVES) {
      const int i = o + lane;
      __builtin_amdgcn_global_load_lds((sm_glob_void_t*)(g + (i < span ? i : 0)), (sm_lds_void_t*)(dst + o), 4, 0, 0);
    }
  }
}
// the image's gz2 rows (n2 x 32 floats, 16-byte aligned) into dst in sw_gz_at's layout: lane L of an instruction fills
// LDS float4 slot o / 4 + L (row R = slot / 8) from the global float4 the swap maps there
__device__ __forceinline__ void sw_dma_gz2(const float* g, float* dst, int nflt, int w) {
  const int lane = threadIdx.x & 63;
  for (int o = 256 * w; o < nflt; o += 256 * SW_WAVES) {
    const int slot = o / 4 + lane, r = slot >> 3, q4 = slot & 7;
    const int i = 4 * (r * 8 + (q4 ^ (r & 4)));
    if (i < nflt)  // (lanes past the rows write nothing: the buffer's rows n2 .. keep their zeros)
      __builtin_amdgcn_global_load_lds((sm_glob_void_t*)(g + i), (sm_lds_void_t*)(dst + o), 16, 0, 0);
  }
}

// NCH: the 16-patch chunks per image (n2 <= 16 NCH), a compile-time constant so every tile of a wave is straight-line
// code (5 at 72 x 96); 0: taken from n2 at run time (other image sizes; the same arithmetic).  Image buffers carry one
// zero float past their end and the gz2 buffers zero rows up to 16 nch: the gathers of rows past n2 and of taps past 9
// read zeros there (gy1 = 0 and G2 += 0 on rows past n2, B operands 0), so no per-row masks are applied.
// MOM: A2 = sum px and A3 = sum xhat px come from the forward's pixel moments (stem12w_final), so the kernel skips
// their 4 MFMA per table-a tile and table b's tiles altogether (23 MFMA per tile instead of 27)
template <int ACT, bool V4, int NCH, bool MOM>
__global__ __launch_bounds__(SW_THREADS) void stem12w_kernel(Stem1 s, Sw12Args q, int cap) {
  extern __shared__ float4 sm_dyn4[];
  __shared__ int s_span;
  const int na = s.na, nbt = s.nbt, ncell = na + nbt, n2 = q.n2;
  const int nch = NCH > 0 ? NCH : (n2 + 15) / 16, ntb = (nbt + 15) / 16;
  const int imgf = sw_img_stride(cap), gzf = sw_gz_stride(n2);
  float* im0 = reinterpret_cast<float*>(sm_dyn4);
  float* im1 = im0 + imgf;
  float* gz0 = im1 + imgf;
  float* gz1 = gz0 + gzf;
  const int l = (int)(threadIdx.x & 63), i = l & 15, g = l >> 4, w = (int)sm_wave();
  if (threadIdx.x == 0) s_span = 0;
  // the zero float past each image buffer, the gz2 buffers' rows n2 .. 16 nch (never written by the DMA)
  if (threadIdx.x < 2) (threadIdx.x ? im1 : im0)[imgf - 4] = 0.0f;
  for (int k = n2 * 32 + (int)threadIdx.x; k < gzf; k += SW_THREADS) {
    gz0[k] = 0.0f;
    gz1[k] = 0.0f;
  }
  __syncthreads();
  int mx = 0;
  for (int k = threadIdx.x; k < ncell * 9; k += SW_THREADS) {
    const int t = s.pix[k];
    mx = mx > t + 1 ? mx : t + 1;
  }
  atomicMax(&s_span, mx);
  __syncthreads();
  const int span = s_span;
  const bool staged = span <= cap;
  const bool v4 = V4 && (span & 3) == 0;
  const int zero = staged ? imgf - 4 : 0;  // where a masked gather reads (LDS: the zero float; global: pixel 0, masked)

  float wb[3];  // B operand of conv1: W1[ch i][tap g + 4 c] (0 for taps >= 9)
#pragma unroll
  for (int c = 0; c < 3; ++c) wb[c] = g + 4 * c < 9 ? s.w[i * 9 + g + 4 * c] : 0.0f;
  const float mu = q.stats[i], is = q.stats[16 + i], wv = q.bw[i], bv = q.bb[i];

  // the wave's tiles: t < nch = (chunk t, position w), and (chunk w, position 8) when w < nch (`extra`).  Per tile the
  // A-layout pixel offsets (row i: cell 9 p + j, taps g, g + 4, 8; rows past n2 clamped: their outputs meet zero gy1
  // and zero B operands) and the B-layout ones (rows 4 g + v, tap i; `zero` past n2 or for taps >= 9)
  constexpr int NM = NCH > 0 ? NCH : SW_MAX_CHUNKS;
  int oa[NM + 1][3], ob[NM + 1][4];
  unsigned bliv = 0u;  // (global gathers only) B-operand bits
  const bool extra = w < nch;
#pragma unroll
  for (int t = 0; t <= NM; ++t) {
    const int c = t < NM ? t : w, j = t < NM ? w : 8;
    const bool on = t < NM ? t < nch : extra;
    const int pa = on ? (16 * c + i < n2 ? 16 * c + i : n2 - 1) : 0;
    const short* ta = s.pix + (size_t)(9 * pa + j) * 9;
    oa[t][0] = ta[g];
    oa[t][1] = ta[g + 4];
    oa[t][2] = ta[8];
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int p = 16 * c + 4 * g + v;
      const bool ok = on && p < n2 && i < 9;
      ob[t][v] = ok ? s.pix[(size_t)(9 * p + j) * 9 + i] : zero;
      bliv |= (ok ? 1u : 0u) << (4 * t + v);
    }
  }
  // gz2 in LDS (sw_gz_at): A of gy1 = row 16 c + i, floats 8 g .. 8 g + 7; B of G2 = rows 16 c + 4 g + v, o = i and
  // 16 + i.  Row bit 2 is (i & 4) for the former and (g & 1) for the latter in every chunk: per-lane bases, the
  // chunk (512 c) and v (32 v) as immediate offsets
  const int zab = i * 32 + ((8 * g) ^ ((i & 4) << 2));
  const int zbb = 128 * g + (i ^ ((g & 1) << 4));
  // conv2's weight fragments (B of gy1 = gz2 W2): position w, and position 8 for the extra tile
  float wf[8], wf8[8];
  {
    const float4* a = reinterpret_cast<const float4*>(q.w2t + (size_t)((w * 4 + g) * 16 + i) * 8);
    const float4* b = reinterpret_cast<const float4*>(q.w2t + (size_t)((8 * 4 + g) * 16 + i) * 8);
    const float4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
    wf[0] = a0.x; wf[1] = a0.y; wf[2] = a0.z; wf[3] = a0.w; wf[4] = a1.x; wf[5] = a1.y; wf[6] = a1.z; wf[7] = a1.w;
    wf8[0] = b0.x; wf8[1] = b0.y; wf8[2] = b0.z; wf8[3] = b0.w; wf8[4] = b1.x; wf8[5] = b1.y; wf8[6] = b1.z; wf8[7] = b1.w;
  }

  double d0 = 0.0, d1 = 0.0, da2 = 0.0, dc1[4] = {0.0, 0.0, 0.0, 0.0}, dc3[4] = {0.0, 0.0, 0.0, 0.0};
  double dg[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, dg8[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};

  const int nmine = s.nimg > (int)blockIdx.x ? (s.nimg - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  const int nflt = n2 * 32;
  if (nmine > 0) {
    if (staged) sw_dma_image(stem_img(s, blockIdx.x), im0, span, v4, w);
    sw_dma_gz2(q.gz2 + (size_t)blockIdx.x * nflt, gz0, nflt, w);
  }
  __syncthreads();
  for (int k = 0; k < nmine; ++k) {
    const int b = (int)blockIdx.x + k * (int)gridDim.x;
    const float* gim = stem_img(s, b);
    const float* im = (k & 1) ? im1 : im0;
    const float* gzs = (k & 1) ? gz1 : gz0;
    if (k + 1 < nmine) {  // the next image and its gz2 rows into the other buffers, shared by the eight waves
      const long long bn = b + (long long)gridDim.x;
      if (staged) sw_dma_image(stem_img(s, bn), (k & 1) ? im0 : im1, span, v4, w);
      sw_dma_gz2(q.gz2 + (size_t)bn * nflt, (k & 1) ? gz0 : gz1, nflt, w);
    }
    float f0 = 0.0f, f1 = 0.0f, fa2 = 0.0f;
    sm4 c1 = {0.0f, 0.0f, 0.0f, 0.0f}, c3 = {0.0f, 0.0f, 0.0f, 0.0f};
    sm4 ga = {0.0f, 0.0f, 0.0f, 0.0f}, gb = {0.0f, 0.0f, 0.0f, 0.0f};
    sm4 ga8 = {0.0f, 0.0f, 0.0f, 0.0f}, gb8 = {0.0f, 0.0f, 0.0f, 0.0f};
    auto run = [&](auto from_lds) {
      constexpr bool LDS = decltype(from_lds)::value;
      const float* src = LDS ? im : gim;
      // one table-a tile: chunk base zc = 512 c (gz2 floats), pixel offsets oa / ob, the position's W2 fragments, its
      // G2 accumulators
      auto tile = [&](int t, int zc, const int (&oa_)[3], const int (&ob_)[4], const float (&f)[8], sm4& ha, sm4& hb) {
        float pa[3], pb[4];
#pragma unroll
        for (int u = 0; u < 3; ++u) pa[u] = src[oa_[u]];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float p = src[ob_[v]];
          pb[v] = LDS || ((bliv >> (4 * t + v)) & 1u) ? p : 0.0f;
        }
        const float* za = gzs + zc + zab;
        const float4 z0 = *reinterpret_cast<const float4*>(za);
        const float4 z1 = *reinterpret_cast<const float4*>(za + 4);
        float zb[4], zb2[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          zb[v] = gzs[zc + zbb + 32 * v];
          zb2[v] = gzs[zc + (zbb ^ 16) + 32 * v];
        }
        const sm4 x = sm_conv(pa, wb);
        sm4 gyt = {0.0f, 0.0f, 0.0f, 0.0f};
        gyt = sm_mfma(z0.x, f[0], gyt);
        gyt = sm_mfma(z0.y, f[1], gyt);
        gyt = sm_mfma(z0.z, f[2], gyt);
        gyt = sm_mfma(z0.w, f[3], gyt);
        gyt = sm_mfma(z1.x, f[4], gyt);
        gyt = sm_mfma(z1.y, f[5], gyt);
        gyt = sm_mfma(z1.z, f[6], gyt);
        gyt = sm_mfma(z1.w, f[7], gyt);
        float gz[4], xh[4], y1[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          xh[v] = (x[v] - mu) * is;
          const float zz = xh[v] * wv + bv;
          gz[v] = gyt[v] * bn_dact<ACT>(zz, q.slope);
          y1[v] = bn_act<ACT>(zz, q.slope);
          f0 += gz[v];
          f1 += gz[v] * xh[v];
          if constexpr (!MOM) fa2 += pb[v];
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          c1 = sm_mfma(gz[v], pb[v], c1);
          if constexpr (!MOM) c3 = sm_mfma(xh[v], pb[v], c3);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          ha = sm_mfma(y1[v], zb[v], ha);
          hb = sm_mfma(y1[v], zb2[v], hb);
        }
      };
#pragma unroll
      for (int t = 0; t < NM; ++t) {
        if (NCH == 0 && t >= nch) break;  // (wave-uniform; compile-time when NCH > 0)
        tile(t, 512 * t, oa[t], ob[t], wf, ga, gb);
      }
      if (extra) tile(NM, 512 * w, oa[NM], ob[NM], wf8, ga8, gb8);
      // table b's tiles (cells under no conv2 patch: gz = 0; only A3 and A2), to the waves nch .. 7 in turn
      for (int tb = w - nch; !MOM && tb >= 0 && tb < ntb; tb += SW_WAVES - nch) {
        const int r0 = 16 * tb, nv = nbt - r0 < 16 ? nbt - r0 : 16;
        const short* ta = s.pix + (size_t)(na + r0 + (i < nv ? i : 0)) * 9;
        float pa[3] = {src[ta[g]], src[ta[g + 4]], src[ta[8]]};
        float pb[4];
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const bool ok = 4 * g + v < nv && i < 9;
          const float p = src[ok ? s.pix[(size_t)(na + r0 + 4 * g + v) * 9 + i] : 0];
          pb[v] = ok ? p : 0.0f;
          fa2 += pb[v];
        }
        const sm4 x = sm_conv(pa, wb);
#pragma unroll
        for (int v = 0; v < 4; ++v) c3 = sm_mfma((x[v] - mu) * is, pb[v], c3);
      }
    };
    if (staged)
      run(std::true_type{});
    else
      run(std::false_type{});
    d0 += (double)f0;
    d1 += (double)f1;
    da2 += (double)fa2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dc1[r] += (double)c1[r];
      dc3[r] += (double)c3[r];
      dg[r] += (double)ga[r];
      dg[4 + r] += (double)gb[r];
      dg8[r] += (double)ga8[r];
      dg8[4 + r] += (double)gb8[r];
    }
    __syncthreads();  // image k read, image k + 1 staged
  }

  // fixed-order block reductions through the (now free) LDS buffers: >= 2 x 1 024 + 2 x 256 floats
  double* red = reinterpret_cast<double*>(im0);
  red[threadIdx.x] = d0;
  red[SW_THREADS + threadIdx.x] = d1;
  __syncthreads();
  if (threadIdx.x < 32) {  // part[block][2][16]: per channel, the waves in order, then the lane groups in order
    const int qq = threadIdx.x >> 4, c = threadIdx.x & 15;
    double acc = 0.0;
    for (int ww = 0; ww < SW_WAVES; ++ww)
      for (int gg = 0; gg < 4; ++gg) acc += red[qq * SW_THREADS + ww * 64 + gg * 16 + c];
    q.part[(size_t)blockIdx.x * 32 + threadIdx.x] = acc;
  }
#pragma unroll
  for (int a = 0; a < 3; a += 2) {  // A1, A3: lane (g, i) holds [channel 4 g + r][tap i]
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) red[r * SW_THREADS + threadIdx.x] = a == 0 ? dc1[r] : dc3[r];
    __syncthreads();
    for (int v = threadIdx.x; v < 16 * 9; v += SW_THREADS) {
      const int c2 = v / 9, tap = v % 9, lane = (c2 >> 2) * 16 + tap, r = c2 & 3;
      double t = 0.0;
      for (int ww = 0; ww < SW_WAVES; ++ww) t += red[r * SW_THREADS + ww * 64 + lane];
      q.wpart[((size_t)blockIdx.x * 3 + a) * 144 + v] = t;
    }
  }
  __syncthreads();
  red[threadIdx.x] = da2;  // A2[tap i]: the lane groups and waves in order, stored for every channel
  __syncthreads();
  for (int v = threadIdx.x; v < 16 * 9; v += SW_THREADS) {
    const int tap = v % 9;
    double t = 0.0;
    for (int ww = 0; ww < SW_WAVES; ++ww)
      for (int gg = 0; gg < 4; ++gg) t += red[ww * 64 + gg * 16 + tap];
    q.wpart[((size_t)blockIdx.x * 3 + 1) * 144 + v] = t;
  }
  // G2: wave w alone holds position w (written as is); position 8 sums waves 0 .. nch - 1 in order
  double* g2 = q.g2part + (size_t)blockIdx.x * SW_G2;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ch = 4 * g + r;
    g2[(w * 16 + ch) * 32 + i] = dg[r];
    g2[(w * 16 + ch) * 32 + 16 + i] = dg[4 + r];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 8; ++r) red[r * SW_THREADS + threadIdx.x] = dg8[r];
  __syncthreads();
  {
    const int v = threadIdx.x;  // (channel, o) of position 8: v = ch * 32 + o, 512 of them
    const int ch = v >> 5, o = v & 31, r = (ch & 3) + (o >= 16 ? 4 : 0), lane = (ch >> 2) * 16 + (o & 15);
    double t = 0.0;
    for (int ww = 0; ww < nch; ++ww) t += red[r * SW_THREADS + ww * 64 + lane];
    g2[8 * 512 + v] = t;
  }
}

// gconv as stem12_final; gw2[o][j * 16 + ch] = sum over the blocks (in order) of g2part[b][j][ch][o]: block 0 the former,
// blocks 1 .. the latter, 128 columns per block, eight segments of the block range each summing 32 partials in flight
__global__ __launch_bounds__(BN_FINAL_THREADS) void stem12w_final(int blocks, const double* __restrict__ wpart,
                                                                 const double* __restrict__ g2part,
                                                                 const float* __restrict__ sums,
                                                                 const float* __restrict__ stats,
                                                                 const float* __restrict__ bw, double m,
                                                                 const double* __restrict__ mom,
                                                                 const float* __restrict__ cw,
                                                                 float* __restrict__ gw, float* __restrict__ gw2) {
  if (blockIdx.x == 0) {
    __shared__ double tot[3 * 144];
    for (int a = 0; a < (mom ? 1 : 3); ++a) bn_final_sums(wpart + a * 144, 144, blocks, tot + a * 144, 3 * 144);
    if (mom) {
      // A2[tap] = sum p_tap and A3[ch][tap] = sum xhat_ch p_tap over every cell (xhat = (x - mu) is, x = W . p) from
      // the moments of d = p - p0: with c = W . p0 - mu,  sum (x - mu) p_tap = sum_k W_k (M[k][tap] + p0_tap S_k)
      // + c (S_tap + N p0_tap)
      __syncthreads();
      for (int v = threadIdx.x; v < 144; v += BN_FINAL_THREADS) {
        const int ch = v / 9, tap = v % 9;
        const double* S = mom;
        const double* p0 = mom + 54;  // (ST_NM)
        double wp0 = 0.0, acc = 0.0;
        for (int k = 0; k < 9; ++k) {
          const int a = k < tap ? k : tap, b = k < tap ? tap : k;  // M[k][tap] in the upper triangle
          const double mkt = mom[9 + a * 9 - a * (a - 1) / 2 + (b - a)];
          const double wk = (double)cw[ch * 9 + k];
          wp0 += wk * p0[k];
          acc += wk * (mkt + p0[tap] * S[k]);
        }
        const double a2 = S[tap] + m * p0[tap];
        acc += (wp0 - (double)stats[ch]) * a2;
        tot[144 + v] = a2;
        tot[288 + v] = (double)stats[16 + ch] * acc;
      }
      __syncthreads();
    }
    for (int v = threadIdx.x; v < 144; v += BN_FINAL_THREADS) {
      const int ch = v / 9;
      const double mg = (double)sums[ch] / m, mgx = (double)sums[16 + ch] / m;
      const double isw = (double)stats[16 + ch] * (double)bw[ch];
      gw[v] = (float)(isw * (tot[v] - mg * tot[144 + v] - mgx * tot[288 + v]));
    }
    return;
  }
  __shared__ double seg[8][128];
  const int col = (blockIdx.x - 1) * 128 + (threadIdx.x & 127), sg = threadIdx.x >> 7;
  const int per = (blocks + 7) / 8, b0 = sg * per, b1 = b0 + per < blocks ? b0 + per : blocks;
  double acc = 0.0;
  if (col < SW_G2) {
    int b = b0;
    for (; b + 31 < b1; b += 32) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = g2part[(size_t)(b + u) * SW_G2 + col];
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
    for (; b < b1; ++b) acc += g2part[(size_t)b * SW_G2 + col];
  }
  seg[sg][threadIdx.x & 127] = acc;
  __syncthreads();
  if (sg == 0 && col < SW_G2) {
    double t = 0.0;
    for (int u = 0; u < 8; ++u) t += seg[u][threadIdx.x];
    const int o = col & 31, jc = col >> 5;  // jc = j * 16 + ch
    gw2[o * 144 + jc] = (float)t;
  }
}

int stem12w_grid(int nimg) { return nimg < SW_GRID ? (nimg < 1 ? 1 : nimg) : SW_GRID; }

long long stem12w_scratch_doubles(int nimg) {
  const long long gr = stem12w_grid(nimg);
  return gr * 32 + 16 + gr * 3 * 144 + gr * SW_G2;
}

bool stem12w_covers(int n2) { return n2 >= 1 && n2 <= 16 * SW_MAX_CHUNKS; }

// every instantiation opts in to its > 64 KB of dynamic LDS once (the largest any shape needs)
template <int ACT, bool V4, int NCH, bool MOM>
static hipError_t sw_launch_t(int grid, size_t lds, hipStream_t st, const Stem1& s, const Sw12Args& q, int cap) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem12w_kernel<ACT, V4, NCH, MOM>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize,
                                             (int)sw_lds_bytes(16 * SW_MAX_CHUNKS, SM_IMG_CAP));
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((stem12w_kernel<ACT, V4, NCH, MOM>), dim3(grid), dim3(SW_THREADS), lds, st, s, q, cap);
  return hipGetLastError();
}
// 72 x 96 images (five chunks) straight-line; other sizes with the chunk count at run time
template <int ACT, bool V4>
static hipError_t sw_launch(int nch, int grid, size_t lds, hipStream_t st, const Stem1& s, const Sw12Args& q, int cap) {
  if (q.mom)
    return nch == SW_MAX_CHUNKS ? sw_launch_t<ACT, V4, SW_MAX_CHUNKS, true>(grid, lds, st, s, q, cap)
                                : sw_launch_t<ACT, V4, 0, true>(grid, lds, st, s, q, cap);
  return nch == SW_MAX_CHUNKS ? sw_launch_t<ACT, V4, SW_MAX_CHUNKS, false>(grid, lds, st, s, q, cap)
                              : sw_launch_t<ACT, V4, 0, false>(grid, lds, st, s, q, cap);
}

hipError_t launch_stem12_backward_w2(const Stem1& s, const float* bw, const float* bb, const float* stats,
                                     const double* moments, int act, float slope, const float* gz2, int n2,
                                     const float* w2t, float* gconv, float* gbw, float* gbb, float* gw2, double* part,
                                     hipStream_t st) {
  const int grid = stem12w_grid(s.nimg);
  float* sums = reinterpret_cast<float*>(part + (size_t)grid * 32);
  double* wpart = part + (size_t)grid * 32 + 16;
  double* g2part = wpart + (size_t)grid * 3 * 144;
  Sw12Args q{bw, bb, stats, gz2, w2t, part, wpart, g2part, slope, n2, moments};
  long long room = s.ld - s.off;
  const int cap = (int)(room < 1 ? 1 : room < SM_IMG_CAP ? room : SM_IMG_CAP);
  const size_t lds = sw_lds_bytes(n2, cap);
  const bool v4 = ((uintptr_t)(s.obs + s.off) & 15) == 0 && (s.ld & 3) == 0;
  const int nch = (n2 + 15) / 16;
  hipError_t e = hipSuccess;
  if (act == GR_POLICY_ACT_ELU) {
    e = v4 ? sw_launch<GR_POLICY_ACT_ELU, true>(nch, grid, lds, st, s, q, cap)
           : sw_launch<GR_POLICY_ACT_ELU, false>(nch, grid, lds, st, s, q, cap);
  } else {
    e = v4 ? sw_launch<GR_POLICY_ACT_LRELU, true>(nch, grid, lds, st, s, q, cap)
           : sw_launch<GR_POLICY_ACT_LRELU, false>(nch, grid, lds, st, s, q, cap);
  }
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bn_bwd_final, dim3(1), dim3(BN_FINAL_THREADS), 0, st, s.c, grid, part, gbw, gbb, sums);
  hipLaunchKernelGGL(stem12w_final, dim3(1 + (SW_G2 + 127) / 128), dim3(BN_FINAL_THREADS), 0, st, grid, wpart, g2part,
                     sums, stats, bw, (double)s.nimg * (double)(s.na + s.nbt), moments, s.w, gconv, gw2);
  return hipGetLastError();
}


// ------------------------------------------------------------- the first block's apply pass + conv2, y1 not stored
// stem12f_kernel gives each compute wave one 16-patch chunk and all nine positions (the conv2 sum over positions in
// one MFMA chain): five compute waves per image (72 x 96: five chunks) on four SIMDs, two workgroups per CU.  Here a
// unit is (chunk c, position group pg = positions 3 pg .. 3 pg + 2): 15 units per image over eight waves (two per
// SIMD, the next image's staging shared), each unit's pixel offsets and W2 fragments held in registers for the whole
// kernel.  A unit's partial z2 (its three positions) goes to LDS; after the image's barrier every thread sums the
// three partials of its outputs in position-group order (fixed: deterministic) and stores z2.  Partials are double
// buffered, so one barrier per image suffices.  y1 = act(bn(conv1)) exactly as stem12f_kernel computes it (conv1
// transposed, the same expression), z2 = (j 0-2) + (j 3-5) + (j 6-8) in fp32.
constexpr int SG_WAVES = 8;
constexpr int SG_THREADS = 64 * SG_WAVES;
constexpr int SG_UNITS = 3 * SW_MAX_CHUNKS;  // 15
constexpr int SG_PLD = 36;                   // partial rows' stride (floats): 4 row groups on distinct banks
constexpr int SG_PART = 16 * SG_PLD;         // floats per unit partial

__host__ __device__ inline size_t sg_lds_bytes(int cap) {
  return 4 * (2 * (size_t)sw_img_stride(cap) + 2 * (size_t)SG_UNITS * SG_PART);
}

template <int ACT, bool V4, int NCH>
__global__ __launch_bounds__(SG_THREADS) void stem12g_kernel(Stem1 s, Sm12fArgs q, int cap) {
  extern __shared__ float4 sm_dyn4[];
  __shared__ int s_span;
  const int ncell = s.na + s.nbt, n2 = q.n2;
  const int nch = NCH > 0 ? NCH : (n2 + 15) / 16, nun = 3 * nch;
  const int imgf = sw_img_stride(cap);
  float* im0 = reinterpret_cast<float*>(sm_dyn4);
  float* im1 = im0 + imgf;
  float* pt0 = im1 + imgf;
  float* pt1 = pt0 + SG_UNITS * SG_PART;
  const int l = (int)(threadIdx.x & 63), lo = l & 15, kq = l >> 4, w = (int)sm_wave();
  if (threadIdx.x == 0) s_span = 0;
  __syncthreads();
  int mx = 0;
  for (int k = threadIdx.x; k < ncell * 9; k += SG_THREADS) {
    const int t = s.pix[k];
    mx = mx > t + 1 ? mx : t + 1;
  }
  atomicMax(&s_span, mx);
  __syncthreads();
  const int span = s_span;
  const bool staged = span <= cap;
  const bool v4 = V4 && (span & 3) == 0;

  // conv1 as C[channel][cell]: A = W1[channel lo][tap kq + 4 c] (0 for taps >= 9); the lane's channels 4 kq + v
  float wa[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) wa[c] = kq + 4 * c < 9 ? s.w[lo * 9 + kq + 4 * c] : 0.0f;
  float mu[4], is[4], wv[4], bv[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int chn = 4 * kq + v;
    mu[v] = q.stats[chn];
    is[v] = q.stats[16 + chn];
    wv[v] = q.bw[chn];
    bv[v] = q.bb[chn];
  }
  // the wave's units w and w + 8: per position jj of the group, the pixel offsets (cell 9 p + j of patch
  // p = 16 c + lo, clamped below n2: those rows' outputs are never stored) and W2's B fragments for o = lo, 16 + lo
  const bool u1on = w + SG_WAVES < nun;
  int po[2][3][3];
  float4 b0[2][3], b1[2][3];
#pragma unroll
  for (int uu = 0; uu < 2; ++uu) {
    const int u = w + SG_WAVES * uu;
    const bool on = u < nun;
    const int c = on ? u / 3 : 0, pg = on ? u % 3 : 0;
    const int p = 16 * c + lo < n2 ? 16 * c + lo : n2 - 1;
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int j = 3 * pg + jj;
      const short* tt = s.pix + (size_t)(9 * p + j) * 9;
      po[uu][jj][0] = tt[kq];
      po[uu][jj][1] = tt[kq + 4];
      po[uu][jj][2] = tt[8];
      b0[uu][jj] = reinterpret_cast<const float4*>(q.w2f)[(j * 4 + kq) * 32 + lo];
      b1[uu][jj] = reinterpret_cast<const float4*>(q.w2f)[(j * 4 + kq) * 32 + 16 + lo];
    }
  }
  const int nmine = s.nimg > (int)blockIdx.x ? (s.nimg - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x : 0;
  if (staged && nmine > 0) sw_dma_image(stem_img(s, blockIdx.x), im0, span, v4, w);
  __syncthreads();
  for (int k = 0; k < nmine; ++k) {
    const int b = (int)blockIdx.x + k * (int)gridDim.x;
    const float* im = (k & 1) ? im1 : im0;
    float* pt = (k & 1) ? pt1 : pt0;
    if (staged && k + 1 < nmine) sw_dma_image(stem_img(s, b + (long long)gridDim.x), (k & 1) ? im0 : im1, span, v4, w);
    auto run = [&](auto from_lds) {
      const float* src = decltype(from_lds)::value ? im : stem_img(s, b);
      auto unit = [&](int uu) {
        float px[3][3];
#pragma unroll
        for (int jj = 0; jj < 3; ++jj)
#pragma unroll
          for (int c = 0; c < 3; ++c) px[jj][c] = src[po[uu][jj][c]];
        sm4 z0 = {0.0f, 0.0f, 0.0f, 0.0f}, z1 = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          sm4 x = {0.0f, 0.0f, 0.0f, 0.0f};
          x = sm_mfma(wa[0], px[jj][0], x);
          x = sm_mfma(wa[1], px[jj][1], x);
          x = sm_mfma(wa[2], px[jj][2], x);
          float yv[4];
#pragma unroll
          for (int v = 0; v < 4; ++v) yv[v] = bn_act<ACT>((x[v] - mu[v]) * is[v] * wv[v] + bv[v], q.slope);
          const float4 f0 = b0[uu][jj], f1 = b1[uu][jj];
          z0 = sm_mfma(yv[0], f0.x, z0);
          z0 = sm_mfma(yv[1], f0.y, z0);
          z0 = sm_mfma(yv[2], f0.z, z0);
          z0 = sm_mfma(yv[3], f0.w, z0);
          z1 = sm_mfma(yv[0], f1.x, z1);
          z1 = sm_mfma(yv[1], f1.y, z1);
          z1 = sm_mfma(yv[2], f1.z, z1);
          z1 = sm_mfma(yv[3], f1.w, z1);
        }
        // lane (o = lo, kq) holds the unit's partial z2[patch 4 kq + v][o] (z0) and [16 + o] (z1)
        float* pr = pt + (w + SG_WAVES * uu) * SG_PART + 4 * kq * SG_PLD;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          pr[v * SG_PLD + lo] = z0[v];
          pr[v * SG_PLD + 16 + lo] = z1[v];
        }
      };
      if (NCH > 0 || w < nun) unit(0);
      if (u1on) unit(1);
    };
    if (staged)
      run(std::true_type{});
    else
      run(std::false_type{});
    __syncthreads();  // the image's partials written, image k + 1 staged
    // z2[b][p][o] = the three position groups' partials in order (consecutive threads: consecutive o, coalesced)
    for (int qo = (int)threadIdx.x; qo < n2 * 32; qo += SG_THREADS) {
      const int p = qo >> 5, o = qo & 31, c = p >> 4, pl = p & 15;
      const float* a = pt + 3 * c * SG_PART + pl * SG_PLD + o;
      q.z2[((size_t)b * n2 + p) * 32 + o] = (a[0] + a[SG_PART]) + a[2 * SG_PART];
    }
  }
}

template <int ACT, bool V4, int NCH>
static hipError_t sg_launch_t(int grid, size_t lds, hipStream_t st, const Stem1& s, const Sm12fArgs& f, int cap) {
  static bool attr = false;
  if (!attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&stem12g_kernel<ACT, V4, NCH>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)sg_lds_bytes(SM_IMG_CAP));
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((stem12g_kernel<ACT, V4, NCH>), dim3(grid), dim3(SG_THREADS), lds, st, s, f, cap);
  return hipGetLastError();
}
template <int ACT, bool V4>
static hipError_t sg_launch(int nch, int grid, size_t lds, hipStream_t st, const Stem1& s, const Sm12fArgs& f, int cap) {
  return nch == SW_MAX_CHUNKS ? sg_launch_t<ACT, V4, SW_MAX_CHUNKS>(grid, lds, st, s, f, cap)
                              : sg_launch_t<ACT, V4, 0>(grid, lds, st, s, f, cap);
}

hipError_t stem12g_launch(const Stem1& s, const Sm12fArgs& f, int act, hipStream_t st) {
  const int grid = stem12w_grid(s.nimg);
  long long room = s.ld - s.off;
  const int cap = (int)(room < 1 ? 1 : room < SM_IMG_CAP ? room : SM_IMG_CAP);
  const size_t lds = sg_lds_bytes(cap);
  const bool v4 = ((uintptr_t)(s.obs + s.off) & 15) == 0 && (s.ld & 3) == 0;
  const int nch = (f.n2 + 15) / 16;
  if (act == GR_POLICY_ACT_ELU)
    return v4 ? sg_launch<GR_POLICY_ACT_ELU, true>(nch, grid, lds, st, s, f, cap)
              : sg_launch<GR_POLICY_ACT_ELU, false>(nch, grid, lds, st, s, f, cap);
  return v4 ? sg_launch<GR_POLICY_ACT_LRELU, true>(nch, grid, lds, st, s, f, cap)
            : sg_launch<GR_POLICY_ACT_LRELU, false>(nch, grid, lds, st, s, f, cap);
}


// ------------------------------------------------------------- the first block's statistics from pixel moments
// The BatchNorm statistics of conv1's output need, per channel, sum (x - sh) and sum (x - sh)^2 over every cell of
// every image (sh: the channel's value at the first cell of image 0, the shift that keeps the second moment free of
// cancellation).  With d = p - p0 the cell's 9 pixels less those of that first cell, x - sh = W d, so both sums are
// linear in the cell moments: sum (x - sh) = W . sum d and sum (x - sh)^2 = W^T (sum d d^T) W.  A lane therefore
// accumulates the 9 + 45 moments of its cells (63 VALU per cell instead of conv1's 144 FMAs + 48 for the sums), and
// each block turns its fp64 moment sums into the 2 x 16 shifted channel sums bn_stats_final reads.  No LDS staging:
// the workgroup ranks the table's cells by their first pixel (row-major on an image grid) and wave w owns ranks
// 64 w .. 64 w + 63 for every image of its run (9 offsets per lane in registers; a 3 x 3 grid cell is three 12-byte
// loads), four images' pixel loads in flight per lane.  The sums are exact algebra of round 5's (SM_STATS), in
// another order: fp32 per lane, fp64 across lanes, waves and blocks in a fixed order.  24 576 images: 195 us with
// round 5's LDS-staged pass, 176 us here (3.9 TB/s; the bound left is not the access order: strided and contiguous
// image runs measure the same)
// 256 workgroups, four images in flight per lane: measured against two / eight images and 512 / 1 024 workgroups
// (199 / 237 / 205 / 244 vs 195 us before the row-major order, gpurun_out/r6o)
constexpr int ST_GRID = 256;
constexpr int ST_U = 4;  // images in flight per lane
constexpr int ST_NM = 9 + 45;  // moments per lane: sum d_k, sum d_k d_l (l >= k)
constexpr int ST_MSTRIDE = 64;  // a block's moment row in the moment partials
static_assert(ST_NM == 54 && ST_NM + 9 <= 64, "the moment layout stem12w_final reads");

__global__ __launch_bounds__(1024) void stem_stats_kernel(Stem1 s, double* __restrict__ part, float* __restrict__ shift,
                                                         double* __restrict__ mpart) {
  __shared__ double red[16][ST_NM];
  __shared__ double tot[ST_NM];
  __shared__ int key[STEM_MAX_CELLS];
  __shared__ short order[STEM_MAX_CELLS];
  const int ncell = s.na + s.nbt, lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // the cells in the order of their first pixel (the sums do not depend on the order; on an image grid it is
  // row-major, so a wave's loads of one tap row touch a few consecutive lines instead of a scattered patch group):
  // rank by counting (keys are distinct offsets, ties broken by cell index)
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) key[c] = s.pix[(size_t)c * 9];
  __syncthreads();
  for (int c = threadIdx.x; c < ncell; c += blockDim.x) {
    const int kc = key[c];
    int r = 0;
    for (int e = 0; e < ncell; ++e) {
      const int ke = key[e];
      r += (ke < kc || (ke == kc && e < c)) ? 1 : 0;
    }
    order[r] = (short)c;
  }
  __syncthreads();
  const int slot = 64 * w + lane;
  const bool on = slot < ncell;
  const int cell = on ? order[slot] : 0;
  int off[9];
  float p0[9];
  {
    const short* t = s.pix + (size_t)cell * 9;
    const float* i0 = stem_img(s, 0);
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      off[k] = t[k];
      p0[k] = i0[s.pix[k]];  // the first cell of image 0 (the table's cell 0)
    }
  }
  // a 3 x 3 pixel cell of an image row stride W: three 12-byte loads instead of nine (wave-uniform test)
  const int rs = off[3] - off[0];
  bool grid3 = true;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) grid3 = grid3 && off[3 * r + c] == off[0] + r * rs + c;
  grid3 = __all(grid3 || !on) != 0;
  if (blockIdx.x == 0 && threadIdx.x < s.c) {  // sh = conv1 at that cell, stem_conv's k-ordered fmaf chain
    float a = s.w[threadIdx.x * 9] * p0[0];
#pragma unroll
    for (int k = 1; k < 9; ++k) a = __builtin_fmaf(s.w[threadIdx.x * 9 + k], p0[k], a);
    shift[threadIdx.x] = a;
  }
  float sd[9], mm[45];
#pragma unroll
  for (int k = 0; k < 9; ++k) sd[k] = 0.0f;
#pragma unroll
  for (int k = 0; k < 45; ++k) mm[k] = 0.0f;
  // a contiguous run of images per workgroup (measured the same as images strided over the workgroups, r6q)
  const int per = (s.nimg + (int)gridDim.x - 1) / (int)gridDim.x;
  const int bbeg = blockIdx.x * per, bend = bbeg + per < s.nimg ? bbeg + per : s.nimg, bstep = 1;
  for (int b0 = bbeg; b0 < bend; b0 += ST_U * bstep) {
    float px[ST_U][9];
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      const int b = b0 + u * bstep;
      const bool ok = on && b < bend;
      const float* img = stem_img(s, ok ? b : 0);
      if (grid3) {
        typedef float f3 __attribute__((ext_vector_type(3)));
#pragma unroll
        for (int r = 0; r < 3; ++r) {
          f3 v;
          __builtin_memcpy(&v, img + off[3 * r], 12);
          px[u][3 * r] = v.x;
          px[u][3 * r + 1] = v.y;
          px[u][3 * r + 2] = v.z;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 9; ++k) px[u][k] = img[off[k]];
      }
      if (!ok) {
#pragma unroll
        for (int k = 0; k < 9; ++k) px[u][k] = p0[k];  // (d = 0: adds nothing)
      }
    }
#pragma unroll
    for (int u = 0; u < ST_U; ++u) {
      float d[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        d[k] = px[u][k] - p0[k];
        sd[k] += d[k];
      }
      int q = 0;
#pragma unroll
      for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int l = k; l < 9; ++l, ++q) mm[q] = __builtin_fmaf(d[k], d[l], mm[q]);
    }
  }
  // fixed-order reductions: the wave's lanes by xor butterflies in fp64, then the waves in order
  auto wave_sum = [&](float v) {
    double x = (double)v;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
    return x;
  };
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const double v = wave_sum(sd[k]);
    if (lane == 0) red[w][k] = v;
  }
#pragma unroll
  for (int k = 0; k < 45; ++k) {
    const double v = wave_sum(mm[k]);
    if (lane == 0) red[w][9 + k] = v;
  }
  __syncthreads();
  if (threadIdx.x < ST_NM) {
    double t = 0.0;
    for (int ww = 0; ww < nw; ++ww) t += red[ww][threadIdx.x];
    tot[threadIdx.x] = t;
    if (mpart) mpart[(size_t)blockIdx.x * ST_MSTRIDE + threadIdx.x] = t;  // (the backward's A2 / A3, stem_moments_final)
  }
  if (mpart && blockIdx.x == 0 && threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < 9; ++k) mpart[(size_t)gridDim.x * ST_MSTRIDE + k] = (double)p0[k];
  }
  __syncthreads();
  if (threadIdx.x < 2 * s.c) {  // part[block][0][ch] = W . S, [1][ch] = W^T M W (fp64)
    const int ch = threadIdx.x % s.c;
    double wk[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) wk[k] = (double)s.w[ch * 9 + k];
    double r = 0.0;
    if (threadIdx.x < s.c) {
#pragma unroll
      for (int k = 0; k < 9; ++k) r += wk[k] * tot[k];
    } else {
      int q = 0;
#pragma unroll
      for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int l = k; l < 9; ++l, ++q) r += (l == k ? 1.0 : 2.0) * wk[k] * wk[l] * tot[9 + q];
    }
    part[(size_t)blockIdx.x * 2 * s.c + threadIdx.x] = r;
  }
}

// the moment totals for gr_stem12_backward_w2: mom[0 .. 8] = sum d, [9 .. 53] = sum d d^T (upper triangle, row-major),
// [54 .. 62] = p0 (the first cell of image 0), all fp64.  Eight segments of the block range, each summing its blocks
// in order with 32 loads in flight, then the segments in order (a single 64-lane loop over 256 blocks: 96 us)
__global__ __launch_bounds__(512) void stem_moments_final(const double* __restrict__ mpart, int grid, double* __restrict__ mom) {
  __shared__ double seg[8][ST_MSTRIDE];
  const int t = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int per = (grid + 7) / 8, b0 = sg * per, b1 = b0 + per < grid ? b0 + per : grid;
  double acc = 0.0;
  if (t < ST_NM) {
    int b = b0;
    for (; b + 31 < b1; b += 32) {
      double v[32];
#pragma unroll
      for (int u = 0; u < 32; ++u) v[u] = mpart[(size_t)(b + u) * ST_MSTRIDE + t];
#pragma unroll
      for (int u = 0; u < 32; ++u) acc += v[u];
    }
    for (; b < b1; ++b) acc += mpart[(size_t)b * ST_MSTRIDE + t];
  }
  seg[sg][t] = acc;
  __syncthreads();
  if (sg == 0) {
    if (t < ST_NM) {
      double a = 0.0;
      for (int u = 0; u < 8; ++u) a += seg[u][t];
      mom[t] = a;
    } else if (t < ST_NM + 9) {
      mom[t] = mpart[(size_t)grid * ST_MSTRIDE + (t - ST_NM)];
    } else {
      mom[t] = 0.0;
    }
  }
}

int stem_stats_launch(const Stem1& s, double* part, float* shift, hipStream_t st, double* mpart, double* mom) {
  const int ncell = s.na + s.nbt;
  const int nw = (ncell + 63) / 64;
  // (no more partial rows than the callers' workspace holds before the shift: stem_blocks(s), gr_stem1_scratch_doubles)
  const int nb = stem_blocks(s);
  int grid = s.nimg < ST_GRID ? (s.nimg < 1 ? 1 : s.nimg) : ST_GRID;
  grid = grid < nb ? grid : nb;
  hipLaunchKernelGGL(stem_stats_kernel, dim3(grid), dim3(64 * nw), 0, st, s, part, shift, mom ? mpart : nullptr);
  if (mom) hipLaunchKernelGGL(stem_moments_final, dim3(1), dim3(512), 0, st, mpart, grid, mom);
  return grid;
}

}  // namespace gr
