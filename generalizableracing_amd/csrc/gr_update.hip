// gr_update.hip — the PPO update's memory-bound pieces: column sums for the bias gradients (rsl_rl/linear.py
// bias_grad) and the MLP head fused with its LeakyReLU (rsl_rl/linear.py LeakyHead, below).
//
// db = sum over the rows of dY [M, N] for the tall mini-batches of the update (M up to ~4e5 rows,
// N = 256 / 4 / 1).  Two launches, no atomics, fixed summation order (deterministic, and safe inside a
// captured hipGraph: the partial-sum buffer is the caller's):
//   1. colsum_partial: workgroup b sums rows [b R, (b + 1) R) of every column into part[b][N].  Threads map
//      to (row phase, column) so one wave instruction reads consecutive bytes of consecutive rows;
//   2. colsum_final: 64 columns per workgroup, its 16 waves sum a sixteenth of the partial rows each (four
//      loads in flight per lane), combined in LDS in wave order.
// HBM-bound: M N sizeof(T) bytes read once.
#include <hip/hip_runtime.h>

#include "../../include/gr.h"
#include "gr_kernels.h"

namespace gr {

constexpr int CS_THREADS = 256;

__device__ __forceinline__ float cs_load(const float* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ float cs_load(const unsigned short* p) {
  return __uint_as_float((unsigned)__builtin_nontemporal_load(p) << 16);
}

template <typename T>
__global__ __launch_bounds__(CS_THREADS) void colsum_partial(const T* __restrict__ x, long long m, int n, int rows,
                                                             float* __restrict__ part) {
  __shared__ float sm[CS_THREADS];
  const int t = threadIdx.x;
  const long long r0 = (long long)blockIdx.x * rows;
  const long long r1 = r0 + rows < m ? r0 + rows : m;
  if (n <= CS_THREADS) {
    const int step = CS_THREADS / n;  // rows per pass
    const int c = t % n, ph = t / n;
    float acc = 0.0f;
    if (ph < step) {
      long long r = r0 + ph;
      float a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
      for (; r + 3 * step < r1; r += 4 * step) {  // four independent loads in flight per thread
        acc += cs_load(x + r * n + c);
        a1 += cs_load(x + (r + step) * n + c);
        a2 += cs_load(x + (r + 2 * step) * n + c);
        a3 += cs_load(x + (r + 3 * step) * n + c);
      }
      for (; r < r1; r += step) acc += cs_load(x + r * n + c);
      acc = (acc + a1) + (a2 + a3);
    }
    sm[t] = acc;
    __syncthreads();
    if (t < n) {
      float s = 0.0f;
      for (int p = 0; p < step; ++p) s += sm[p * n + t];
      part[(size_t)blockIdx.x * n + t] = s;
    }
  } else {
    for (int c = t; c < n; c += CS_THREADS) {
      float acc = 0.0f;
      for (long long r = r0; r < r1; ++r) acc += cs_load(x + r * n + c);
      part[(size_t)blockIdx.x * n + c] = acc;
    }
  }
}

constexpr int CF_WAVES = 16;  // waves per final workgroup: the partial rows are split over them

__global__ __launch_bounds__(CF_WAVES * 64) void colsum_final(const float* __restrict__ part, int blocks, int n,
                                                              float* __restrict__ out) {
  __shared__ float sm[CF_WAVES * 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  // wave w sums partial rows w, w + 16, ...: four loads in flight per lane
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
  if (c < n) {
    int b = w;
    for (; b + 3 * CF_WAVES < blocks; b += 4 * CF_WAVES) {
      a0 += part[(size_t)b * n + c];
      a1 += part[(size_t)(b + CF_WAVES) * n + c];
      a2 += part[(size_t)(b + 2 * CF_WAVES) * n + c];
      a3 += part[(size_t)(b + 3 * CF_WAVES) * n + c];
    }
    for (; b < blocks; b += CF_WAVES) a0 += part[(size_t)b * n + c];
  }
  sm[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && c < n) {
    float s = 0.0f;
    for (int k = 0; k < CF_WAVES; ++k) s += sm[k * 64 + lane];
    out[c] = s;
  }
}

int column_sum_blocks(long long m) {
  long long b = (m + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

hipError_t launch_column_sum(const void* x, int dtype, long long m, int n, float* part, float* out, hipStream_t s) {
  const int blocks = column_sum_blocks(m);
  const int rows = (int)((m + blocks - 1) / blocks);
  if (dtype == GR_DTYPE_BF16)
    hipLaunchKernelGGL(colsum_partial<unsigned short>, dim3(blocks), dim3(CS_THREADS), 0, s,
                       static_cast<const unsigned short*>(x), m, n, rows, part);
  else
    hipLaunchKernelGGL(colsum_partial<float>, dim3(blocks), dim3(CS_THREADS), 0, s, static_cast<const float*>(x), m,
                       n, rows, part);
  hipLaunchKernelGGL(colsum_final, dim3((n + 63) / 64), dim3(CF_WAVES * 64), 0, s, part, blocks, n, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// The MLP head fused with the LeakyReLU in front of it (rsl_rl/linear.py LeakyHead): for the actor's / critic's last
// Linear (out k <= 8 features, in h <= 256) on the update's tall mini-batches.  z [M][h] is the pre-activation of
// the last hidden layer, W [k][h], b [k].
//   forward : y = lrelu(z) W^T + b                                   (reads z once; no activation pass, no GEMM)
//   backward: gz = (gy W) * lrelu'(z),  gW = gy^T lrelu(z),  gb = sum gy   (reads z and gy once, writes gz)
// torch would run, per mini-batch and network: the LeakyReLU forward (read z, write h), the head GEMM (read h), the
// head's input-gradient GEMM (write gh; a K <= 8 GEMM on general tiles), the LeakyReLU backward (read gh and z,
// write gz), the head's weight-gradient GEMM (read gy, h) and its bias sum.  A wave owns a row at a time, lane l
// columns 4l .. 4l + 3 (one 1 KB coalesced access per row); the weight / bias gradients are per-workgroup partial
// sums reduced in a fixed order by head_final (deterministic, graph-capturable, no atomics).
constexpr int HD_WAVES = 4;
typedef float hd_v4 __attribute__((ext_vector_type(4)));
constexpr int HD_MAXK = 8;

__device__ __forceinline__ float hd_act(float z, float slope) { return z > 0.0f ? z : z * slope; }
__device__ __forceinline__ float hd_der(float z, float slope) { return z > 0.0f ? 1.0f : slope; }

// forward: a wave takes 4 rows at a time, 16 lanes per row; lane q of a row holds columns 4 q + 64 j (j < 4), so
// each load instruction reads 256 contiguous bytes of every row and a row's dot products reduce over 16 lanes
template <int K>
__global__ __launch_bounds__(HD_WAVES * 64) void head_forward(const float* __restrict__ z, long long m, int h,
                                                              const float* __restrict__ w,
                                                              const float* __restrict__ b, float slope,
                                                              float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 15, sub = lane >> 4;
  float wr[K][16];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = 4 * q + 64 * j;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) wr[k][4 * j + e] = c < h ? w[(size_t)k * h + c + e] : 0.0f;
  }
  const long long stride = (long long)gridDim.x * HD_WAVES * 4;
  for (long long r0 = ((long long)blockIdx.x * HD_WAVES + (threadIdx.x >> 6)) * 4; r0 < m; r0 += stride) {
    const long long r = r0 + sub;
    float acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0f;
    if (r < m) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = 4 * q + 64 * j;
        hd_v4 zz = {0.0f, 0.0f, 0.0f, 0.0f};
        if (c < h) zz = __builtin_nontemporal_load(reinterpret_cast<const hd_v4*>(z + r * h + c));
        const float a[4] = {hd_act(zz.x, slope), hd_act(zz.y, slope), hd_act(zz.z, slope), hd_act(zz.w, slope)};
#pragma unroll
        for (int k = 0; k < K; ++k)
          acc[k] += ((a[0] * wr[k][4 * j] + a[1] * wr[k][4 * j + 1]) + a[2] * wr[k][4 * j + 2]) + a[3] * wr[k][4 * j + 3];
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1) acc[k] += __shfl_xor(acc[k], off);
    if (r < m && q < K) {
      float v = acc[0];
#pragma unroll
      for (int k = 1; k < K; ++k) v = q == k ? acc[k] : v;
      y[r * K + q] = v + b[q];
    }
  }
}

template <int K>
__global__ __launch_bounds__(HD_WAVES * 64) void head_backward(const float* __restrict__ z,
                                                               const float* __restrict__ gy, long long m, int h,
                                                               const float* __restrict__ w, float slope, int rows,
                                                               float* __restrict__ gz, float* __restrict__ part) {
  __shared__ float sm[HD_WAVES][K * 256 + K];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = 4 * lane;
  const bool on = c < h;
  float wr[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[k][j] = on ? w[(size_t)k * h + c + j] : 0.0f;
  float gw[K][4], gb[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    gb[k] = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) gw[k][j] = 0.0f;
  }
  const long long r0 = (long long)blockIdx.x * rows;
  const long long r1 = r0 + rows < m ? r0 + rows : m;
  constexpr int U = 4;  // rows in flight per wave (their loads issued together)
  for (long long rb = r0 + wv; rb < r1; rb += U * HD_WAVES) {
    float g[U][K];
    hd_v4 zz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = rb + (long long)u * HD_WAVES;
      const bool ok = r < r1;
#pragma unroll
      for (int k = 0; k < K; ++k) g[u][k] = ok ? gy[r * K + k] : 0.0f;
      zz[u] = hd_v4{0.0f, 0.0f, 0.0f, 0.0f};
      if (on && ok) zz[u] = __builtin_nontemporal_load(reinterpret_cast<const hd_v4*>(z + r * h + c));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long r = rb + (long long)u * HD_WAVES;
      const float zv[4] = {zz[u].x, zz[u].y, zz[u].z, zz[u].w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gh = g[u][0] * wr[0][j];
#pragma unroll
        for (int k = 1; k < K; ++k) gh += g[u][k] * wr[k][j];
        o[j] = gh * hd_der(zv[j], slope);
        const float a = hd_act(zv[j], slope);
#pragma unroll
        for (int k = 0; k < K; ++k) gw[k][j] += g[u][k] * a;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) gb[k] += g[u][k];
      if (on && r < r1) {
        const hd_v4 ov = {o[0], o[1], o[2], o[3]};
        __builtin_nontemporal_store(ov, reinterpret_cast<hd_v4*>(gz + r * h + c));
      }
    }
  }
  // the workgroup's partial sums, waves combined in order: part[block][k * h + col], then part[block][k * h + k']
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int j = 0; j < 4; ++j) sm[wv][k * 256 + c + j] = gw[k][j];
    if (lane == 0) sm[wv][K * 256 + k] = gb[k];
  }
  __syncthreads();
  float* pb = part + (size_t)blockIdx.x * (K * h + K);
  for (int i = threadIdx.x; i < K * 256 + K; i += HD_WAVES * 64) {
    const bool bias = i >= K * 256;
    const int k = bias ? i - K * 256 : i / 256, col = bias ? 0 : i % 256;
    if (!bias && col >= h) continue;
    float v = sm[0][i];
#pragma unroll
    for (int q = 1; q < HD_WAVES; ++q) v += sm[q][i];
    pb[bias ? K * h + k : k * h + col] = v;
  }
}

// gw [k][h] and gb [k] from the per-workgroup partials [blocks][k h + k]: 64 outputs per workgroup, its 16 waves
// sum a sixteenth of the partial rows each (four loads in flight per lane), combined in LDS in wave order
__global__ __launch_bounds__(CF_WAVES * 64) void head_final(const float* __restrict__ part, int blocks, int n,
                                                            float* __restrict__ gw, float* __restrict__ gb, int nw) {
  __shared__ float sm[CF_WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
  if (i < n) {
    int b = wv;
    for (; b + 3 * CF_WAVES < blocks; b += 4 * CF_WAVES) {
      a0 += part[(size_t)b * n + i];
      a1 += part[(size_t)(b + CF_WAVES) * n + i];
      a2 += part[(size_t)(b + 2 * CF_WAVES) * n + i];
      a3 += part[(size_t)(b + 3 * CF_WAVES) * n + i];
    }
    for (; b < blocks; b += CF_WAVES) a0 += part[(size_t)b * n + i];
  }
  sm[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wv == 0 && i < n) {
    float s = 0.0f;
    for (int k = 0; k < CF_WAVES; ++k) s += sm[k * 64 + lane];
    if (i < nw)
      gw[i] = s;
    else
      gb[i - nw] = s;
  }
}

int head_blocks(long long m) {
  long long b = (m + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

#define HD_DISPATCH(KK, ...)                   \
  switch (KK) {                                \
    case 1: __VA_ARGS__(1); break;             \
    case 2: __VA_ARGS__(2); break;             \
    case 3: __VA_ARGS__(3); break;             \
    case 4: __VA_ARGS__(4); break;             \
    case 5: __VA_ARGS__(5); break;             \
    case 6: __VA_ARGS__(6); break;             \
    case 7: __VA_ARGS__(7); break;             \
    default: __VA_ARGS__(8); break;            \
  }

hipError_t launch_head_forward(const float* z, long long m, int h, const float* w, const float* b, int k, float slope,
                               float* y, hipStream_t s) {
  const long long fb = (m + 127) / 128;  // ~8 row groups of 4 per wave: enough loads in flight
  const int blocks = (int)(fb < 1 ? 1 : (fb > 8192 ? 8192 : fb));
#define HD_FWD(KK) \
  hipLaunchKernelGGL(head_forward<KK>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, z, m, h, w, b, slope, y)
  HD_DISPATCH(k, HD_FWD)
#undef HD_FWD
  return hipGetLastError();
}

hipError_t launch_head_backward(const float* z, const float* gy, long long m, int h, const float* w, int k,
                                float slope, float* gz, float* part, float* gw, float* gb, hipStream_t s) {
  const int blocks = head_blocks(m);
  const int rows = (int)((m + blocks - 1) / blocks);
#define HD_BWD(KK)                                                                                               \
  hipLaunchKernelGGL(head_backward<KK>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, z, gy, m, h, w, slope, rows, gz, \
                     part)
  HD_DISPATCH(k, HD_BWD)
#undef HD_BWD
  const int n = k * h + k;
  hipLaunchKernelGGL(head_final, dim3((n + 63) / 64), dim3(CF_WAVES * 64), 0, s, part, blocks, n, gw, gb, k * h);
  return hipGetLastError();
}

}  // namespace gr
