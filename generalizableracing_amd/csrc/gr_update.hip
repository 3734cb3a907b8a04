// gr_update.hip — column sums for the PPO update's bias gradients (rsl_rl/linear.py bias_grad).
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

}  // namespace gr
