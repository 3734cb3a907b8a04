// Cycle cost of the portable math / RNG building blocks on gfx950 (one wave per
// SIMD on every CU, dependent chains, s_memtime).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o build/mathbench tools/mathbench.hip && build/mathbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../generalizableracing_amd/csrc/gr_rng.h"

#define ITERS 256

// Philox variants for the cost model: fully unrolled; mul_hi/mul_lo instead of mad_u64
__device__ __forceinline__ gr_u32x4 philox_unrolled(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                    uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1; c3 = (uint32_t)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  gr_u32x4 r = {c0, c1, c2, c3};
  return r;
}
__device__ __forceinline__ gr_u32x4 philox_hilo(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c1 = lo1; c3 = lo0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  gr_u32x4 r = {c0, c1, c2, c3};
  return r;
}

template <int F>
__device__ __forceinline__ float step(float x, uint32_t& u, uint32_t k0, uint32_t k1) {
  if (F == 0) { gr_u32x4 r = gr_philox4x32_10(u, u ^ 1u, 7u, 9u, k0, k1); u = r.x ^ r.y ^ r.z ^ r.w; return x; }
  if (F == 1) { float a, b; gr_box_muller(u, u * 747796405u, &a, &b); u += gr_f2u(a + b); return x; }
  if (F == 2) { float s, c; gr_sincosf(x, &s, &c); return s + c; }
  if (F == 3) return gr_logf(x + 1.5f);
  if (F == 4) return gr_expf(x * 0.01f);
  if (F == 5) return gr_tanhf(x);
  if (F == 6) return gr_atan2f(x, 1.25f - x);
  if (F == 7) return 1.0f / (x + 1.5f);
  if (F == 8) return gr_sqrtf(x + 2.0f);
  if (F == 9) return x * 1.0001f + 0.5f;  // mul + add (no contraction)
  if (F == 10) { gr_u32x4 r = philox_unrolled(u, u ^ 1u, 7u, 9u, k0, k1); u = r.x ^ r.y ^ r.z ^ r.w; return x; }
  if (F == 11) { gr_u32x4 r = philox_hilo(u, u ^ 1u, 7u, 9u, k0, k1); u = r.x ^ r.y ^ r.z ^ r.w; return x; }
  if (F == 12) {  // four independent unrolled draws per iteration (ILP), cost per call = /4
    gr_u32x4 a = philox_unrolled(u, 1u, 7u, 9u, k0, k1), b = philox_unrolled(u, 2u, 7u, 9u, k0, k1);
    gr_u32x4 c = philox_unrolled(u, 3u, 7u, 9u, k0, k1), d = philox_unrolled(u, 4u, 7u, 9u, k0, k1);
    u = a.x ^ b.y ^ c.z ^ d.w;
    return x;
  }
  return x;
}

template <int F>
__global__ __launch_bounds__(256) void bench(unsigned long long* out, float* sink, uint32_t k0, uint32_t k1) {
  float x = 0.1f + threadIdx.x * 1e-3f;
  uint32_t u = threadIdx.x * 2654435761u + blockIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) x = step<F>(x, u, k0, k1);
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  sink[blockIdx.x * 256 + threadIdx.x] = x + (float)u;
}

template <int F>
double run(unsigned long long* d_out, float* d_sink, int blocks) {
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(bench<F>, dim3(blocks), dim3(256), 0, 0, d_out, d_sink, 1u, 2u);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(blocks * 4);
  (void)hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost);
  std::vector<unsigned long long> s(h);
  std::sort(s.begin(), s.end());
  return (double)s[s.size() / 2] / ITERS;
}

#include <algorithm>
int main() {
  const int blocks = 256;
  unsigned long long* d_out;
  float* d_sink;
  (void)hipMalloc(&d_out, blocks * 4 * 8);
  (void)hipMalloc(&d_sink, blocks * 256 * 4);
  const char* names[] = {"philox4x32_10", "box_muller", "sincos", "log", "exp", "tanh", "atan2", "div", "sqrt",
                         "mul+add", "philox_unrolled", "philox_mulhi_lo", "philox_unrolled_x4_ilp(per 4)"};
  double c[13] = {run<0>(d_out, d_sink, blocks), run<1>(d_out, d_sink, blocks), run<2>(d_out, d_sink, blocks),
                  run<3>(d_out, d_sink, blocks), run<4>(d_out, d_sink, blocks), run<5>(d_out, d_sink, blocks),
                  run<6>(d_out, d_sink, blocks), run<7>(d_out, d_sink, blocks), run<8>(d_out, d_sink, blocks),
                  run<9>(d_out, d_sink, blocks), run<10>(d_out, d_sink, blocks), run<11>(d_out, d_sink, blocks),
                  run<12>(d_out, d_sink, blocks)};
  printf("{");
  for (int i = 0; i < 13; ++i) printf("%s\"%s\": %.1f", i ? ", " : "", names[i], c[i]);
  printf("}\n");
  return 0;
}
