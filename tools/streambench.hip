// Floor references for the fused step on gfx950, same launch shape and bytes as
// env step at 65 536 envs (256 workgroups x 512 threads, hipGraph of 64 launches):
//   empty  : launch + end-of-kernel cost alone
//   stream : each env reads 16 float4 (256 B) and writes 18 float4 (288 B), all coalesced,
//            i.e. the step's algorithmic traffic with no arithmetic
//   hipcc --offload-arch=gfx950 -O3 -o build/streambench tools/streambench.hip && build/streambench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 65536, RD = 16, WR = 18;

__global__ __launch_bounds__(512) void empty_kernel(float* out) {
  if (threadIdx.x == 1023) out[0] = 0.0f;  // never true: keeps the kernel
}

__global__ __launch_bounds__(512) void stream_kernel(const float4* __restrict__ in, float4* __restrict__ out) {
  const int t = threadIdx.x & 255, role = threadIdx.x >> 8;
  const int i = blockIdx.x * 256 + t;
  if (role == 0) {
    float4 acc = make_float4(0, 0, 0, 0);
    float4 v[RD];
#pragma unroll
    for (int k = 0; k < RD; ++k) v[k] = in[(size_t)k * N + i];
#pragma unroll
    for (int k = 0; k < RD; ++k) { acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w; }
#pragma unroll
    for (int k = 0; k < WR / 2; ++k) out[(size_t)k * N + i] = make_float4(acc.x + k, acc.y, acc.z, acc.w);
  } else {
#pragma unroll
    for (int k = WR / 2; k < WR; ++k) out[(size_t)k * N + i] = make_float4((float)k, 0, 0, (float)i);
  }
}

template <typename F>
double time_graph(F launch) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int k = 0; k < 8; ++k) launch(s);
  (void)hipStreamSynchronize(s);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int k = 0; k < 64; ++k) launch(s);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int reps = 50;
  (void)hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3 / (reps * 64);
}

int main() {
  float4 *in, *out;
  (void)hipMalloc(&in, (size_t)RD * N * 16);
  (void)hipMalloc(&out, (size_t)WR * N * 16);
  (void)hipMemset(in, 0, (size_t)RD * N * 16);
  const double te = time_graph([&](hipStream_t s) {
    hipLaunchKernelGGL(empty_kernel, dim3(N / 256), dim3(512), 0, s, reinterpret_cast<float*>(out));
  });
  const double tl = time_graph([&](hipStream_t s) {
    hipLaunchKernelGGL(empty_kernel, dim3(N / 256), dim3(512), 58 * 1024, s, reinterpret_cast<float*>(out));
  });
  const double ts = time_graph([&](hipStream_t s) {
    hipLaunchKernelGGL(stream_kernel, dim3(N / 256), dim3(512), 0, s, in, out);
  });
  const double bytes = (double)N * (RD + WR) * 16;
  printf("{\"empty_us\": %.3f, \"empty_58KiB_lds_us\": %.3f, \"stream_us\": %.3f, \"stream_GBps\": %.1f, "
         "\"bytes\": %.0f}\n", te, tl, ts, bytes / (ts * 1e-6) / 1e9, bytes);
  return 0;
}
