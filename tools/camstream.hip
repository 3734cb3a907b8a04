// HBM floor references for the depth-camera kernel at 65 536 envs (GB-sized: far beyond the
// 256 MB Infinity Cache, unlike tools/streambench.hip whose 36 MB fit in it):
//   copy_rows : the reuse call's traffic with no arithmetic — per env (one wave) read the
//               27 648-B depth image, write it into two 27 712-B obs rows at +64 B
//               (the layout gr_camera_render writes), 1 KB float4 accesses
//   read_only : read the same 1.8 GB;  write_only : write the same 3.6 GB
//   hipcc --offload-arch=gfx950 -O3 -o build/camstream tools/camstream.hip && build/camstream
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int N = 65536, NPIX = 6912, ROW = 16 + NPIX, NQ = NPIX / 4;

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy_rows(const float4* __restrict__ dep, float* __restrict__ op,
                                                 float* __restrict__ oc, int nt) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float4* d = dep + (size_t)i * NQ;
  float4* p = reinterpret_cast<float4*>(op + (size_t)i * ROW + 16);
  float4* c = reinterpret_cast<float4*>(oc + (size_t)i * ROW + 16);
  for (int q0 = 0; q0 < NQ; q0 += 64 * 3) {
    float4 v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = d[q0 + 64 * j + lane];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int q = q0 + 64 * j + lane;
      if (nt) {
        const v4f x = {v[j].x, v[j].y, v[j].z, v[j].w};
        __builtin_nontemporal_store(x, reinterpret_cast<v4f*>(p + q));
        __builtin_nontemporal_store(x * 0.1f, reinterpret_cast<v4f*>(c + q));
      } else {
        p[q] = v[j];
        c[q] = make_float4(v[j].x * 0.1f, v[j].y, v[j].z, v[j].w);
      }
    }
  }
}

__global__ __launch_bounds__(256) void read_only(const float4* __restrict__ dep, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const float4* d = dep + (size_t)i * NQ;
  float acc = 0.0f;
  for (int q0 = 0; q0 < NQ; q0 += 64 * 3) {
    float4 v[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) v[j] = d[q0 + 64 * j + lane];
#pragma unroll
    for (int j = 0; j < 3; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
  }
  if (acc == 1234.5f) out[i] = acc;
}

__global__ __launch_bounds__(256) void write_only(float* __restrict__ op, float* __restrict__ oc) {
  const int lane = threadIdx.x & 63, i = blockIdx.x * 4 + (threadIdx.x >> 6);
  float4* p = reinterpret_cast<float4*>(op + (size_t)i * ROW + 16);
  float4* c = reinterpret_cast<float4*>(oc + (size_t)i * ROW + 16);
  for (int q = lane; q < NQ; q += 64) {
    p[q] = make_float4((float)q, 0, 0, 0);
    c[q] = make_float4(0, (float)q, 0, 0);
  }
}

template <typename F>
float time_ms(F launch) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int k = 0; k < 3; ++k) launch();
  (void)hipDeviceSynchronize();
  const int reps = 20;
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; ++r) launch();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  float *dep, *op, *oc, *out;
  (void)hipMalloc(&dep, sizeof(float) * (size_t)N * NPIX);
  (void)hipMalloc(&op, sizeof(float) * (size_t)N * ROW);
  (void)hipMalloc(&oc, sizeof(float) * (size_t)N * ROW);
  (void)hipMalloc(&out, sizeof(float) * N);
  (void)hipMemset(dep, 0, sizeof(float) * (size_t)N * NPIX);
  const double rd = 4.0 * N * NPIX, wr = 2.0 * 4.0 * N * NPIX;
  const dim3 g(N / 4), b(256);
  float t_copy = time_ms([&] { hipLaunchKernelGGL(copy_rows, g, b, 0, 0, (const float4*)dep, op, oc, 0); });
  float t_copy_nt = time_ms([&] { hipLaunchKernelGGL(copy_rows, g, b, 0, 0, (const float4*)dep, op, oc, 1); });
  float t_rd = time_ms([&] { hipLaunchKernelGGL(read_only, g, b, 0, 0, (const float4*)dep, out); });
  float t_wr = time_ms([&] { hipLaunchKernelGGL(write_only, g, b, 0, 0, op, oc); });
  printf("{\"copy_rows_ms\": %.4f, \"copy_rows_GBps\": %.1f, \"copy_rows_nt_ms\": %.4f, \"copy_rows_nt_GBps\": %.1f, "
         "\"read_only_ms\": %.4f, \"read_GBps\": %.1f, \"write_only_ms\": %.4f, \"write_GBps\": %.1f, "
         "\"bytes_copy\": %.0f}\n",
         t_copy, (rd + wr) / (t_copy * 1e6), t_copy_nt, (rd + wr) / (t_copy_nt * 1e6), t_rd, rd / (t_rd * 1e6), t_wr,
         wr / (t_wr * 1e6), rd + wr);
  return 0;
}
