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

// ------------------------------------------------------------- BatchNorm + activation applied on load
// A patch GEMM whose input is act(bn(z)) (the vision stem's block 2 feeding conv3) can read z and apply the
// BatchNorm's batch statistics and the activation as it loads, so act(bn(z)) is never written nor read back.  The
// arithmetic is bn_apply's (gr_bn.hip): act(((z - mean) * invstd) * w + b), no contraction, so the values are
// bit-identical to the materialised rows.  Column k of the patch rows is channel k % c.
// (struct BnAct: gr_kernels.h)
__device__ __forceinline__ float bnact_apply(float z, float mu, float is, float w, float b, int act, float slope) {
  const float y = (z - mu) * is * w + b;
  return act == GR_POLICY_ACT_ELU ? (y > 0.0f ? y : expm1f(y)) : (y > 0.0f ? y : y * slope);
}
// four consecutive channels' parameters c0 .. c0 + 3
struct BnAct4 {
  float mu[4], is[4], w[4], b[4];
};
__device__ __forceinline__ BnAct4 bnact_params(const BnAct& p, int c0) {
  BnAct4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r.mu[e] = p.stats[c0 + e];
    r.is[e] = p.stats[p.c + c0 + e];
    r.w[e] = p.w[c0 + e];
    r.b[e] = p.b[c0 + e];
  }
  return r;
}

// ------------------------------------------------------------------ weight gradient of a tall patch GEMM
// gw[n][K] = gy[M][n]^T x[M][K] over up to millions of rows, in slabs of N = 16 NT outputs (32 or 64): the vision
// stem's conv2 (x = its input patches [M][144], n 32), conv3 ([M][128], n 64) and its final Linear ([M][1280],
// n 192): hipBLASLt's split-K tiles streamed them at 1.3-3.7 TB/s.  A workgroup takes a run of rows and one slab
// of N outputs x 16 KT columns (blockIdx.y; x rows ld floats apart, gy rows n); each wave holds its rows' whole [N][16 KT] product in MFMA accumulators
// (NT x KT tiles of v_mfma_f32_16x16x4f32).  Per four rows (the k step) lane (i = l % 16, g = l / 16) supplies row
// g's gy columns NT i .. NT i + NT - 1 (A of tiles nt: output row NT i + nt) and the slab's x columns KT i .. KT i +
// KT - 1 (B of tiles kt: column KT i + kt), read as float2 / float4 loads (measured faster than float4 loads of
// columns 64 q + 4 i, which read each 256-byte stretch whole); pw_depth row quads per register set, the next set's
// loads in flight under the current set's MFMAs.  The workgroup's wave sums are added in wave order through LDS
// into its row of partials [N][K], and colsum_final sums the rows in order: deterministic, no atomics.
constexpr int PW_WAVES = 4;
// row quads per register set: 2 for 32 outputs (same-box A/B, r5pw6: depth 2 307 us, 3 319, 4 325; more workgroups
// no faster), 1 for 64 (the accumulators take 128 registers)
template <int NT>
constexpr int pw_depth() { return NT == 2 ? 2 : 1; }
typedef float pw4 __attribute__((ext_vector_type(4)));
typedef float pw4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float pw2u __attribute__((ext_vector_type(2), aligned(4)));

// (64 outputs: two waves per SIMD, which the compiler fits in 182 registers without spilling; same-box A/B r5pwi:
// conv3 112 -> 96 us, the Linear 189 -> 164 us; the 32-output instances are faster as they are)
template <int NT, int KT, bool BNA = false>
__global__ __launch_bounds__(PW_WAVES * 64) __attribute__((amdgpu_waves_per_eu(NT == 4 ? 2 : 1)))
void pw_partial(const float* __restrict__ x, long long ld,
                                                             const float* __restrict__ gy, long long m, int n_total,
                                                             int k_total, long long rows_per_wave,
                                                             float* __restrict__ part, BnAct bna) {
  constexpr int N = 16 * NT, KS = 16 * KT, PW_DEPTH = pw_depth<NT>();
  __shared__ float red[N * KS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, i = lane & 15, g = lane >> 4;
  const int kslabs = k_total / KS;
  const int col0 = (blockIdx.y % kslabs) * KS, n0 = (blockIdx.y / kslabs) * N;  // this workgroup's slab
  pw4 acc[NT][KT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) acc[nt][kt] = pw4{0.0f, 0.0f, 0.0f, 0.0f};
  // BNA: this lane's KT columns col0 + KT i .. + KT - 1 are channels (col0 + KT i) % c .. + KT - 1 (KT % 4 == 0,
  // c a multiple of KT)
  BnAct4 bp[BNA ? KT / 4 : 1];
  if constexpr (BNA) {
#pragma unroll
    for (int u = 0; u < KT / 4; ++u) bp[u] = bnact_params(bna, (col0 + KT * i + 4 * u) % bna.c);
  }
  const long long r0 = ((long long)blockIdx.x * PW_WAVES + w) * rows_per_wave;
  const long long r1 = r0 + rows_per_wave < m ? r0 + rows_per_wave : m;
  auto load_row = [&](long long r, float (&a)[NT], float (&b)[KT]) {
    const float* yr = gy + r * n_total + n0 + NT * i;
    if constexpr (NT == 4) {
      const pw4u v = *reinterpret_cast<const pw4u*>(yr);
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    } else {
      const pw2u v = *reinterpret_cast<const pw2u*>(yr);
      a[0] = v.x; a[1] = v.y;
    }
    const float* xr = x + r * ld + col0 + KT * i;
#pragma unroll
    for (int kt = 0; kt + 4 <= KT; kt += 4) {
      const pw4u v = *reinterpret_cast<const pw4u*>(xr + kt);  // (4-byte aligned: still one dwordx4 load)
      b[kt] = v.x; b[kt + 1] = v.y; b[kt + 2] = v.z; b[kt + 3] = v.w;
    }
#pragma unroll
    for (int kt = KT / 4 * 4; kt < KT; ++kt) b[kt] = xr[kt];
  };
  auto load = [&](long long q, float (&a)[PW_DEPTH][NT], float (&b)[PW_DEPTH][KT]) {
#pragma unroll
    for (int d = 0; d < PW_DEPTH; ++d) load_row(q + 4 * d + g, a[d], b[d]);
  };
  // (BNA: the BatchNorm + activation is applied to a set when it is consumed, after the next set's loads were issued)
  auto mma = [&](const float (&a)[PW_DEPTH][NT], float (&b)[PW_DEPTH][KT]) {
    if constexpr (BNA) {
#pragma unroll
      for (int d = 0; d < PW_DEPTH; ++d)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          const BnAct4& q = bp[kt / 4];
          const int e = kt % 4;
          b[d][kt] = bnact_apply(b[d][kt], q.mu[e], q.is[e], q.w[e], q.b[e], bna.act, bna.slope);
        }
    }
#pragma unroll
    for (int d = 0; d < PW_DEPTH; ++d)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
          acc[nt][kt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[d][nt], b[d][kt], acc[nt][kt], 0, 0, 0);
  };
  // two register sets of PW_DEPTH row quads: the next set's loads are in flight under this set's MFMAs (full sets
  // only; the run's last, partial set is loaded with its dead rows' gy zeroed)
  constexpr int STEP = 4 * PW_DEPTH;
  const long long full = r0 + (r1 > r0 ? (r1 - r0) / STEP * STEP : 0);  // end of the full sets
  float a0[PW_DEPTH][NT], b0[PW_DEPTH][KT], a1[PW_DEPTH][NT], b1[PW_DEPTH][KT];
  long long q = r0;
  if (q < full) load(q, a0, b0);
  while (q < full) {
    const bool more = q + STEP < full;
    if (more) load(q + STEP, a1, b1);
    __builtin_amdgcn_sched_barrier(0);  // (the next set's loads stay ahead of these MFMAs)
    mma(a0, b0);
    q += STEP;
    if (!more) break;
    const bool more2 = q + STEP < full;
    if (more2) load(q + STEP, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    q += STEP;
    if (!more2) break;
  }
  if (full < r1) {  // the partial set: rows past r1 read row r0 (in bounds) against a zero gy
#pragma unroll
    for (int d = 0; d < PW_DEPTH; ++d) {
      const long long r = full + 4 * d + g;
      const bool live = r < r1;
      load_row(live ? r : r0, a0[d], b0[d]);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) a0[d][nt] = live ? a0[d][nt] : 0.0f;
    }
    mma(a0, b0);
  }
  // lane (n = i, g) holds, for tile (nt, kt), output row NT (4 g + v) + nt (the A row 4 g + v) and slab column
  // KT i + kt
  for (int ww = 0; ww < PW_WAVES; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            float* dst = red + (NT * (4 * g + v) + nt) * KS + KT * i + kt;
            *dst = ww == 0 ? acc[nt][kt][v] : *dst + acc[nt][kt][v];
          }
    }
    __syncthreads();
  }
  // this workgroup's row of partials [n_total][k_total], its slab
  float* prow = part + ((size_t)blockIdx.x * n_total + n0) * k_total + col0;
  for (int e = threadIdx.x; e < N * KS; e += PW_WAVES * 64) prow[(size_t)(e / KS) * k_total + e % KS] = red[e];
}

// the column slab width for (n, k): conv2's single 144-column slab, else 128-column slabs, with n in one 32-row slab
// or 64-row slabs (0: not covered)
static int pw_slab(int n, int k) {
  if (n == 32 && (k == 144 || k == 128)) return k;
  if (n % 64 == 0 && n <= 256 && k % 128 == 0 && k <= 4096) return 128;
  return 0;
}

int patch_wgrad_blocks(long long m, int n, int k) {
  const int slab = pw_slab(n, k);
  if (!slab) return 0;
  const long long slabs = (long long)(k / slab) * (n == 32 ? 1 : n / 64);
  // about 512 workgroups over rows x slabs, 1 024 rows per wave at most (64 at least)
  long long rpb = (m * slabs + 511) / 512;
  rpb = rpb < 256 ? 256 : (rpb > 4096 ? 4096 : rpb);
  const long long b = (m + rpb - 1) / rpb;
  return (int)(b < 1 ? 1 : (b > 512 ? 512 : b));
}

hipError_t launch_patch_wgrad(const float* x, long long ld, const float* gy, long long m, int n, int k, float* part,
                              float* gw, const BnAct* bna, hipStream_t s) {
  const int slab = pw_slab(n, k);
  const int blocks = patch_wgrad_blocks(m, n, k);
  if (!slab || !blocks) return hipErrorInvalidValue;
  const BnAct none{};
  long long rpw = (m + (long long)blocks * PW_WAVES - 1) / ((long long)blocks * PW_WAVES);
  rpw = (rpw + 3) & ~3LL;
  const dim3 grid(blocks, (k / slab) * (n == 32 ? 1 : n / 64)), wg(PW_WAVES * 64);
  if (bna) {  // (covered: n 64 in 128-column slabs, c dividing 8 consecutive columns' channel run: c % 8 == 0)
    if (n % 64 || bna->c % 8) return hipErrorInvalidValue;
    hipLaunchKernelGGL((pw_partial<4, 8, true>), grid, wg, 0, s, x, ld, gy, m, n, k, rpw, part, *bna);
  } else if (n == 32 && k == 144)
    hipLaunchKernelGGL((pw_partial<2, 9>), grid, wg, 0, s, x, ld, gy, m, n, k, rpw, part, none);
  else if (n == 32)
    hipLaunchKernelGGL((pw_partial<2, 8>), grid, wg, 0, s, x, ld, gy, m, n, k, rpw, part, none);
  else
    hipLaunchKernelGGL((pw_partial<4, 8>), grid, wg, 0, s, x, ld, gy, m, n, k, rpw, part, none);
  hipLaunchKernelGGL(colsum_final, dim3((n * k + 63) / 64), dim3(CF_WAVES * 64), 0, s, part, blocks, n * k, gw);
  return hipGetLastError();
}

// ------------------------------------------------------------------- tall-skinny patch GEMM, forward / dgrad
// C[M][N] = A[M][K] B[K][N] for tall A and a small B: the vision stem's conv3 forward (A = its 2 x 2 patches [M][128],
// B = W3^T, N 64), its input gradient (A = gz3 [M][64], B = W3, N 128) and the final Linear's input gradient (A = gy
// [M][192], B = W [192][1280], in 64-output slabs, blockIdx.y), where hipBLASLt ran at 0.8-2.4 TB/s.  The workgroup stages B once in LDS, transposed (Bt[n][k], rows padded by 4 floats);
// the k order is permuted so that both operands are read four steps at a time: k(s, g) = 16 (s / 4) + 4 g + s % 4,
// lane (i = l % 16, g = l / 16) taking A[row i][16 q + 4 g .. + 3] (a float4 from global) and Bt[16 nt + i][16 q +
// 4 g .. + 3] (a 16-byte LDS read) for the four steps of quad q.  A wave walks 16-row tiles strided by the grid, the
// next tile's A loaded under the current tile's MFMAs; lane (n, g) stores C[4 g + v][16 nt + n].  Each output is one
// fixed-order fp32 MFMA chain over k: deterministic.  (Same-box A/B, r5ts2, 24 576 images: forward 124 -> 92 us,
// input gradient 125 -> 109 us against B held in registers, 128 of them, two waves per SIMD; 172 / 157 us hipBLASLt.)
typedef float ts4u __attribute__((ext_vector_type(4), aligned(4)));
constexpr int TS_WAVES = 4;

template <int K, int N, bool B_NK, bool BNA = false>
__global__ __launch_bounds__(TS_WAVES * 64) void tsgemm_kernel(const float* __restrict__ a, long long lda,
                                                               const float* __restrict__ bm, int n_total,
                                                               float* __restrict__ c, long long ldc, long long m,
                                                               BnAct bna) {
  // N: this workgroup's slab of the n_total outputs (blockIdx.y)
  constexpr int S = K / 4, NT = N / 16, Q = K / 16, LDK = K + 4;
  __shared__ float bt[N * LDK];
  const int n0 = blockIdx.y * N;
  for (int e = threadIdx.x; e < N * K; e += TS_WAVES * 64) {
    const int n = e / K, k = e % K;
    // B_NK: bm is W [n_total][K] (B = W^T), else B [K][n_total]
    bt[n * LDK + k] = B_NK ? bm[(size_t)(n0 + n) * K + k] : bm[(size_t)k * n_total + n0 + n];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  // BNA (c = 32 channels: the pattern repeats every two quads): quad q's four columns 16 q + 4 g .. + 3 are channels
  // 16 (q % 2) + 4 g .. + 3
  BnAct4 bp[BNA ? 2 : 1];
  if constexpr (BNA) {
#pragma unroll
    for (int u = 0; u < 2; ++u) bp[u] = bnact_params(bna, 16 * u + 4 * g);
  }
  const long long tiles = (m + 15) / 16;
  const long long wave = (long long)blockIdx.x * TS_WAVES + (threadIdx.x >> 6);
  const long long stride = (long long)gridDim.x * TS_WAVES;
  auto load = [&](long long t, float (&av)[S]) {
    long long r = 16 * t + i;
    r = r < m ? r : m - 1;  // (rows past the end read the last row; their outputs are not stored)
    const float* ar = a + r * lda + 4 * g;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const ts4u v = *reinterpret_cast<const ts4u*>(ar + 16 * q);
      av[4 * q] = v.x; av[4 * q + 1] = v.y; av[4 * q + 2] = v.z; av[4 * q + 3] = v.w;
    }
  };
  // (BNA: the BatchNorm + activation is applied when the tile is consumed, a tile after its loads were issued, so the
  // loads' latency stays hidden under the previous tile's MFMAs)
  auto tile = [&](long long t, float (&av)[S]) {
    if constexpr (BNA) {
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          av[4 * q + e] = bnact_apply(av[4 * q + e], bp[q % 2].mu[e], bp[q % 2].is[e], bp[q % 2].w[e], bp[q % 2].b[e],
                                      bna.act, bna.slope);
    }
    pw4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = pw4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      pw4 bq[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bq[nt] = *reinterpret_cast<const pw4*>(bt + (16 * nt + i) * LDK + 16 * q + 4 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[4 * q + e], bq[nt][e], acc[nt], 0, 0, 0);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const long long r = 16 * t + 4 * g + v;
      if (r < m) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) c[r * ldc + n0 + 16 * nt + i] = acc[nt][v];
      }
    }
  };
  // two register sets, the next tile's loads issued ahead of this tile's MFMAs (no copies between the sets)
  float a0[S], a1[S];
  long long t = wave;
  if (t < tiles) load(t, a0);
  while (t < tiles) {
    const long long t1 = t + stride;
    if (t1 < tiles) load(t1, a1);
    __builtin_amdgcn_sched_barrier(0);
    tile(t, a0);
    if (t1 >= tiles) break;
    const long long t2 = t1 + stride;
    if (t2 < tiles) load(t2, a0);
    __builtin_amdgcn_sched_barrier(0);
    tile(t1, a1);
    t = t2;
  }
}

bool tsgemm_covered(int k, int n, bool b_nk) {
  return (k == 128 && n == 64 && b_nk) || (k == 64 && n == 128 && !b_nk) ||
         (k == 192 && !b_nk && n % 64 == 0 && n <= 4096);  // (the last in 64-output slabs: the final Linear's dgrad)
}

hipError_t launch_tsgemm(const float* a, long long lda, const float* bm, bool b_nk, float* c, long long ldc,
                         long long m, int k, int n, const BnAct* bna, hipStream_t s) {
  if (!tsgemm_covered(k, n, b_nk)) return hipErrorInvalidValue;
  const BnAct none{};
  const long long tiles = (m + 15) / 16;
  long long blocks = (tiles + TS_WAVES - 1) / TS_WAVES;
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);  // 256 CUs x 4 workgroups, walked in strides
  const dim3 wg(TS_WAVES * 64);
  if (bna) {  // (covered: conv3's forward from block 2's BatchNorm input, c dividing 4-column runs)
    if (k != 128 || bna->c != 32) return hipErrorInvalidValue;
    hipLaunchKernelGGL((tsgemm_kernel<128, 64, true, true>), dim3(blocks), wg, 0, s, a, lda, bm, n, c, ldc, m, *bna);
  } else if (k == 128)
    hipLaunchKernelGGL((tsgemm_kernel<128, 64, true>), dim3(blocks), wg, 0, s, a, lda, bm, n, c, ldc, m, none);
  else if (k == 64)
    hipLaunchKernelGGL((tsgemm_kernel<64, 128, false>), dim3(blocks), wg, 0, s, a, lda, bm, n, c, ldc, m, none);
  else {  // 64-output slabs: about 1 024 workgroups over rows x slabs
    const long long slabs = n / 64;
    long long rb = (1024 + slabs - 1) / slabs;
    rb = rb < blocks ? rb : blocks;
    hipLaunchKernelGGL((tsgemm_kernel<192, 64, false>), dim3(rb, slabs), wg, 0, s, a, lda, bm, n, c, ldc, m, none);
  }
  return hipGetLastError();
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
// The actor / critic MLP's memory-bound layers for the PPO update's tall mini-batches (rsl_rl/linear.py MLP):
// the MLP is x -> L1 -> lrelu -> L2 -> lrelu -> L3 with L1: d -> h1 (d <= 32), L2: h1 -> h2 (the 256 x 256 GEMM, on
// hipBLASLt), L3: h2 -> k (k <= 8).  Everything around the big GEMM runs here, each matrix read once:
//   in_forward  : h1 = lrelu(x W1^T + b1)                          (K = d GEMM + bias + activation, writes h1)
//   in_backward : gz1 = gh1 * lrelu'(h1); gW1 = gz1^T x, gb1 = sum gz1   (reads gh1, h1, x; gz1 never stored)
//   head_forward: y = lrelu(z2) W3^T + b3                          (reads z2; no activation pass, no GEMM)
//   head_backward: gz2 = (gy W3) * lrelu'(z2); gW3 = gy^T lrelu(z2), gb3 = sum gy, gb2 = sum gz2
// (lrelu'(h) = lrelu'(z): a LeakyReLU keeps the sign, and maps 0 to 0.)  A wave owns a row at a time, lane l
// columns 4 l .. 4 l + 3 (one 1 KB coalesced access per row of 256); four rows' loads are issued together.  Dot
// products are fmaf chains (these ops are held to float64 at 1e-6 of scale, not to bits; with separate multiply and
// add the first layer's 16-term dots were VALU-bound).  Weight /
// bias gradients: every wave writes its partial sums as one row of `part`, and partials_final adds the rows in a
// fixed order (deterministic, graph-capturable, no atomics).
#ifndef GR_HD_WAVES
#define GR_HD_WAVES 4
#endif
#ifndef GR_HD_U
#define GR_HD_U 4
#endif
#ifndef GR_HD_RPW
#define GR_HD_RPW 256  // head_backward rows per wave (128: +7 % at 393 216 rows, scripts/time_update_kernels.py)
#endif
#ifndef GR_IN_RPW
#define GR_IN_RPW 128  // in_backward rows per wave (256: +13 %)
#endif
constexpr int HD_WAVES = GR_HD_WAVES;  // waves per workgroup
constexpr int HD_U = GR_HD_U;          // rows in flight per wave
typedef float hd_v4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float hd_act(float z, float slope) { return z > 0.0f ? z : z * slope; }
__device__ __forceinline__ float hd_der(float z, float slope) { return z > 0.0f ? 1.0f : slope; }
#ifndef GR_HD_NT_LOAD
#define GR_HD_NT_LOAD 1  // non-temporal loads of the once-read [rows, h] matrices
#endif
#ifndef GR_HD_NT_STORE
#define GR_HD_NT_STORE 1  // non-temporal stores of the [rows, h] outputs (h1, gz2)
#endif
__device__ __forceinline__ void hd_st(float* p, const hd_v4& v) {
#if GR_HD_NT_STORE
  __builtin_nontemporal_store(v, reinterpret_cast<hd_v4*>(p));
#else
  *reinterpret_cast<hd_v4*>(p) = v;
#endif
}
__device__ __forceinline__ hd_v4 hd_ld(const float* p) {
#if GR_HD_NT_LOAD
  return __builtin_nontemporal_load(reinterpret_cast<const hd_v4*>(p));
#else
  return *reinterpret_cast<const hd_v4*>(p);
#endif
}

// rows per wave for the backward kernels: enough waves to fill the chip, few enough partial rows.  256 rows per
// wave, at most 4096 waves (partial rows); a batch that gives fewer than 1024 waves that way (e.g. 24 576 rows, config
// C2's mini-batch: 96 waves, each a serial 256-row chain of ~100 us) is spread over up to 1024 waves of >= 16 rows
#ifndef GR_IN_SMALL_WAVES
#define GR_IN_SMALL_WAVES 1024  // in_backward: waves for batches below target x that (its partial rows are 17 KB each)
#endif
__host__ __device__ inline long long hd_rows_per_wave(long long m, long long target = GR_HD_RPW, long long small = 1024) {
  long long w = (m + target - 1) / target;
  if (w < small) {
    const long long w16 = (m + 15) / 16;
    w = w16 < small ? w16 : small;
  }
  w = w < 1 ? 1 : (w > 4096 ? 4096 : w);
  return (m + w - 1) / w;
}
int head_partial_rows(long long m) {
  const long long rpw = hd_rows_per_wave(m);
  return (int)((m + rpw - 1) / rpw);
}
int in_partial_rows(long long m) {
  const long long rpw = hd_rows_per_wave(m, GR_IN_RPW, GR_IN_SMALL_WAVES);
  return (int)((m + rpw - 1) / rpw);
}

// ---- forward of the head: a wave takes 4 rows at a time, 16 lanes per row; lane q of a row holds columns
// 4 q + 64 j (j < 4), so each load instruction reads 256 contiguous bytes of every row and a row's dot products
// reduce over 16 lanes
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
        if (c < h) zz = hd_ld(z + r * h + c);
        const float a[4] = {hd_act(zz.x, slope), hd_act(zz.y, slope), hd_act(zz.z, slope), hd_act(zz.w, slope)};
#pragma unroll
        for (int k = 0; k < K; ++k) {
          float t = __builtin_fmaf(a[0], wr[k][4 * j], acc[k]);
          t = __builtin_fmaf(a[1], wr[k][4 * j + 1], t);
          t = __builtin_fmaf(a[2], wr[k][4 * j + 2], t);
          acc[k] = __builtin_fmaf(a[3], wr[k][4 * j + 3], t);
        }
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

// ---- backward of the head; partial row of a wave: [gW3 (k h) | gb3 (k) | gb2 = column sums of gz2 (h)]
template <int K>
__global__ __launch_bounds__(HD_WAVES * 64) void head_backward(const float* __restrict__ z,
                                                               const float* __restrict__ gy, long long m, int h,
                                                               const float* __restrict__ w, float slope, long long rpw,
                                                               float* __restrict__ gz, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  // (wave-uniform, so the per-row gy / x reads are scalar loads into SGPRs)
  const long long wid = (long long)blockIdx.x * HD_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long r0 = wid * rpw;
  if (r0 >= m) return;
  const long long r1 = r0 + rpw < m ? r0 + rpw : m;
  const int c = 4 * lane;
  const bool on = c < h;
  float wr[K][4];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) wr[k][j] = on ? w[(size_t)k * h + c + j] : 0.0f;
  float gw[K][4], gb[K], gs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    gb[k] = 0.0f;
#pragma unroll
    for (int j = 0; j < 4; ++j) gw[k][j] = 0.0f;
  }
  for (long long rb = r0; rb < r1; rb += HD_U) {
    float g[HD_U][K];
    hd_v4 zz[HD_U];
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const long long r = rb + u;
      const bool ok = r < r1;
#pragma unroll
      for (int k = 0; k < K; ++k) g[u][k] = ok ? gy[r * K + k] : 0.0f;
      zz[u] = hd_v4{0.0f, 0.0f, 0.0f, 0.0f};
      if (on && ok) zz[u] = hd_ld(z + r * h + c);
    }
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const long long r = rb + u;
      const float zv[4] = {zz[u].x, zz[u].y, zz[u].z, zz[u].w};
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float gh = g[u][0] * wr[0][j];
#pragma unroll
        for (int k = 1; k < K; ++k) gh = __builtin_fmaf(g[u][k], wr[k][j], gh);
        o[j] = gh * hd_der(zv[j], slope);
        gs[j] += o[j];
        const float a = hd_act(zv[j], slope);
#pragma unroll
        for (int k = 0; k < K; ++k) gw[k][j] = __builtin_fmaf(g[u][k], a, gw[k][j]);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) gb[k] += g[u][k];
      if (on && r < r1) {
        hd_st(gz + r * h + c, hd_v4{o[0], o[1], o[2], o[3]});
      }
    }
  }
  float* pr = part + (size_t)wid * ((K * h + K + h + 3) & ~3);  // (rows padded to 16 B: float4 stores)
  if (on) {
#pragma unroll
    for (int k = 0; k < K; ++k) *reinterpret_cast<hd_v4*>(pr + k * h + c) = hd_v4{gw[k][0], gw[k][1], gw[k][2], gw[k][3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) pr[K * h + K + c + j] = gs[j];
  }
  if (lane < K) {
    float v = gb[0];
#pragma unroll
    for (int k = 1; k < K; ++k) v = lane == k ? gb[k] : v;
    pr[K * h + lane] = v;
  }
}

// ---- first layer forward: h1 = lrelu(x W1^T + b1); lane l computes columns 4 l .. 4 l + 3 of each row
template <int D>
__global__ __launch_bounds__(HD_WAVES * 64) void in_forward(const float* __restrict__ x, long long m, int ldx,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            int h, float slope, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int c = 4 * lane;
  const bool on = c < h;
  float wr[4][D], br[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    br[j] = on ? b[c + j] : 0.0f;
#pragma unroll
    for (int k = 0; k < D; ++k) wr[j][k] = on ? w[(size_t)(c + j) * D + k] : 0.0f;
  }
  const long long stride = (long long)gridDim.x * HD_WAVES * HD_U;
  for (long long rb = ((long long)blockIdx.x * HD_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * HD_U;
       rb < m; rb += stride) {
    float xr[HD_U][D];
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const long long r = rb + u < m ? rb + u : m - 1;
#pragma unroll
      for (int k = 0; k < D; k += 4) {
        const hd_v4 v = *reinterpret_cast<const hd_v4*>(x + r * ldx + k);
        xr[u][k] = v.x; xr[u][k + 1] = v.y; xr[u][k + 2] = v.z; xr[u][k + 3] = v.w;
      }
    }
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const long long r = rb + u;
      float o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float acc = xr[u][0] * wr[j][0];
#pragma unroll
        for (int k = 1; k < D; ++k) acc = __builtin_fmaf(xr[u][k], wr[j][k], acc);
        o[j] = hd_act(acc + br[j], slope);
      }
      if (on && r < m) {
        hd_st(y + r * h + c, hd_v4{o[0], o[1], o[2], o[3]});
      }
    }
  }
}

// ---- the same on MFMA for d = 16, h a multiple of 16 (the actor / critic's 16 observations): a wave takes 16 rows at a
// time and computes y^T = W1 x^T + b1 per 16-unit tile with four v_mfma_f32_16x16x4f32 (lane (g, j): W1 row 16 t + j
// and x row j, elements 4 g .. 4 g + 3, so k step s contracts elements 4 g + s; its accumulator holds units
// 16 t + 4 g .. + 3 of row j: one 16-byte store).  The VALU form is VALU-bound (256 x 16 MACs per row on 64 lanes);
// this one moves only its bytes.  Summation order differs from the VALU form (both are held to float64).
typedef float hd_f4 __attribute__((ext_vector_type(4)));
template <int NT>
__global__ __launch_bounds__(HD_WAVES * 64) void in_forward_mfma(const float* __restrict__ x, long long m, int ldx,
                                                                 const float* __restrict__ w,
                                                                 const float* __restrict__ b, float slope,
                                                                 float* __restrict__ y) {
  constexpr int H = 16 * NT;
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  hd_f4 wr[NT], br[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    wr[t] = *reinterpret_cast<const hd_f4*>(w + (size_t)(16 * t + j) * 16 + 4 * g);
    br[t] = *reinterpret_cast<const hd_f4*>(b + 16 * t + 4 * g);
  }
  const long long tiles = (m + 15) / 16;
  for (long long tile = (long long)blockIdx.x * HD_WAVES + (threadIdx.x >> 6); tile < tiles;
       tile += (long long)gridDim.x * HD_WAVES) {
    const long long row = tile * 16 + j;
    const long long rr = row < m ? row : m - 1;
    const hd_f4 xv = *reinterpret_cast<const hd_f4*>(x + rr * ldx + 4 * g);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      hd_f4 acc = br[t];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[t][k], xv[k], acc, 0, 0, 0);
      if (row < m)
        hd_st(y + row * H + 16 * t + 4 * g,
              hd_v4{hd_act(acc[0], slope), hd_act(acc[1], slope), hd_act(acc[2], slope), hd_act(acc[3], slope)});
    }
  }
}

// ---- first layer backward; partial row of a wave: [gW1 (h d, row-major [h][d]) | gb1 (h)]
template <int D>
__global__ __launch_bounds__(HD_WAVES * 64) void in_backward(const float* __restrict__ gh, const float* __restrict__ hv,
                                                             const float* __restrict__ x, long long m, int ldx, int h,
                                                             float slope, long long rpw, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  // (wave-uniform, so the per-row gy / x reads are scalar loads into SGPRs)
  const long long wid = (long long)blockIdx.x * HD_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long r0 = wid * rpw;
  if (r0 >= m) return;
  const long long r1 = r0 + rpw < m ? r0 + rpw : m;
  const int c = 4 * lane;
  const bool on = c < h;
  float gw[4][D], gb[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < D; ++k) gw[j][k] = 0.0f;
  for (long long rb = r0; rb < r1; rb += HD_U) {
    hd_v4 gg[HD_U], hh[HD_U];
    float xr[HD_U][D];
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const long long r = rb + u;
      const bool ok = r < r1;
      const long long rr = ok ? r : r0;
      gg[u] = hd_v4{0.0f, 0.0f, 0.0f, 0.0f};
      hh[u] = hd_v4{0.0f, 0.0f, 0.0f, 0.0f};
      if (on && ok) {
        gg[u] = hd_ld(gh + r * h + c);
        hh[u] = hd_ld(hv + r * h + c);
      }
#pragma unroll
      for (int k = 0; k < D; k += 4) {
        const hd_v4 v = *reinterpret_cast<const hd_v4*>(x + rr * ldx + k);
        xr[u][k] = ok ? v.x : 0.0f; xr[u][k + 1] = ok ? v.y : 0.0f;
        xr[u][k + 2] = ok ? v.z : 0.0f; xr[u][k + 3] = ok ? v.w : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < HD_U; ++u) {
      const float gz[4] = {gg[u].x * hd_der(hh[u].x, slope), gg[u].y * hd_der(hh[u].y, slope),
                           gg[u].z * hd_der(hh[u].z, slope), gg[u].w * hd_der(hh[u].w, slope)};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        gb[j] += gz[j];
#pragma unroll
        for (int k = 0; k < D; ++k) gw[j][k] = __builtin_fmaf(gz[j], xr[u][k], gw[j][k]);
      }
    }
  }
  float* pr = part + (size_t)wid * (h * D + h);
  if (on) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int k = 0; k < D; k += 4)
        *reinterpret_cast<hd_v4*>(pr + (size_t)(c + j) * D + k) = hd_v4{gw[j][k], gw[j][k + 1], gw[j][k + 2], gw[j][k + 3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) pr[h * D + c + j] = gb[j];
  }
}

// out[n] = sum over the `rows` partial rows [rows][n], in row order per 16-wave slice: 64 outputs per workgroup,
// its 16 waves take every 16th partial row (four loads in flight per lane), combined in LDS in wave order
__device__ __forceinline__ void partials_final_body(const float* __restrict__ part, int rows, int n, int ld,
                                                    float* __restrict__ out) {
  __shared__ float sm[CF_WAVES * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
  if (i < n) {
    int b = wv;
    for (; b + 3 * CF_WAVES < rows; b += 4 * CF_WAVES) {
      a0 += part[(size_t)b * ld + i];
      a1 += part[(size_t)(b + CF_WAVES) * ld + i];
      a2 += part[(size_t)(b + 2 * CF_WAVES) * ld + i];
      a3 += part[(size_t)(b + 3 * CF_WAVES) * ld + i];
    }
    for (; b < rows; b += CF_WAVES) a0 += part[(size_t)b * ld + i];
  }
  sm[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wv == 0 && i < n) {
    float s = 0.0f;
    for (int k = 0; k < CF_WAVES; ++k) s += sm[k * 64 + lane];
    out[i] = s;
  }
}

__global__ __launch_bounds__(CF_WAVES * 64) void partials_final(const float* __restrict__ part, int rows, int n,
                                                                int ld, float* __restrict__ out) {
  partials_final_body(part, rows, n, ld, out);
}

#define HD_DISPATCH_K(KK, F)          \
  switch (KK) {                       \
    case 1: F(1); break;              \
    case 2: F(2); break;              \
    case 3: F(3); break;              \
    case 4: F(4); break;              \
    case 5: F(5); break;              \
    case 6: F(6); break;              \
    case 7: F(7); break;              \
    default: F(8); break;             \
  }
#define HD_DISPATCH_D(DD, F)          \
  switch (DD) {                       \
    case 4: F(4); break;              \
    case 8: F(8); break;              \
    case 12: F(12); break;            \
    case 16: F(16); break;            \
    case 20: F(20); break;            \
    case 24: F(24); break;            \
    case 28: F(28); break;            \
    default: F(32); break;            \
  }

static int hd_grid(long long waves) {
  const long long b = (waves + HD_WAVES - 1) / HD_WAVES;
  return (int)(b < 1 ? 1 : b);
}

hipError_t launch_head_forward(const float* z, long long m, int h, const float* w, const float* b, int k, float slope,
                               float* y, hipStream_t s) {
  const long long fb = (m + 127) / 128;  // ~8 row groups of 4 per wave: enough loads in flight
  const int blocks = (int)(fb < 1 ? 1 : (fb > 8192 ? 8192 : fb));
#define HD_FWD(KK) \
  hipLaunchKernelGGL(head_forward<KK>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, z, m, h, w, b, slope, y)
  HD_DISPATCH_K(k, HD_FWD)
#undef HD_FWD
  return hipGetLastError();
}

hipError_t launch_head_backward(const float* z, const float* gy, long long m, int h, const float* w, int k,
                                float slope, float* gz, float* part, float* sums, hipStream_t s) {
  const long long rpw = hd_rows_per_wave(m);
  const int prow = head_partial_rows(m);
  const int blocks = hd_grid(prow);
#define HD_BWD(KK) \
  hipLaunchKernelGGL(head_backward<KK>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, z, gy, m, h, w, slope, rpw, gz, part)
  HD_DISPATCH_K(k, HD_BWD)
#undef HD_BWD
  const int n = k * h + k + h;
  hipLaunchKernelGGL(partials_final, dim3((n + 63) / 64), dim3(CF_WAVES * 64), 0, s, part, prow, n, (n + 3) & ~3, sums);
  return hipGetLastError();
}

hipError_t launch_in_forward(const float* x, long long m, int d, int ldx, const float* w, const float* b, int h,
                             float slope, float* y, hipStream_t s) {
  if (d == 16 && (h == 256 || h == 128) && ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(b)) & 15) == 0) {
    const long long tiles = (m + 15) / 16;
    const long long fb = (tiles + 4 * HD_WAVES - 1) / (4 * HD_WAVES);  // ~4 row tiles per wave
    const int blocks = (int)(fb < 1 ? 1 : (fb > 8192 ? 8192 : fb));
    if (h == 256)
      hipLaunchKernelGGL(in_forward_mfma<16>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, x, m, ldx, w, b, slope, y);
    else
      hipLaunchKernelGGL(in_forward_mfma<8>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, x, m, ldx, w, b, slope, y);
    return hipGetLastError();
  }
  const long long fb = (m + 8 * HD_WAVES * HD_U - 1) / (8 * HD_WAVES * HD_U);  // ~8 row groups per wave
  const int blocks = (int)(fb < 1 ? 1 : (fb > 8192 ? 8192 : fb));
#define IN_FWD(DD) \
  hipLaunchKernelGGL(in_forward<DD>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, x, m, ldx, w, b, h, slope, y)
  HD_DISPATCH_D(d, IN_FWD)
#undef IN_FWD
  return hipGetLastError();
}

hipError_t launch_in_backward(const float* gh, const float* hv, const float* x, long long m, int d, int ldx, int h,
                              float slope, float* part, float* sums, hipStream_t s) {
  const long long rpw = hd_rows_per_wave(m, GR_IN_RPW, GR_IN_SMALL_WAVES);
  const int prow = in_partial_rows(m);
  const int blocks = hd_grid(prow);
#define IN_BWD(DD) \
  hipLaunchKernelGGL(in_backward<DD>, dim3(blocks), dim3(HD_WAVES * 64), 0, s, gh, hv, x, m, ldx, h, slope, rpw, part)
  HD_DISPATCH_D(d, IN_BWD)
#undef IN_BWD
  const int n = h * d + h;
  hipLaunchKernelGGL(partials_final, dim3((n + 63) / 64), dim3(CF_WAVES * 64), 0, s, part, prow, n, n, sums);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// The PPO losses of a mini-batch (standalone/rsl_rl/ext/algorithms/ppo.py:152-169 with the adaptive-rate KL of
// :133-150 and the Gaussian log prob of rsl_rl's ActorCritic), forward and backward, one thread per sample: ~50
// tiny torch launches of [rows] / [rows, 4] tensors each way become one launch + one fixed-order reduction.
// Forward sums [surrogate terms, value terms, KL terms]; backward d/dmu, d/dvalue per row and d/dstd (summed).
// Semantics of the torch ops it replaces: Normal.log_prob = -(a - mu)^2 / (2 sigma^2) - log sigma - log sqrt(2 pi);
// torch.max of two tensors splits the gradient in half on ties; clamp passes it on [lo, hi] inclusive.
constexpr float LOG_SQRT_2PI = 0.918938533204672741780f;

// torch.clamp / torch.max keep a NaN operand (fminf / fmaxf would drop it)
__device__ __forceinline__ float clamp_keep_nan(float x, float lo, float hi) {
  return x != x ? x : fminf(fmaxf(x, lo), hi);
}
__device__ __forceinline__ float max_keep_nan(float a, float b) { return (a != a || b != b) ? a + b : fmaxf(a, b); }

struct LossRow {
  float logp, ratio, s1, s2, v, vc, ret, vdiff;
};

__device__ __forceinline__ float pl_at(const float* p, long long ld, long long i, int j) { return p[i * ld + j]; }

__device__ __forceinline__ void pl_row(const gr_ppo_loss_args& a, long long i, const float* sd, LossRow& r,
                                       float* kl) {
  float lp = 0.0f, k = 0.0f;
  for (int j = 0; j < a.k; ++j) {
    const float mu = pl_at(a.mu, a.ld_mu, i, j), x = pl_at(a.act, a.ld_act, i, j);
    const float d = x - mu, var = sd[j] * sd[j];
    lp += (-(d * d) / (2.0f * var) - logf(sd[j])) - LOG_SQRT_2PI;
    if (kl) {
      const float so = pl_at(a.sig_old, a.ld_sig_old, i, j), mo = pl_at(a.mu_old, a.ld_mu_old, i, j);
      const float dm = mo - mu;
      k += (logf(sd[j] / so + 1.0e-5f) + (so * so + dm * dm) / (2.0f * (sd[j] * sd[j]))) - 0.5f;
    }
  }
  if (kl) *kl = k;
  r.logp = lp;
  r.ratio = expf(lp - a.logp_old[i * a.ld_logp_old]);
  const float A = a.adv[i * a.ld_adv];
  const float rc = clamp_keep_nan(r.ratio, 1.0f - a.clip, 1.0f + a.clip);
  r.s1 = -A * r.ratio;
  r.s2 = -A * rc;
  r.v = a.value[i * a.ld_value];
  r.ret = a.ret[i * a.ld_ret];
  const float vo = a.value_old[i * a.ld_value_old];
  r.vdiff = r.v - vo;
  r.vc = vo + clamp_keep_nan(r.vdiff, -a.clip, a.clip);
}

__device__ __forceinline__ float pl_wave_sum(float v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__global__ __launch_bounds__(256) void ppo_loss_forward(gr_ppo_loss_args a, float* __restrict__ part) {
  __shared__ float sm[4][3];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  float sd[8];
  for (int j = 0; j < a.k; ++j) sd[j] = a.std[j];
  float t[3] = {0.0f, 0.0f, 0.0f};
  if (i < a.rows) {
    LossRow r;
    float kl;
    pl_row(a, i, sd, r, &kl);
    t[0] = max_keep_nan(r.s1, r.s2);
    const float l1 = (r.v - r.ret) * (r.v - r.ret), l2 = (r.vc - r.ret) * (r.vc - r.ret);
    t[1] = a.clipped_value ? max_keep_nan(l1, l2) : (r.ret - r.v) * (r.ret - r.v);
    t[2] = kl;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float v = pl_wave_sum(t[q]);
    if (lane == 0) sm[wv][q] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) part[(size_t)blockIdx.x * 4 + threadIdx.x] = ((sm[0][threadIdx.x] + sm[1][threadIdx.x]) + sm[2][threadIdx.x]) + sm[3][threadIdx.x];
}

// g[0], g[1]: the upstream gradients of the surrogate and value losses (device scalars; the means' 1 / rows is
// applied here)
// (gr_ppo_loss_backward_loss: g[0] is the upstream gradient of the combined loss surrogate + value_coef * value,
// gv_index 0 and gv_coef value_coef: torch's MulBackward gives the value mean g * value_coef)
__global__ __launch_bounds__(256) void ppo_loss_backward(gr_ppo_loss_args a, const float* __restrict__ g,
                                                         int gv_index, float gv_coef, float* __restrict__ dmu,
                                                         float* __restrict__ dvalue, float* __restrict__ part) {
  __shared__ float sm[4][8];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  float sd[8];
  for (int j = 0; j < a.k; ++j) sd[j] = a.std[j];
  float ds[8];
  for (int j = 0; j < 8; ++j) ds[j] = 0.0f;
  if (i < a.rows) {
    LossRow r;
    pl_row(a, i, sd, r, nullptr);
    const float inv_m = 1.0f / (float)a.rows;
    const float gs = g[0] * inv_m, gv = (gv_coef * g[gv_index]) * inv_m;
    const float A = a.adv[i * a.ld_adv];
    const float w1 = r.s1 > r.s2 ? 1.0f : (r.s1 == r.s2 ? 0.5f : 0.0f), w2 = 1.0f - w1;
    const float inclip = (r.ratio >= 1.0f - a.clip && r.ratio <= 1.0f + a.clip) ? 1.0f : 0.0f;
    const float dratio = gs * (w1 * -A + w2 * (-A * inclip));
    const float dlogp = dratio * r.ratio;
    for (int j = 0; j < a.k; ++j) {
      const float mu = pl_at(a.mu, a.ld_mu, i, j), x = pl_at(a.act, a.ld_act, i, j);
      const float d = x - mu, var = sd[j] * sd[j];
      dmu[i * a.k + j] = dlogp * (d / var);
      ds[j] = dlogp * (d * d / (var * sd[j]) - 1.0f / sd[j]);
    }
    float dv;
    if (a.clipped_value) {
      const float l1 = (r.v - r.ret) * (r.v - r.ret), l2 = (r.vc - r.ret) * (r.vc - r.ret);
      const float u1 = l1 > l2 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f), u2 = 1.0f - u1;
      const float vin = (r.vdiff >= -a.clip && r.vdiff <= a.clip) ? 1.0f : 0.0f;
      dv = gv * (u1 * 2.0f * (r.v - r.ret) + u2 * 2.0f * (r.vc - r.ret) * vin);
    } else {
      dv = gv * (2.0f * (r.v - r.ret));
    }
    dvalue[i] = dv;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int j = 0; j < a.k; ++j) {
    const float v = pl_wave_sum(ds[j]);
    if (lane == 0) sm[wv][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < a.k)
    part[(size_t)blockIdx.x * 8 + threadIdx.x] = ((sm[0][threadIdx.x] + sm[1][threadIdx.x]) + sm[2][threadIdx.x]) + sm[3][threadIdx.x];
}

int ppo_loss_blocks(long long rows) { return (int)((rows + 255) / 256); }

hipError_t launch_ppo_loss_forward(const gr_ppo_loss_args& a, float* part, float* sums, hipStream_t s) {
  const int blocks = ppo_loss_blocks(a.rows);
  hipLaunchKernelGGL(ppo_loss_forward, dim3(blocks), dim3(256), 0, s, a, part);
  hipLaunchKernelGGL(partials_final, dim3(1), dim3(CF_WAVES * 64), 0, s, part, blocks, 3, 4, sums);
  return hipGetLastError();
}

// the forward's sums in partials_final's order, then the means and the combined loss (torch: sums / rows, then
// surrogate + value_coef * value); acc[0..1] += (surrogate, value) and kl_out[0] = kl when given
__global__ __launch_bounds__(CF_WAVES * 64) void ppo_loss_final(const float* __restrict__ part, int rows,
                                                                float* __restrict__ sums, long long m, float value_coef,
                                                                float* __restrict__ loss, float* __restrict__ stats,
                                                                float* __restrict__ acc, float* __restrict__ kl_out) {
  partials_final_body(part, rows, 3, 4, sums);
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_block();
    const float inv_m = 1.0f / (float)m;  // (torch's tensor / CPU scalar multiplies by the reciprocal)
    const float surr = sums[0] * inv_m, val = sums[1] * inv_m, kl = sums[2] * inv_m;
    loss[0] = surr + value_coef * val;
    stats[0] = surr;
    stats[1] = val;
    stats[2] = kl;
    if (acc) {
      acc[0] = acc[0] + surr;
      acc[1] = acc[1] + val;
    }
    if (kl_out) kl_out[0] = kl;
  }
}

hipError_t launch_ppo_loss_forward_loss(const gr_ppo_loss_args& a, float* part, float* sums, float value_coef,
                                        float* loss, float* stats, float* acc, float* kl_out, hipStream_t s) {
  const int blocks = ppo_loss_blocks(a.rows);
  hipLaunchKernelGGL(ppo_loss_forward, dim3(blocks), dim3(256), 0, s, a, part);
  hipLaunchKernelGGL(ppo_loss_final, dim3(1), dim3(CF_WAVES * 64), 0, s, part, blocks, sums, (long long)a.rows,
                     value_coef, loss, stats, acc, kl_out);
  return hipGetLastError();
}

// gr_ppo_loss_forward_backward: ppo_loss_forward and ppo_loss_backward (combined-loss form) in one pass over the
// rows, for a caller that knows the upstream gradient's device address before the backward runs (the graph-captured
// step's persistent seed): the per-row gradients and the std gradient's partial rows come out of the forward pass,
// and one final launch reduces both the loss sums and the std gradient, in the orders of the two-pass form
// (bit-identical to gr_ppo_loss_forward_loss + gr_ppo_loss_backward_loss)
__global__ __launch_bounds__(256) void ppo_loss_fwd_bwd(gr_ppo_loss_args a, const float* __restrict__ g,
                                                        float value_coef, float* __restrict__ part,
                                                        float* __restrict__ dmu, float* __restrict__ dvalue,
                                                        float* __restrict__ dpart) {
  __shared__ float sm[4][3];
  __shared__ float smd[4][8];
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  float sd[8];
  for (int j = 0; j < a.k; ++j) sd[j] = a.std[j];
  float t[3] = {0.0f, 0.0f, 0.0f};
  float ds[8];
  for (int j = 0; j < 8; ++j) ds[j] = 0.0f;
  if (i < a.rows) {
    LossRow r;
    float kl;
    pl_row(a, i, sd, r, &kl);
    // forward (ppo_loss_forward)
    t[0] = max_keep_nan(r.s1, r.s2);
    const float l1 = (r.v - r.ret) * (r.v - r.ret), l2 = (r.vc - r.ret) * (r.vc - r.ret);
    t[1] = a.clipped_value ? max_keep_nan(l1, l2) : (r.ret - r.v) * (r.ret - r.v);
    t[2] = kl;
    // backward (ppo_loss_backward, gv_index 0, gv_coef value_coef)
    const float inv_m = 1.0f / (float)a.rows;
    const float gs = g[0] * inv_m, gv = (value_coef * g[0]) * inv_m;
    const float A = a.adv[i * a.ld_adv];
    const float w1 = r.s1 > r.s2 ? 1.0f : (r.s1 == r.s2 ? 0.5f : 0.0f), w2 = 1.0f - w1;
    const float inclip = (r.ratio >= 1.0f - a.clip && r.ratio <= 1.0f + a.clip) ? 1.0f : 0.0f;
    const float dratio = gs * (w1 * -A + w2 * (-A * inclip));
    const float dlogp = dratio * r.ratio;
    for (int j = 0; j < a.k; ++j) {
      const float mu = pl_at(a.mu, a.ld_mu, i, j), x = pl_at(a.act, a.ld_act, i, j);
      const float d = x - mu, var = sd[j] * sd[j];
      dmu[i * a.k + j] = dlogp * (d / var);
      ds[j] = dlogp * (d * d / (var * sd[j]) - 1.0f / sd[j]);
    }
    float dv;
    if (a.clipped_value) {
      const float u1 = l1 > l2 ? 1.0f : (l1 == l2 ? 0.5f : 0.0f), u2 = 1.0f - u1;
      const float vin = (r.vdiff >= -a.clip && r.vdiff <= a.clip) ? 1.0f : 0.0f;
      dv = gv * (u1 * 2.0f * (r.v - r.ret) + u2 * 2.0f * (r.vc - r.ret) * vin);
    } else {
      dv = gv * (2.0f * (r.v - r.ret));
    }
    dvalue[i] = dv;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float v = pl_wave_sum(t[q]);
    if (lane == 0) sm[wv][q] = v;
  }
  for (int j = 0; j < a.k; ++j) {
    const float v = pl_wave_sum(ds[j]);
    if (lane == 0) smd[wv][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) part[(size_t)blockIdx.x * 4 + threadIdx.x] = ((sm[0][threadIdx.x] + sm[1][threadIdx.x]) + sm[2][threadIdx.x]) + sm[3][threadIdx.x];
  if (threadIdx.x < a.k)
    dpart[(size_t)blockIdx.x * 8 + threadIdx.x] = ((smd[0][threadIdx.x] + smd[1][threadIdx.x]) + smd[2][threadIdx.x]) + smd[3][threadIdx.x];
}

__global__ __launch_bounds__(CF_WAVES * 64) void ppo_loss_final_fb(const float* __restrict__ part,
                                                                   const float* __restrict__ dpart, int rows, int k,
                                                                   float* __restrict__ sums, long long m,
                                                                   float value_coef, float* __restrict__ loss,
                                                                   float* __restrict__ stats, float* __restrict__ acc,
                                                                   float* __restrict__ kl_out, float* __restrict__ dstd) {
  partials_final_body(part, rows, 3, 4, sums);
  __syncthreads();
  if (threadIdx.x == 0) {  // (as ppo_loss_final)
    __threadfence_block();
    const float inv_m = 1.0f / (float)m;
    const float surr = sums[0] * inv_m, val = sums[1] * inv_m, kl = sums[2] * inv_m;
    loss[0] = surr + value_coef * val;
    stats[0] = surr;
    stats[1] = val;
    stats[2] = kl;
    if (acc) {
      acc[0] = acc[0] + surr;
      acc[1] = acc[1] + val;
    }
    if (kl_out) kl_out[0] = kl;
  }
  __syncthreads();
  partials_final_body(dpart, rows, k, 8, dstd);
}

hipError_t launch_ppo_loss_forward_backward(const gr_ppo_loss_args& a, const float* g, float value_coef, float* part,
                                            float* sums, float* loss, float* stats, float* acc, float* kl_out,
                                            float* dmu, float* dvalue, float* dpart, float* dstd, hipStream_t s) {
  const int blocks = ppo_loss_blocks(a.rows);
  hipLaunchKernelGGL(ppo_loss_fwd_bwd, dim3(blocks), dim3(256), 0, s, a, g, value_coef, part, dmu, dvalue, dpart);
  hipLaunchKernelGGL(ppo_loss_final_fb, dim3(1), dim3(CF_WAVES * 64), 0, s, part, dpart, blocks, a.k, sums,
                     (long long)a.rows, value_coef, loss, stats, acc, kl_out, dstd);
  return hipGetLastError();
}

hipError_t launch_ppo_loss_backward(const gr_ppo_loss_args& a, const float* g, int gv_index, float gv_coef, float* dmu,
                                    float* dvalue, float* part, float* dstd, hipStream_t s) {
  const int blocks = ppo_loss_blocks(a.rows);
  hipLaunchKernelGGL(ppo_loss_backward, dim3(blocks), dim3(256), 0, s, a, g, gv_index, gv_coef, dmu, dvalue, part);
  hipLaunchKernelGGL(partials_final, dim3(1), dim3(CF_WAVES * 64), 0, s, part, blocks, a.k, 8, dstd);
  return hipGetLastError();
}

// the graph-captured update's adaptive learning-rate rule (ppo.py:133-150 on the device, ppo.py _GraphedStep):
// kl > 2 desired: lr / 1.5 clamped below at lr_min; desired / 2 > kl > 0: lr * 1.5 clamped above at lr_max; in the
// fp32 ops of the torch expression it replaces (the thresholds are the Python doubles rounded to fp32)
__global__ void adaptive_lr(const float* __restrict__ kl, float* __restrict__ lr, float hi, float lo, float lr_min,
                            float lr_max) {
  if (threadIdx.x != 0) return;
  const float k = kl[0], r = lr[0];
  float up = r * 1.5f;
  up = up > lr_max ? lr_max : up;
  float down = r / 1.5f;
  down = down < lr_min ? lr_min : down;
  lr[0] = k > hi ? down : ((lo > k && k > 0.0f) ? up : r);
}

hipError_t launch_adaptive_lr(const float* kl, float* lr, float hi, float lo, float lr_min, float lr_max,
                              hipStream_t s) {
  hipLaunchKernelGGL(adaptive_lr, dim3(1), dim3(64), 0, s, kl, lr, hi, lo, lr_min, lr_max);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------------------------
// Adam and the gradient-norm clip of the PPO update over a device table of parameter segments
// (rsl_rl/flat_adam.py): torch.nn.utils.clip_grad_norm_ + torch.optim.Adam (ppo.py:179-181) as 2 + 2 launches
// instead of ~55 small per-tensor ones.  A workgroup of 256 threads owns GR_ADAM_BLOCK consecutive elements of one
// segment, thread t elements t, t + 256, t + 512, t + 768 (coalesced; the segments need no alignment: gradients are
// views of one flat buffer at any offset).

// the workgroup's segment: ballot over the table's block_start (ascending); wave-uniform, readfirstlane'd so the
// segment's fields are scalar loads
__device__ __forceinline__ int adam_segment_of(const gr_adam_args& a, int b) {
  const int l = threadIdx.x & 63;
  const int bs = l < a.nseg ? a.seg[l].block_start : 0x7fffffff;
  const unsigned long long m = __ballot(bs <= b);
  return __builtin_amdgcn_readfirstlane(__popcll(m) - 1);
}

// per workgroup: the sum of squares of its elements in double -> part[b]
__global__ __launch_bounds__(256) void adam_norm_part(gr_adam_args a) {
  __shared__ double sm[4];
  const int b = blockIdx.x, s = adam_segment_of(a, b);
  const gr_adam_segment g = a.seg[s];  // (a copy: scalar loads, no reload after the stores)
  const long long base = (long long)(b - g.block_start) * GR_ADAM_BLOCK;
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j < g.numel) {
      const double x = g.grad[j];
      acc += x * x;
    }
  }
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) a.part[b] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
}

// every workgroup sums part[] in the same order (the same coefficient everywhere), then scales its elements:
// coefficient min(1, max_norm / (norm + 1e-6)) (torch: clip_coef_clamped, multiplied always); workgroup 0 writes
// the norm
__global__ __launch_bounds__(256) void adam_clip_apply(gr_adam_args a, float max_norm, float* __restrict__ norm_out) {
  __shared__ double sm[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < a.nblocks; i += 256) acc += a.part[i];
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float norm = (float)sqrt((sm[0] + sm[1]) + (sm[2] + sm[3]));
  float c = max_norm / (norm + 1.0e-6f);
  c = (c < 1.0f || c != c) ? c : 1.0f;  // torch.clamp(clip_coef, max=1.0) keeps a NaN (non-finite gradients)
  const int b = blockIdx.x, s = adam_segment_of(a, b);
  if (b == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = norm;
  const gr_adam_segment g = a.seg[s];  // (a copy: scalar loads, no reload after the stores)
  const long long base = (long long)(b - g.block_start) * GR_ADAM_BLOCK;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j < g.numel) g.grad[j] = g.grad[j] * c;
  }
}

// step counters of the segments: +1, then the segment's coefficients in double (one thread per segment)
__global__ __launch_bounds__(64) void adam_count(gr_adam_args a) {
  const int s = threadIdx.x;
  if (s >= a.nseg) return;
  const int k = a.seg[s].step_slot;
  const float t = a.step[k] + 1.0f;
  a.step[k] = t;
  const double lr = a.lr_ptr ? (double)a.lr_ptr[0] : a.lr;
  a.coef[2 * k] = (float)(lr / (1.0 - pow(a.beta1, (double)t)));
  a.coef[2 * k + 1] = (float)sqrt(1.0 - pow(a.beta2, (double)t));
}

// torch's lerp (weight < 0.5): m + w (g - m); addcmul: v + ((1 - b2) g) g; addcdiv: p + (-step_size) (m / denom)
__global__ __launch_bounds__(256) void adam_update(gr_adam_args a) {
  const int b = blockIdx.x, s = adam_segment_of(a, b);
  const gr_adam_segment g = a.seg[s];  // (a copy: scalar loads, no reload after the stores)
  const long long base = (long long)(b - g.block_start) * GR_ADAM_BLOCK;
  const int k = g.step_slot;
  const float step_size = a.coef[2 * k], bc2s = a.coef[2 * k + 1];
  const float w1 = (float)(1.0 - a.beta1), b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long j = base + q * 256 + threadIdx.x;
    if (j >= g.numel) break;
    const float gr = g.grad[j];
    float m = g.exp_avg[j], v = g.exp_avg_sq[j];
    m = m + w1 * (gr - m);
    v = v * b2;
    v = v + (w2 * gr) * gr;
    g.exp_avg[j] = m;
    g.exp_avg_sq[j] = v;
    const float denom = sqrtf(v) / bc2s + a.eps;
    g.param[j] = g.param[j] + (-step_size) * (m / denom);
  }
}

// gr_adam_clip_step: the rate rule, the clip and Adam in 2 launches instead of 5 (adaptive_lr, norm_part, clip_apply,
// count, update), the same arithmetic.  Launch 1: the per-block squared norms; workgroup 0 also applies the rate rule
// (when kl is given) and each segment's first workgroup counts its step (nothing reads either before launch 2).
// Launch 2: every workgroup sums the partial norms in the same order (clip coefficient), derives its segment's bias
// corrections from the counted step (in double, as adam_count), then clips and updates its elements in one pass.
__global__ __launch_bounds__(256) void adam_norm_count(gr_adam_args a, const float* __restrict__ kl, float* lr,
                                                       float hi, float lo, float lr_min, float lr_max) {
  __shared__ double sm[4];
  const int b = blockIdx.x, s = adam_segment_of(a, b);
  const gr_adam_segment g = a.seg[s];
  const long long base = (long long)(b - g.block_start) * GR_ADAM_BLOCK;
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long long j = base + k * 256 + threadIdx.x;
    if (j < g.numel) {
      const double x = g.grad[j];
      acc += x * x;
    }
  }
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    a.part[b] = (sm[0] + sm[1]) + (sm[2] + sm[3]);
    if (b == g.block_start) a.step[g.step_slot] = a.step[g.step_slot] + 1.0f;
    if (b == 0 && kl) {  // adaptive_lr's expression
      const float k = kl[0], r = lr[0];
      float up = r * 1.5f;
      up = up > lr_max ? lr_max : up;
      float down = r / 1.5f;
      down = down < lr_min ? lr_min : down;
      lr[0] = k > hi ? down : ((lo > k && k > 0.0f) ? up : r);
    }
  }
}

__global__ __launch_bounds__(256) void adam_clip_update(gr_adam_args a, float max_norm, float* __restrict__ norm_out) {
  __shared__ double sm[4];
  double acc = 0.0;
  for (int i = threadIdx.x; i < a.nblocks; i += 256) acc += a.part[i];
  for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  const float norm = (float)sqrt((sm[0] + sm[1]) + (sm[2] + sm[3]));
  float c = max_norm / (norm + 1.0e-6f);
  c = (c < 1.0f || c != c) ? c : 1.0f;  // (as adam_clip_apply)
  const int b = blockIdx.x, s = adam_segment_of(a, b);
  if (b == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = norm;
  const gr_adam_segment g = a.seg[s];
  const long long base = (long long)(b - g.block_start) * GR_ADAM_BLOCK;
  // (as adam_count, from the step launch 1 counted)
  const float t = a.step[g.step_slot];
  const double lrd = a.lr_ptr ? (double)a.lr_ptr[0] : a.lr;
  const float step_size = (float)(lrd / (1.0 - pow(a.beta1, (double)t)));
  const float bc2s = (float)sqrt(1.0 - pow(a.beta2, (double)t));
  const float w1 = (float)(1.0 - a.beta1), b2 = (float)a.beta2, w2 = (float)(1.0 - a.beta2);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long long j = base + q * 256 + threadIdx.x;
    if (j >= g.numel) break;
    const float gr = g.grad[j] * c;
    g.grad[j] = gr;  // (clip_grad_norm_ scales the gradients in place)
    float m = g.exp_avg[j], v = g.exp_avg_sq[j];
    m = m + w1 * (gr - m);
    v = v * b2;
    v = v + (w2 * gr) * gr;
    g.exp_avg[j] = m;
    g.exp_avg_sq[j] = v;
    const float denom = sqrtf(v) / bc2s + a.eps;
    g.param[j] = g.param[j] + (-step_size) * (m / denom);
  }
}

hipError_t launch_adam_clip_step(const gr_adam_args& a, float max_norm, float* norm_out, const float* kl, float* lr,
                                 float hi, float lo, float lr_min, float lr_max, hipStream_t s) {
  hipLaunchKernelGGL(adam_norm_count, dim3(a.nblocks), dim3(256), 0, s, a, kl, lr, hi, lo, lr_min, lr_max);
  hipLaunchKernelGGL(adam_clip_update, dim3(a.nblocks), dim3(256), 0, s, a, max_norm, norm_out);
  return hipGetLastError();
}

hipError_t launch_adam_clip(const gr_adam_args& a, float max_norm, float* norm_out, hipStream_t s) {
  hipLaunchKernelGGL(adam_norm_part, dim3(a.nblocks), dim3(256), 0, s, a);
  hipLaunchKernelGGL(adam_clip_apply, dim3(a.nblocks), dim3(256), 0, s, a, max_norm, norm_out);
  return hipGetLastError();
}

hipError_t launch_adam_step(const gr_adam_args& a, hipStream_t s) {
  hipLaunchKernelGGL(adam_count, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(adam_update, dim3(a.nblocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace gr
