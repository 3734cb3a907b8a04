// gr_mlp.hip — the PPO update's actor and critic MLPs as whole-network fp32-MFMA kernels (gr_mlp_forward /
// gr_mlp_backward, include/gr.h).
//
// Reference: PPO.update (standalone/rsl_rl/ext/algorithms/ppo.py:103-190) evaluates, per mini-batch, the actor
// and the critic of upstream rsl_rl's ActorCritic (x -> Linear(d, H) -> LeakyReLU -> Linear(H, H) -> LeakyReLU ->
// Linear(H, k)) and back-propagates the loss through both.  In round 3 that was, per network and direction, a
// fused first layer, a hipBLASLt GEMM for the H x H layer, a fused head, a split-K batched GEMM + sum for the hidden
// weight gradient and three partial-sum reductions: ~20 launches per mini-batch step, the GEMMs at 0.41-0.56 of the
// fp32 MFMA peak on config C2's 24 576-row mini-batches (profiles/round03_train4096_fused_graphed_kernel_stats.csv).
//
// Here, for both networks at once (blockIdx.y = network):
//   mlp_fwd   : per 64-row tile, layer 1 -> LDS (h1, also stored for the backward) -> layer 2 on MFMA with the
//               wave's W2 rows in registers (z2 stored) -> activation -> layer 3 partials -> y.  The layout of
//               policy_f32_kernel (gr_policy_f32.hip): 8 waves, wave w owns hidden units [H/8 w, H/8 (w + 1)).
//   mlp_bwd   : per 64-row tile, gh2 = gy W3 (one MFMA per 16 x 16 tile, K = k <= 4) -> gz2 = gh2 lrelu'(z2) -> LDS
//               -> gh1 = gz2 W2 on MFMA with the wave's W2 COLUMNS in registers -> gz1 = gh1 lrelu'(h1) -> LDS;
//               the small weight gradients on MFMA contracting over the tile's rows (gW3 = gy^T h2, gW1 = gz1^T x)
//               and the bias sums in registers, one partial row per workgroup; gz2 stored for mlp_wgrad.
//   mlp_wgrad : gW2 = gz2^T h1, split over the rows (128 x 128 output blocks x row chunks), tiles staged in LDS
//               transposed so every fragment is one ds_read_b128; the four blocks of a chunk share an XCD (L2).
//   mlp_final : every partial row summed in a fixed order into the gradient vector [gW1 | gb1 | gW2 | gb2 | gW3 |
//               gb3] of each network (deterministic, no atomics).
// MFMA fragment convention (v_mfma_f32_16x16x4_f32): lane l = 16 g + j holds A[row j][k = g] and B[k = g][col j];
// the C tile holds rows 4 g + r of column j in register r.  "k order": k step 4 q + r of a contraction over H
// units is unit 16 q + 4 g + r, so a float4 of 4 consecutive units feeds 4 k steps.
#include <hip/hip_runtime.h>

#include "../../include/gr.h"
#include "gr_kernels.h"

namespace gr {

typedef float m4 __attribute__((ext_vector_type(4)));

constexpr int MW = 8;         // waves per workgroup (2 per SIMD)
constexpr int MC = 4;         // 16-row column tiles per workgroup tile
constexpr int ME = 16 * MC;   // rows per workgroup tile
constexpr int M_BLOCKS = 256; // persistent workgroups (one per CU; their registers / LDS hold one)

__device__ __forceinline__ m4 mf(float a, float b, m4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ m4 ld4(const float* p) { return *reinterpret_cast<const m4*>(p); }
__device__ __forceinline__ void st4(float* p, m4 v) { *reinterpret_cast<m4*>(p) = v; }
__device__ __forceinline__ float lrelu(float z, float s) { return z > 0.0f ? z : z * s; }
__device__ __forceinline__ float lrelu_d(float z, float s) { return z > 0.0f ? 1.0f : s; }
__device__ __forceinline__ m4 zero4() { return (m4){0.0f, 0.0f, 0.0f, 0.0f}; }

// ------------------------------------------------------------------------------------------------ forward
// LDS (floats): h1 [2][ME][H + 4], layer-3 partials [2][MW][ME][4], b1 [H], b2 [H]
constexpr size_t mlp_fwd_lds_bytes(int h) { return 4 * ((size_t)2 * ME * (h + 4) + 2 * MW * ME * 4 + 2 * h); }

template <int H, int Q1>
__global__ __launch_bounds__(MW * 64) void mlp_fwd(gr_mlp_args a) {
  constexpr int TW = H / (16 * MW);  // 16-unit tiles per wave and layer
  constexpr int Q = H / 16;
  constexpr int HP = H + 4;  // row stride of the LDS h1 tile (float4 reads of 16 rows hit distinct bank quads)
  const gr_mlp_net& net = a.net[blockIdx.y];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int n = (int)a.rows;  // (gr_mlp_* check rows * max(H, ldx) < 2^31: 32-bit offsets)
  const int D = net.d, K = net.k;
  const int ldx = (int)net.ldx;
  const float slope = a.slope;
  extern __shared__ float lds[];
  float* h1s = lds;                            // [2][ME][HP]
  float* parts = h1s + 2 * ME * HP;            // [2][MW][ME][4]
  float* b1s = parts + 2 * MW * ME * 4;        // [H]
  float* b2s = b1s + H;                        // [H]
  const float* __restrict__ W1 = net.w1;
  const float* __restrict__ W2 = net.w2;
  const float* __restrict__ W3 = net.w3;

  const int stride = gridDim.x * ME;
  m4 xo[MC][Q1];
  auto load_x = [&](int base) {
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      int r = base + 16 * c + j;
      r = r < n ? r : n - 1;
#pragma unroll
      for (int q = 0; q < Q1; ++q) {
        const int k = 16 * q + 4 * g;
        // (Q1 == 1 branch-free: a load inside a branch is waited for at the branch's end, which drains every
        // older load; with two input tiles the branch-free form costs spills)
        if constexpr (Q1 == 1) {
          const m4 v = ld4(net.x + r * ldx + (k < D ? k : 0));
          xo[c][q] = k < D ? v : zero4();
        } else {
          xo[c][q] = k < D ? ld4(net.x + r * ldx + k) : zero4();
        }
      }
    }
  };
  // issue order: what layer 1 of the first tile needs (biases, W1, x) before W2 / W3, so that layer 1 runs while
  // the W2 rows (256 KB per workgroup) are still arriving
  for (int i = threadIdx.x; i < H; i += MW * 64) {
    b1s[i] = net.b1[i];
    b2s[i] = net.b2[i];
  }
  float w1r[TW][Q1][4], w2r[TW][4 * Q], w3r[TW][4];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = 16 * (wave * TW + t) + j;
#pragma unroll
    for (int q = 0; q < Q1; ++q) {
      const int k = 16 * q + 4 * g;
      const m4 v0 = ld4(W1 + (size_t)row * D + (k < D ? k : 0));
      const m4 v = k < D ? v0 : zero4();
#pragma unroll
      for (int r = 0; r < 4; ++r) w1r[t][q][r] = v[r];
    }
  }
  load_x(blockIdx.x * ME);
  const float b3l = net.b3[g < K ? g : 0];
  const float b3v = g < K ? b3l : 0.0f;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int row = 16 * (wave * TW + t) + j;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const m4 v = ld4(W2 + (size_t)row * H + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) w2r[t][4 * q + r] = v[r];
    }
    // layer 3 A operand: rows = outputs (j < K), k = the wave's units
    const m4 v3l = ld4(W3 + (size_t)(j < K ? j : 0) * H + 16 * (wave * TW + t) + 4 * g);
    const m4 v3 = j < K ? v3l : zero4();
#pragma unroll
    for (int r = 0; r < 4; ++r) w3r[t][r] = v3[r];
  }
  // the 8 waves' layer-3 partials of a tile -> y; column tile e by wave (2 kt + e) mod 8
  auto epilogue = [&](int kt, int base) {
    const int e = (wave - 2 * kt) & (MW - 1);
    if (e >= MC) return;
    const float* pp = parts + (size_t)(kt & 1) * MW * ME * 4 + (16 * e + j) * 4 + g;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < MW; ++w) v += pp[w * ME * 4];
    const int r = base + 16 * e + j;
    if (r < n && g < K) net.y[r * K + g] = v + b3v;
  };
  __syncthreads();  // biases staged
  int kt = 0, prev_base = 0;
  for (int base = blockIdx.x * ME; base < n; base += stride, ++kt) {
    float* h1 = h1s + (kt & 1) * ME * HP;
    m4 acc[TW][MC];
    // ---- layer 1: the wave's h1 units of the tile -> LDS [row][unit] (the next tile's rows are loaded into the
    // same registers once these MFMAs have read them)
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const m4 bb = ld4(b1s + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
      for (int c = 0; c < MC; ++c) acc[t][c] = bb;
    }
#pragma unroll
    for (int kk = 0; kk < 4 * Q1; ++kk)
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int c = 0; c < MC; ++c) acc[t][c] = mf(w1r[t][kk >> 2][kk & 3], xo[c][kk >> 2][kk & 3], acc[t][c]);
    if (base + stride < n) load_x(base + stride);
    if (net.h1mask) {
      // the sign of h1 for mlp_bwd256h (the only thing the backward needs of h1): per 16-row x 16-unit tile and
      // register r the wave's ballot, bit 16 g + j = (unit 16 u16 + 4 g + r, row 16 c + j) > 0; lane
      // (t MC + c) 4 + r stores word [row tile][u16][r] (a vector store per lane)
      unsigned long long my = 0ull;
#pragma unroll
      for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int c = 0; c < MC; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const unsigned long long b = __ballot(acc[t][c][r] > 0.0f);
            if (lane == (t * MC + c) * 4 + r) my = b;
          }
      if (lane < TW * MC * 4) {
        const int t = lane / (MC * 4), c = (lane / 4) % MC, r = lane & 3;
        if (base + 16 * c < n)
          net.h1mask[(((size_t)(base / 16 + c)) * (H / 16) + wave * TW + t) * 4 + r] = my;
      }
    }
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < MC; ++c) {
        m4 v = acc[t][c];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = lrelu(v[r], slope);
        st4(h1 + (16 * c + j) * HP + 16 * (wave * TW + t) + 4 * g, v);
      }
    __syncthreads();  // h1 of this tile complete; the layer-3 partials of the previous tile complete
    if (kt > 0) epilogue(kt - 1, prev_base);
    // h1 rows -> global for the backward (coalesced: wave w stores rows w, w + 8, ...; lane l units 4 l .. 4 l + 3)
    if (4 * lane < H) {
#pragma unroll
      for (int rr = 0; rr < ME / MW; ++rr) {
        const int row = wave + MW * rr;
        if (base + row < n) st4(net.h1 + (base + row) * H + 4 * lane, ld4(h1 + row * HP + 4 * lane));
      }
    }
    // ---- layer 2: the wave's z2 units from all of h1
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const m4 bb = ld4(b2s + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
      for (int c = 0; c < MC; ++c) acc[t][c] = bb;
    }
    m4 hb[2][MC];
#pragma unroll
    for (int c = 0; c < MC; ++c) hb[0][c] = ld4(h1 + (16 * c + j) * HP + 4 * g);
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      if (q + 1 < Q) {
#pragma unroll
        for (int c = 0; c < MC; ++c) hb[(q + 1) & 1][c] = ld4(h1 + (16 * c + j) * HP + 16 * (q + 1) + 4 * g);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int c = 0; c < MC; ++c) acc[t][c] = mf(w2r[t][4 * q + r], hb[q & 1][c][r], acc[t][c]);
    }
    // z2 -> global (lane (g, j): units 16 t' + 4 g .. + 3 of row 16 c + j; the wave's TW tiles fill whole lines)
#pragma unroll
    for (int c = 0; c < MC; ++c) {
      const int r = base + 16 * c + j;
      if (r < n) {
#pragma unroll
        for (int t = 0; t < TW; ++t) st4(net.z2 + r * H + 16 * (wave * TW + t) + 4 * g, acc[t][c]);
      }
    }
    // ---- layer 3 partial over the wave's units -> LDS
    m4 o[MC];
#pragma unroll
    for (int c = 0; c < MC; ++c) o[c] = zero4();
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < MC; ++c) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[c] = mf(w3r[t][r], lrelu(acc[t][c][r], slope), o[c]);
      }
    if (g == 0) {
#pragma unroll
      for (int c = 0; c < MC; ++c) st4(parts + ((size_t)((kt & 1) * MW + wave) * ME + 16 * c + j) * 4, o[c]);
    }
    prev_base = base;
  }
  __syncthreads();
  if (kt > 0) epilogue(kt - 1, prev_base);
}

// ------------------------------------------------------------------------------------------------ backward
// (32-row tiles: the W2 columns take 128 registers; with 64-row tiles the accumulators spilled)
constexpr int BC = 2;
constexpr int BE = 16 * BC;
// per-workgroup partial row (floats): [gW1 (H D) | gb1 (H) | gb2 (H) | gW3 (k H) | gb3 (k)], padded to 4
__host__ __device__ constexpr int mlp_bwd_row(int h, int d, int k) { return (h * d + h + h + k * h + k + 3) & ~3; }
// LDS (floats): two [BE][H + 4] tiles (gz2; h2 then gz1) + gy rows [BE][4]
constexpr size_t mlp_bwd_lds_bytes(int h) { return 4 * ((size_t)2 * BE * (h + 4) + BE * 4); }

template <int H, int DT>
__global__ __launch_bounds__(MW * 64) void mlp_bwd(gr_mlp_args a, int rows_per_net_part) {
  constexpr int TW = H / (16 * MW);
  constexpr int Q = H / 16;
  constexpr int HP = H + 4;
  const gr_mlp_net& net = a.net[blockIdx.y];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int n = (int)a.rows;  // (gr_mlp_* check rows * max(H, ldx) < 2^31: 32-bit offsets)
  const int D = net.d, K = net.k;
  const int ldx = (int)net.ldx;
  const float slope = a.slope;
  extern __shared__ float lds[];
  float* gz2s = lds;               // [BE][HP]
  float* bufb = gz2s + BE * HP;    // [BE][HP]: h2, then gz1
  float* gys = bufb + BE * HP;     // [BE][4]
  const float* __restrict__ W2 = net.w2;
  const float* __restrict__ W3 = net.w3;

  // A operands: gh1^T = W2^T gz2^T -> row j of tile t is hidden unit i = 16 (wave TW + t) + j of h1, k step 4 q + r
  // is z2 unit 16 q + 4 g + r: W2[16 q + 4 g + r][i]
  float w2c[TW][4 * Q], w3a[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int i = 16 * (wave * TW + t) + j;
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) w2c[t][4 * q + r] = W2[(size_t)(16 * q + 4 * g + r) * H + i];
    // gh2^T = W3^T gy^T: row j = unit 16 (wave TW + t) + j, k = output g
    w3a[t] = g < K ? W3[(size_t)g * H + i] : 0.0f;
  }
  m4 gw1[TW][DT], gw3[TW];
  float gb1[TW][4], gb2[TW][4], gb3 = 0.0f;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    gw3[t] = zero4();
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) gw1[t][dt] = zero4();
#pragma unroll
    for (int r = 0; r < 4; ++r) gb1[t][r] = gb2[t][r] = 0.0f;
  }

  const int stride = gridDim.x * BE;
  for (int base = blockIdx.x * BE; base < n; base += stride) {
    // ---- gy rows of the tile -> LDS (rows past the end: 0, so they add nothing anywhere)
    if (threadIdx.x < BE * 4) {
      const int row = threadIdx.x >> 2, kk = threadIdx.x & 3;
      const int r = base + row;
      gys[threadIdx.x] = (r < n && kk < K) ? net.gy[r * K + kk] : 0.0f;
    }
    __syncthreads();  // (1) gy staged; the previous tile's readers of gz2s / bufb are done
    // ---- gh2 = gy W3 (one MFMA per tile, K = k <= 4), gz2 = gh2 lrelu'(z2), h2 = lrelu(z2)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int r = base + 16 * c + j;
      const int rr = r < n ? r : n - 1;
      const float gyv = gys[(16 * c + j) * 4 + g];  // B[k = g][row j]
      if (wave == 0) gb3 += gyv;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int u = 16 * (wave * TW + t) + 4 * g;
        const m4 gh = mf(w3a[t], gyv, zero4());
        const m4 z = ld4(net.z2 + rr * H + u);
        m4 gz, h2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          gz[q] = gh[q] * lrelu_d(z[q], slope);
          h2[q] = lrelu(z[q], slope);
          gb2[t][q] += gz[q];
        }
        st4(gz2s + (16 * c + j) * HP + u, gz);
        st4(bufb + (16 * c + j) * HP + u, h2);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // (2) gz2 and h2 of the tile in LDS
    // ---- gW3 += gy^T h2: rows = outputs (j < k), contraction over the tile's rows (k step = rows 4 s + g)
#pragma unroll 4
    for (int s = 0; s < BE / 4; ++s) {
      const int row = 4 * s + g;
      const float av = j < 4 ? gys[row * 4 + j] : 0.0f;
#pragma unroll
      for (int t = 0; t < TW; ++t) gw3[t] = mf(av, bufb[row * HP + 16 * (wave * TW + t) + j], gw3[t]);
    }
    // ---- gh1 = gz2 W2 for the wave's h1 units, all rows of the tile
    m4 acc[TW][BC];
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < BC; ++c) acc[t][c] = zero4();
    // (B fragments single-buffered: the W2 columns take 128 registers; the SIMD's other wave covers the LDS latency)
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      m4 gb[BC];
#pragma unroll
      for (int c = 0; c < BC; ++c) gb[c] = ld4(gz2s + (16 * c + j) * HP + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int c = 0; c < BC; ++c) acc[t][c] = mf(w2c[t][4 * q + r], gb[c][r], acc[t][c]);
      __builtin_amdgcn_sched_barrier(0);  // (no hoisting of later fragments' loads: registers)
    }
    // gz1 = gh1 lrelu'(h1) (h1 from the forward's saved rows)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int r = base + 16 * c + j;
      const int rr = r < n ? r : n - 1;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const m4 hv = ld4(net.h1 + rr * H + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[t][c][q] *= lrelu_d(hv[q], slope);
          gb1[t][q] += acc[t][c][q];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // (3) every wave is done with h2 (bufb) and gz2s
    // gz1 -> bufb; gz2 rows -> global for mlp_wgrad (coalesced rows)
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < BC; ++c) st4(bufb + (16 * c + j) * HP + 16 * (wave * TW + t) + 4 * g, acc[t][c]);
    if (4 * lane < H) {
#pragma unroll
      for (int rr = 0; rr < BE / MW; ++rr) {
        const int row = wave + MW * rr;
        if (base + row < n) st4(net.gz2 + (base + row) * H + 4 * lane, ld4(gz2s + row * HP + 4 * lane));
      }
    }
    __syncthreads();  // (4) gz1 in LDS
    // ---- gW1 += gz1^T x: rows = the wave's h1 units, cols = inputs (DT tiles of 16), k step = rows 4 s + g
#pragma unroll 4
    for (int s = 0; s < BE / 4; ++s) {
      const int row = 4 * s + g;
      int r = base + row;
      r = r < n ? r : n - 1;  // (the tail rows' gz1 is 0)
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int dcol = 16 * dt + j;
        const float xv = dcol < D ? net.x[r * ldx + dcol] : 0.0f;
#pragma unroll
        for (int t = 0; t < TW; ++t) gw1[t][dt] = mf(bufb[row * HP + 16 * (wave * TW + t) + j], xv, gw1[t][dt]);
      }
    }
  }
  // ---- the workgroup's partial row
  float* pr = a.partial + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (size_t)rows_per_net_part;
  // bias sums: over the 16 lanes j of each g group (fixed butterfly order)
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v1 = gb1[t][q], v2 = gb2[t][q];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        v1 += __shfl_xor(v1, off);
        v2 += __shfl_xor(v2, off);
      }
      gb1[t][q] = v1;
      gb2[t][q] = v2;
    }
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int u0 = 16 * (wave * TW + t);
    // gW1 [H][D]: C rows = units u0 + 4 g + q, col = input 16 dt + j
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (16 * dt + j < D) pr[(size_t)(u0 + 4 * g + q) * D + 16 * dt + j] = gw1[t][dt][q];
    if (j == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pr[H * D + u0 + 4 * g + q] = gb1[t][q];
        pr[H * D + H + u0 + 4 * g + q] = gb2[t][q];
      }
    }
    // gW3 [k][H]: C rows = outputs 4 g + q (g == 0, q < k), col = unit u0 + j
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < K) pr[H * D + 2 * H + q * H + u0 + j] = gw3[t][q];
    }
  }
  if (wave == 0) {
    float v = gb3;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off);
    if (j == 0 && g < K) pr[H * D + 2 * H + K * H + g] = v;
  }
}

// ------------------------------------------------------------------------------------------------ backward, H = 256
// mlp_bwd's arithmetic with the tile's inputs (z2, h1, x, gy rows) staged into LDS by LDS-DMA (global_load_lds) one
// tile ahead.  At one workgroup per CU (the W2 columns hold 128 registers of each lane) the barriers keep the SIMD's
// two waves in step, so mlp_bwd's global loads after its barriers stalled both: here they are issued while the
// previous tile computes and waited for with counted vmcnt, behind raw barriers that do not drain them.
//   per tile i, per wave, in issue order:  P_a (after barrier 2): z2 rows of tile i+1 (4 x 1 KB), gy of tile i+1
//   (waves 6, 7: 1 each);  P_b (after barrier 3): gz2 row stores (4), h1 rows of tile i+1 (4), x of tile i+1
//   (waves 0 .. 2 DT - 1: 1 each).  Loads, stores and LDS-DMA retire in issue order on vmcnt, so
//   - end of tile i, before barrier 1 of i+1: vmcnt(8) leaves only P_b's 8-9 youngest -> z2 / gy of i+1 are in LDS;
//   - tile i+1 before its gz1: vmcnt(4) leaves only what follows h1 (x, then P_a of i+1 with its 4 z2 rows) -> h1
//     and x of i+1 are in; vmcnt(0) when there is no tile i+2 (no P_a).
// Every DMA is issued for every row (past the end: row n - 1, finite data that the tail's zero gy cancels), so the
// counts hold; the tail rows' gy is masked where it is read.
constexpr int HB = 256, HBP = HB + 4;
__host__ __device__ constexpr size_t mlp_bwd256_lds_bytes(int dt) {
  return 4 * ((size_t)4 * BE * HBP + 2 * BE * 16 * dt + 2 * BE * 4);
}
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;
// LDS-DMA, one wave instruction: lane l's `size` bytes from g (per lane) to LDS at l_base (wave-uniform) + l * size
__device__ __forceinline__ void glds16(const float* g, float* l_base) {
  __builtin_amdgcn_global_load_lds((glob_void_t*)g, (lds_void_t*)l_base, 16, 0, 0);
}
__device__ __forceinline__ void glds4(const float* g, float* l_base) {
  __builtin_amdgcn_global_load_lds((glob_void_t*)g, (lds_void_t*)l_base, 4, 0, 0);
}
// workgroup barrier that leaves vector-memory operations in flight (__syncthreads() would wait for vmcnt(0))
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int DT>
__global__ __launch_bounds__(MW * 64) void mlp_bwd256(gr_mlp_args a, int rows_per_net_part) {
  constexpr int H = HB, HP = HBP, TW = H / (16 * MW), Q = H / 16;
  constexpr int XW = 16 * DT;  // x row in LDS (floats)
  const gr_mlp_net& net = a.net[blockIdx.y];
  // (the wave index as a scalar: the DMA rows and LDS bases are wave-uniform, so they stay in SGPRs)
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4,
            j = lane & 15;
  const int n = (int)a.rows;  // (gr_mlp_* check rows * max(H, ldx) < 2^31: 32-bit offsets)
  const int D = net.d, K = net.k;
  const int ldx = (int)net.ldx;
  const float slope = a.slope;
  extern __shared__ float lds[];
  float* gz2s = lds;             // [BE][HP]
  float* bufb = gz2s + BE * HP;  // [BE][HP]: h2, then gz1
  float* z2s = bufb + BE * HP;   // [BE][HP]: z2 rows of the tile (LDS-DMA)
  float* h1s = z2s + BE * HP;    // [BE][HP]: h1 rows of the tile (LDS-DMA)
  float* xs = h1s + BE * HP;     // [2][BE][XW]: x rows (LDS-DMA, by tile parity)
  float* gys = xs + 2 * BE * XW; // [2][BE][4]: gy rows (LDS-DMA, by tile parity; outputs >= k stay 0)
  const float* __restrict__ W2 = net.w2;
  const float* __restrict__ W3 = net.w3;
  // the row arrays' addresses in SGPRs for the whole kernel (opaque, so they are not re-loaded from the kernel
  // arguments inside the tile loop: an outstanding scalar load there makes hipcc wait lgkmcnt(0) instead of the
  // counted wait that keeps the next fragments' LDS reads in flight under the MFMAs)
  const float* z2g = net.z2;
  const float* h1g = net.h1;
  const float* xg = net.x;
  const float* gyg = net.gy;
  float* gz2g = net.gz2;
  asm volatile("" : "+s"(z2g), "+s"(h1g), "+s"(xg), "+s"(gyg), "+s"(gz2g));

  float w2c[TW][4 * Q], w3a[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) w3a[t] = g < K ? W3[(size_t)g * H + 16 * (wave * TW + t) + j] : 0.0f;
  // (consumed here, before any DMA: hipcc otherwise waits vmcnt(0) at the first use of an ordinary load's result
  // while an LDS-DMA is in flight, draining the next tile's DMA every tile)
#pragma unroll
  for (int t = 0; t < TW; ++t) asm volatile("" : "+v"(w3a[t]));
  // W2 columns (lane (g, j): W2[16 q + 4 g + r][unit i]), staged through LDS by LDS-DMA in 4 chunks of 64 W2 rows,
  // two in flight, into the tiles' space ([64][HP] twice): one 1-KB row per wave instruction, instead of 128
  // column loads per lane gathering 64-byte segments (8 x the L2 requests; ~10 us of a 24 576-row backward)
  float* const stg0 = lds;                // gz2s + bufb
  float* const stg1 = lds + 2 * BE * HP;  // z2s + h1s
  auto issue_w2 = [&](int c, float* dst) {
#pragma unroll
    for (int rr = 0; rr < 64 / MW; ++rr) {
      const int row = wave + MW * rr;
      glds16(W2 + (size_t)(64 * c + row) * H + 4 * lane, dst + row * HP);
    }
  };
  issue_w2(0, stg0);
  issue_w2(1, stg1);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c < 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // chunk c in (chunk c + 1 may be in flight)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    const float* src = (c & 1) ? stg1 : stg0;
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      const int i = 16 * (wave * TW + t) + j;
#pragma unroll
      for (int q = 4 * c; q < 4 * c + 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) w2c[t][4 * q + r] = src[(16 * (q - 4 * c) + 4 * g + r) * HP + i];
    }
    if (c + 2 < 4) {
      raw_barrier();  // every wave has read chunk c
      issue_w2(c + 2, (c & 1) ? stg1 : stg0);
    }
  }
  raw_barrier();  // every wave has read the last chunk (its space is the DMA targets, zeroed next)
  m4 gw1[TW][DT], gw3[TW];
  float gb1[TW][4], gb2[TW][4], gb3 = 0.0f;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    gw3[t] = zero4();
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) gw1[t][dt] = zero4();
#pragma unroll
    for (int r = 0; r < 4; ++r) gb1[t][r] = gb2[t][r] = 0.0f;
  }
  // the DMA targets start at 0: lanes it never writes (x columns >= d, gy outputs >= k) must read 0, and
  // never-written LDS may hold NaN patterns
  for (int i = threadIdx.x; i < 2 * BE * HP + 2 * BE * XW + 2 * BE * 4; i += MW * 64) z2s[i] = 0.0f;
  __syncthreads();  // (no DMA in flight yet; also waits for the weight loads)

  auto clamp_row = [&](int r) { return r < n ? r : n - 1; };
  // P_a: z2 rows (wave w: rows w, w + 8, w + 16, w + 24) and gy (waves 6, 7: 16 rows x 4 outputs each)
  auto issue_a = [&](int tb, int par) {
#pragma unroll
    for (int rr = 0; rr < BE / MW; ++rr) {
      const int row = wave + MW * rr;
      glds16(z2g + clamp_row(tb + row) * H + 4 * lane, z2s + row * HP);
    }
    if (wave >= MW - 2) {
      const int row = 16 * (wave - (MW - 2)) + (lane >> 2), kk = lane & 3;
      if (kk < K) glds4(gyg + clamp_row(tb + row) * K + kk, gys + par * BE * 4 + 16 * (wave - (MW - 2)) * 4);
    }
  };
  // P_b: h1 rows, x (waves 0 .. 2 DT - 1: 16 / DT rows x XW floats each)
  auto issue_b = [&](int tb, int par) {
#pragma unroll
    for (int rr = 0; rr < BE / MW; ++rr) {
      const int row = wave + MW * rr;
      glds16(h1g + clamp_row(tb + row) * H + 4 * lane, h1s + row * HP);
    }
    if (wave < 2 * DT) {
      constexpr int RPI = 16 / DT;  // rows per instruction
      const int row = RPI * wave + lane / (4 * DT), c4 = 4 * (lane % (4 * DT));
      if (c4 < D) glds16(xg + clamp_row(tb + row) * ldx + c4, xs + par * BE * XW + RPI * wave * XW);
    }
  };

  const int stride = gridDim.x * BE;
  int base = blockIdx.x * BE;
  if (base < n) {
    issue_a(base, 0);
    issue_b(base, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier();
  for (int kt = 0; base < n; base += stride, ++kt) {
    const bool has_next = base + stride < n;
    const float* gyt = gys + (kt & 1) * BE * 4;
    const float* xt = xs + (kt & 1) * BE * XW;
    // ---- gh2 = gy W3, gz2 = gh2 lrelu'(z2), h2 = lrelu(z2)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int row = 16 * c + j;
      const float gyv = base + row < n ? gyt[row * 4 + g] : 0.0f;  // B[k = g][row j]
      if (wave == 0) gb3 += gyv;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const int u = 16 * (wave * TW + t) + 4 * g;
        const m4 gh = mf(w3a[t], gyv, zero4());
        const m4 z = ld4(z2s + row * HP + u);
        m4 gz, h2;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          gz[q] = gh[q] * lrelu_d(z[q], slope);
          h2[q] = lrelu(z[q], slope);
          gb2[t][q] += gz[q];
        }
        st4(gz2s + row * HP + u, gz);
        st4(bufb + row * HP + u, h2);
      }
    }
    raw_barrier();  // (2) gz2 and h2 of the tile in LDS; every wave is done with z2s
    if (has_next) issue_a(base + stride, (kt + 1) & 1);
    // ---- gW3 += gy^T h2 (k step = rows 4 s + g)
#pragma unroll 4
    for (int s = 0; s < BE / 4; ++s) {
      const int row = 4 * s + g;
      const float av = (j < 4 && base + row < n) ? gyt[row * 4 + j] : 0.0f;
#pragma unroll
      for (int t = 0; t < TW; ++t) gw3[t] = mf(av, bufb[row * HP + 16 * (wave * TW + t) + j], gw3[t]);
    }
    // ---- gh1 = gz2 W2 for the wave's h1 units
    m4 acc[TW][BC];
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < BC; ++c) acc[t][c] = zero4();
    // (B fragments single-buffered, the next block's reads not hoisted: measured faster than double-buffered
    // fragments, with hipcc's or with counted waits (mlp_bwd256 at 393 216 rows 1.06 vs 1.08-1.11 ms))
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      m4 gb[BC];
#pragma unroll
      for (int c = 0; c < BC; ++c) gb[c] = ld4(gz2s + (16 * c + j) * HP + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < TW; ++t)
#pragma unroll
          for (int c = 0; c < BC; ++c) acc[t][c] = mf(w2c[t][4 * q + r], gb[c][r], acc[t][c]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // h1 (and x) of this tile: this wave's DMA retired, then every wave's (barrier)
    if (has_next) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // (2b)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int row = 16 * c + j;
#pragma unroll
      for (int t = 0; t < TW; ++t) {
        const m4 hv = ld4(h1s + row * HP + 16 * (wave * TW + t) + 4 * g);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          acc[t][c][q] *= lrelu_d(hv[q], slope);
          gb1[t][q] += acc[t][c][q];
        }
      }
    }
    raw_barrier();  // (3) every wave is done with h2 (bufb), gz2s and h1s
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
      for (int c = 0; c < BC; ++c) st4(bufb + (16 * c + j) * HP + 16 * (wave * TW + t) + 4 * g, acc[t][c]);
#pragma unroll
    for (int rr = 0; rr < BE / MW; ++rr) {
      const int row = wave + MW * rr;
      if (base + row < n) st4(gz2g + (base + row) * H + 4 * lane, ld4(gz2s + row * HP + 4 * lane));
    }
    if (has_next) issue_b(base + stride, (kt + 1) & 1);
    raw_barrier();  // (4) gz1 in LDS
    // ---- gW1 += gz1^T x (k step = rows 4 s + g)
#pragma unroll 4
    for (int s = 0; s < BE / 4; ++s) {
      const int row = 4 * s + g;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int dcol = 16 * dt + j;
        const float xv = dcol < D ? xt[row * XW + dcol] : 0.0f;
#pragma unroll
        for (int t = 0; t < TW; ++t) gw1[t][dt] = mf(bufb[row * HP + 16 * (wave * TW + t) + j], xv, gw1[t][dt]);
      }
    }
    if (has_next) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // z2 / gy of the next tile
      raw_barrier();  // (1) of the next tile: its z2 / gy in LDS; the readers of bufb (gz1) and xt are done
    }
  }
  // ---- the workgroup's partial row (as mlp_bwd)
  float* pr = a.partial + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * (size_t)rows_per_net_part;
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v1 = gb1[t][q], v2 = gb2[t][q];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        v1 += __shfl_xor(v1, off);
        v2 += __shfl_xor(v2, off);
      }
      gb1[t][q] = v1;
      gb2[t][q] = v2;
    }
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int u0 = 16 * (wave * TW + t);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (16 * dt + j < D) pr[(size_t)(u0 + 4 * g + q) * D + 16 * dt + j] = gw1[t][dt][q];
    if (j == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        pr[H * D + u0 + 4 * g + q] = gb1[t][q];
        pr[H * D + H + u0 + 4 * g + q] = gb2[t][q];
      }
    }
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < K) pr[H * D + 2 * H + q * H + u0 + j] = gw3[t][q];
    }
  }
  if (wave == 0) {
    float v = gb3;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off);
    if (j == 0 && g < K) pr[H * D + 2 * H + K * H + g] = v;
  }
}

// ------------------------------------------------------------------------------------------------ backward, H = 256,
// two workgroups per CU (round 5)
// mlp_bwd256 keeps all 8 waves of a CU in one workgroup: five barriers per 32-row tile hold the two waves of every
// SIMD in step, so the non-MFMA phases of both (gz2, gz1, the small weight gradients' dependent MFMA chains, the
// DMA waits) leave the matrix pipe idle at once (MFMA busy 56 % at 24 576 rows, 67 % at 393 216).  Here a workgroup
// is 4 waves and owns HALF of the h1 units (128; wave w: units 128 h + 32 w .. + 31, the W2 columns of those in
// registers as before), so two workgroups share a CU and drift apart: one's elementwise phase runs under the
// other's GEMM.  Per tile, two barriers:
//   B1  z2 / gy / x / h1-sign rows of the tile in LDS (LDS-DMA issued one tile ahead; z2 single-buffered, the
//       small inputs double-buffered); every wave is done with the previous tile's gz2 (its GEMM operand).
//       gW3 += gy^T h2 for the workgroup's half of the z2 units (B operand lrelu(z2) from LDS); gz2 = (gy W3) *
//       lrelu'(z2) for ALL 256 z2 units (each workgroup of the pair computes the full tile: the GEMM contracts over
//       it), wave w the units 32 w .. + 31 and 128 + 32 w .. + 31, of which the half's own ones feed gb2 and the
//       global gz2 rows mlp_wgrad reads.
//   B2  gz2 tile complete, z2 free: the next tile's DMA is issued.  GEMM gh1 = gz2 W2 as C[rows x units]
//       (A = gz2 fragments from LDS, B = the W2 columns), so its output fragment is directly the A operand of
//       gW1 = gz1^T x (k = the tile's rows) and gz1 = gh1 lrelu'(h1) needs only the SIGN of h1: 1 bit per element
//       from mlp_fwd (gr_mlp_net.h1mask) instead of the h1 rows (1 KB per row and network).
// LDS (floats): z2s [BE][HBP], gz2s [BE][HBP], xs [2][BE][16 DT], gys [2][BE][4], masks [2][2][8][4] x u64; the W2
// staging at start-up (2 chunks of 64 W2 rows x 128 columns) reuses z2s + gz2s.
constexpr int HWV = 4;          // waves per workgroup
constexpr int HSP = 128 + 4;    // LDS row stride of the W2 staging chunks
__host__ __device__ constexpr size_t mlp_bwd256h_lds_bytes(int dt) {
  return 4 * ((size_t)2 * BE * HBP + 2 * BE * 16 * dt + 2 * BE * 4 + 2 * 2 * 8 * 4 * 2);
}

template <int DT>
__global__ __launch_bounds__(HWV * 64, 2) void mlp_bwd256h(gr_mlp_args a, int rows_per_net_part) {
  constexpr int H = HB, HP = HBP, Q = H / 16;
  constexpr int XW = 16 * DT;
  const gr_mlp_net& net = a.net[blockIdx.y];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), g = lane >> 4,
            j = lane & 15;
  const int half = blockIdx.x & 1, rg = blockIdx.x >> 1, groups = gridDim.x >> 1;
  const int n = (int)a.rows;  // (gr_mlp_* check rows * max(H, ldx) < 2^31: 32-bit offsets)
  const int D = net.d, K = net.k;
  const int ldx = (int)net.ldx;
  const float slope = a.slope;
  extern __shared__ float lds[];
  float* z2s = lds;                                           // [BE][HP]
  float* gz2s = z2s + BE * HP;                                // [BE][HP]
  float* xs = gz2s + BE * HP;                                 // [2][BE][XW]
  float* gys = xs + 2 * BE * XW;                              // [2][BE][4]
  unsigned long long* mks = reinterpret_cast<unsigned long long*>(gys + 2 * BE * 4);  // [2][2 c][8 u16][4 r]
  const float* __restrict__ W2 = net.w2;
  const float* __restrict__ W3 = net.w3;
  const float* z2g = net.z2;
  const float* xg = net.x;
  const float* gyg = net.gy;
  const unsigned long long* mkg = reinterpret_cast<const unsigned long long*>(net.h1mask);
  float* gz2g = net.gz2;
  asm volatile("" : "+s"(z2g), "+s"(xg), "+s"(gyg), "+s"(mkg), "+s"(gz2g));
  const int U0 = 128 * half + 32 * wave;  // this wave's h1 units (GEMM output) U0 .. U0 + 31
  // this wave's z2 unit tiles for gz2: o-tiles 2w, 2w + 1, 8 + 2w, 9 + 2w; the half's own ones are 8 half + 2w + e
  float w3a[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ot = (e < 2 ? 2 * wave + e : 8 + 2 * wave + (e - 2));
    w3a[e] = g < K ? W3[(size_t)g * H + 16 * ot + j] : 0.0f;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(w3a[e]));  // (consumed before any DMA, as mlp_bwd256)
  // W2 columns U0 .. U0 + 31 (lane (g, j): W2[16 q + 4 g + r][U0 + 16 t + j]), staged by LDS-DMA: 4 chunks of 64 W2
  // rows x the half's 128 columns, two in flight, one 512-B row per wave instruction (lanes 0..31)
  float w2c[2][4 * Q];
  float* const stg0 = lds;
  float* const stg1 = lds + 64 * HSP;
  auto issue_w2 = [&](int c, float* dst) {
#pragma unroll
    for (int k = 0; k < 64 / HWV; ++k) {
      const int row = wave + HWV * k;
      if (lane < 32) glds16(W2 + (size_t)(64 * c + row) * H + 128 * half + 4 * lane, dst + row * HSP);
    }
  };
  issue_w2(0, stg0);
  issue_w2(1, stg1);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c < 3) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // chunk c in (chunk c + 1 may be in flight)
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();
    const float* src = (c & 1) ? stg1 : stg0;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int i = 32 * wave + 16 * t + j;
#pragma unroll
      for (int q = 4 * c; q < 4 * c + 4; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) w2c[t][4 * q + r] = src[(16 * (q - 4 * c) + 4 * g + r) * HSP + i];
    }
    if (c + 2 < 4) {
      raw_barrier();  // every wave has read chunk c
      issue_w2(c + 2, (c & 1) ? stg1 : stg0);
    }
  }
  raw_barrier();  // every wave has read the last chunk (its space is the DMA targets, zeroed next)
  m4 gw1[2][DT], gw3[2];
  float gb1[2], gb2[2][4], gb3 = 0.0f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    gw3[t] = zero4();
    gb1[t] = 0.0f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) gw1[t][dt] = zero4();
#pragma unroll
    for (int r = 0; r < 4; ++r) gb2[t][r] = 0.0f;
  }
  // the small DMA targets start at 0 (x columns >= d, gy outputs >= k are never written; never-written LDS may
  // hold NaN patterns)
  for (int i = threadIdx.x; i < 2 * BE * XW + 2 * BE * 4; i += HWV * 64) xs[i] = 0.0f;
  __syncthreads();

  auto clamp_row = [&](int r) { return r < n ? r : n - 1; };
  // one tile's inputs: z2 rows (wave w: rows w + 4 k), gy (wave 3), x (waves 0 .. 2 DT - 1), h1 signs (wave 2)
  auto issue_in = [&](int tb, int par) {
#pragma unroll
    for (int k = 0; k < BE / HWV; ++k) {
      const int row = wave + HWV * k;
      glds16(z2g + (size_t)clamp_row(tb + row) * H + 4 * lane, z2s + row * HP);
    }
    if (wave == HWV - 1) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int row = 16 * h + (lane >> 2), kk = lane & 3;
        if (kk < K) glds4(gyg + (size_t)clamp_row(tb + row) * K + kk, gys + par * BE * 4 + 16 * h * 4);
      }
    }
    if (wave < 2 * DT) {
      constexpr int RPI = 16 / DT;  // rows per instruction
      const int row = RPI * wave + lane / (4 * DT), c4 = 4 * (lane % (4 * DT));
      if (c4 < D) glds16(xg + (size_t)clamp_row(tb + row) * ldx + c4, xs + par * BE * XW + RPI * wave * XW);
    }
    if (wave == 2 && lane < 32) {
      // [c][u16 8 half .. + 7][r]: 2 x 256 contiguous bytes (row tiles tb / 16 + c, clamped)
      const int c = lane >> 4, rt = clamp_row(tb + 16 * c) >> 4;
      glds16(reinterpret_cast<const float*>(mkg + ((size_t)rt * (H / 16) + 8 * half) * 4) + 4 * (lane & 15),
             reinterpret_cast<float*>(mks + par * 64));
    }
  };

  const int stride = groups * BE;
  int base = rg * BE;
  if (base < n) issue_in(base, 0);
  for (int kt = 0; base < n; base += stride, ++kt) {
    const int par = kt & 1;
    const bool has_next = base + stride < n;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // (B1) this tile's inputs in LDS; every wave is done with the previous tile's gz2
    const float* gyt = gys + par * BE * 4;
    const float* xt = xs + par * BE * XW;
    const unsigned long long* mkt = mks + par * 64;
    // ---- gW3 += gy^T h2 for the half's z2 units 128 half + 32 w + 16 t + j (k step = rows 4 s + g)
#pragma unroll 4
    for (int s = 0; s < BE / 4; ++s) {
      const int row = 4 * s + g;
      const float av = (j < 4 && base + row < n) ? gyt[row * 4 + j] : 0.0f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
        gw3[t] = mf(av, lrelu(z2s[row * HP + 128 * half + 32 * wave + 16 * t + j], slope), gw3[t]);
    }
    // ---- gz2 = (gy W3) lrelu'(z2) for the wave's four z2 unit tiles, all rows of the tile -> LDS; the half's own
    // ones also -> gb2 and the global gz2 rows (mlp_wgrad)
#pragma unroll
    for (int c = 0; c < BC; ++c) {
      const int row = 16 * c + j;
      const bool live = base + row < n;
      const float gyv = live ? gyt[row * 4 + g] : 0.0f;  // B[k = g][row j]
      if (half == 0 && wave == 0) gb3 += gyv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int ot = (e < 2 ? 2 * wave + e : 8 + 2 * wave + (e - 2));
        const int u = 16 * ot + 4 * g;
        const m4 gh = mf(w3a[e], gyv, zero4());
        const m4 z = ld4(z2s + row * HP + u);
        m4 gz;
#pragma unroll
        for (int q = 0; q < 4; ++q) gz[q] = gh[q] * lrelu_d(z[q], slope);
        st4(gz2s + row * HP + u, gz);
        if ((e >> 1) == half) {  // (wave-uniform)
#pragma unroll
          for (int q = 0; q < 4; ++q) gb2[e & 1][q] += gz[q];
          if (live) st4(gz2g + (size_t)(base + row) * H + u, gz);
        }
      }
    }
    raw_barrier();  // (B2) gz2 of the tile in LDS; every wave is done with z2s
    if (has_next) issue_in(base + stride, par ^ 1);
    // ---- gh1 = gz2 W2 as C[rows 16 c .. + 15 x units U0 + 16 t .. + 15]
    m4 acc[2][BC];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int c = 0; c < BC; ++c) acc[t][c] = zero4();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      m4 gb[BC];
#pragma unroll
      for (int c = 0; c < BC; ++c) gb[c] = ld4(gz2s + (16 * c + j) * HP + 16 * q + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int c = 0; c < BC; ++c) acc[t][c] = mf(gb[c][r], w2c[t][4 * q + r], acc[t][c]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- gz1 = gh1 lrelu'(h1) (sign bits from the forward), gb1, gW1 += gz1^T x: lane (g, j) holds rows
    // 16 c + 4 g + r of unit U0 + 16 t + j, which is gW1's A fragment for k step (c, r) as it stands
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int c = 0; c < BC; ++c) {
        // word [c][u16 = 2 w + t][r' = j % 4]: bit 16 (j / 4) + 4 g + r = (row 16 c + 4 g + r, unit 16 u16 + j)
        const unsigned long long mw = mkt[(c * 8 + 2 * wave + t) * 4 + (j & 3)];
        const uint32_t nib = (uint32_t)(mw >> (16 * (j >> 2) + 4 * g)) & 0xfu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float gz1 = acc[t][c][r] * (((nib >> r) & 1u) ? 1.0f : slope);
          gb1[t] += gz1;
          const int row = 16 * c + 4 * g + r;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            const int dcol = 16 * dt + j;
            gw1[t][dt] = mf(gz1, dcol < D ? xt[row * XW + dcol] : 0.0f, gw1[t][dt]);
          }
        }
      }
    }
  }
  // ---- the workgroup's part of the partial row of its row group (the pair's two halves fill it)
  float* pr = a.partial + ((size_t)blockIdx.y * groups + rg) * (size_t)rows_per_net_part;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int u0 = U0 + 16 * t;
    // gW1 [H][D]: C rows = units u0 + 4 g + q, col = input 16 dt + j
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (16 * dt + j < D) pr[(size_t)(u0 + 4 * g + q) * D + 16 * dt + j] = gw1[t][dt][q];
    // gb1: unit u0 + j, summed over the 4 row groups g
    float v = gb1[t];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (g == 0) pr[H * D + u0 + j] = v;
    // gb2: z2 unit 128 half + 32 w + 16 t + 4 g + q, summed over the rows j
    const int o0 = 128 * half + 32 * wave + 16 * t;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float b2 = gb2[t][q];
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) b2 += __shfl_xor(b2, off);
      if (j == 0) pr[H * D + H + o0 + 4 * g + q] = b2;
    }
    // gW3 [k][H]: C rows = outputs 4 g + q (g == 0, q < k), col = z2 unit o0 + j
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < K) pr[H * D + 2 * H + q * H + o0 + j] = gw3[t][q];
    }
  }
  if (half == 0 && wave == 0) {
    float v = gb3;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off);
    if (j == 0 && g < K) pr[H * D + 2 * H + K * H + g] = v;
  }
}

// ------------------------------------------------------------------------------------------------ gW2
// gW2 [H][H] = gz2^T h1 per network: a workgroup takes a 128 x 128 output block (rows u of gW2 = gz2 columns,
// cols i = h1 columns) over a chunk of the mini-batch rows; 8 waves as 2 (u) x 4 (i) of 64 x 32 (4 x 2 tiles).
// The rows are staged 32 at a time, transposed into LDS ([col][row + 4]), so a fragment of 4 consecutive rows is
// one ds_read_b128 (k order: k step 4 s + r of a 16-row group s is row 16 s + 4 g + r).
constexpr int WG_BLK = 128;  // output block edge
constexpr int WG_R = 32;     // rows per LDS stage
constexpr int WG_RP = WG_R + 4;
constexpr size_t mlp_wgrad_lds_bytes() { return 4 * (size_t)2 * 2 * WG_BLK * WG_RP; }

template <int H>
__global__ __launch_bounds__(MW * 64) void mlp_wgrad(gr_mlp_args a, int splits, long long rows_per_split,
                                                     float* __restrict__ part) {
  constexpr int NB = H / WG_BLK;  // blocks per edge
  // XCD-aware: workgroup b runs on XCD b % 8; the NB * NB blocks of one (network, split) are b, b + 8, ... so they
  // share that XCD's L2 (each stage of rows is read by NB blocks)
  const int b = blockIdx.x, xcd = b & 7, q = b >> 3;
  const int blk = q % (NB * NB), grp = (q / (NB * NB)) * 8 + xcd;  // grp = net * splits + split
  const int net_i = grp / splits, split = grp % splits;
  if (net_i >= a.nets) return;
  const gr_mlp_net& net = a.net[net_i];
  const int bu = (blk / NB) * WG_BLK, bi = (blk % NB) * WG_BLK;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  const int wu = (wave >> 2) * 64, wi = (wave & 3) * 32;  // the wave's 64 x 32 sub-block
  extern __shared__ float lds[];
  const long long n = a.rows;
  const long long r_begin = (long long)split * rows_per_split;
  const long long r_end = r_begin + rows_per_split < n ? r_begin + rows_per_split : n;
  m4 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = zero4();
  // staging: 32 rows x 32 float4 per matrix = 16 units of 8 rows x 8 float4 (one wave instruction: 8 rows x 128
  // contiguous bytes; the transposed LDS writes of its 64 lanes then hit 32 distinct banks), 2 units per wave.
  // Split in two: the loads into registers are issued before the current stage's MFMAs, the transposed LDS writes
  // after them (so the loads' latency is covered by the MFMAs instead of stalling both waves of the SIMD)
  m4 sv[2][2];
  auto stage_load = [&](long long r0) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const float* src = m == 0 ? net.gz2 : net.h1;
      const int col0 = m == 0 ? bu : bi;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int unit = wave + MW * p;  // 0..15
        const int row = 8 * (unit & 3) + (lane & 7), c4 = 4 * (8 * (unit >> 2) + (lane >> 3));
        const long long r = r0 + row;
        sv[m][p] = r < r_end ? ld4(src + r * H + col0 + c4) : zero4();
      }
    }
  };
  auto stage_write = [&](float* dst) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      float* d = dst + m * WG_BLK * WG_RP;
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int unit = wave + MW * p;
        const int row = 8 * (unit & 3) + (lane & 7), c4 = 4 * (8 * (unit >> 2) + (lane >> 3));
#pragma unroll
        for (int e = 0; e < 4; ++e) d[(c4 + e) * WG_RP + row] = sv[m][p][e];
      }
    }
  };
  int buf = 0;
  if (r_begin < r_end) {
    stage_load(r_begin);
    stage_write(lds);
  }
  for (long long r0 = r_begin; r0 < r_end; r0 += WG_R) {
    __syncthreads();  // stage `buf` complete; the other buffer's readers are done
    float* cur = lds + buf * 2 * WG_BLK * WG_RP;
    const bool more = r0 + WG_R < r_end;
    if (more) stage_load(r0 + WG_R);
    const float* A = cur;                    // gz2 block, [u][row]
    const float* B = cur + WG_BLK * WG_RP;   // h1 block, [i][row]
#pragma unroll
    for (int s = 0; s < WG_R / 16; ++s) {
      m4 af[4], bf[2];
#pragma unroll
      for (int t = 0; t < 4; ++t) af[t] = ld4(A + (wu + 16 * t + j) * WG_RP + 16 * s + 4 * g);
#pragma unroll
      for (int u = 0; u < 2; ++u) bf[u] = ld4(B + (wi + 16 * u + j) * WG_RP + 16 * s + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int u = 0; u < 2; ++u) acc[t][u] = mf(af[t][r], bf[u][r], acc[t][u]);
    }
    if (more) stage_write(lds + (buf ^ 1) * 2 * WG_BLK * WG_RP);
    buf ^= 1;
  }
  // partial block -> part[net][split][H][H]
  float* pp = part + ((size_t)net_i * splits + split) * H * H;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int q2 = 0; q2 < 4; ++q2)
        pp[(size_t)(bu + wu + 16 * t + 4 * g + q2) * H + bi + wi + 16 * u + j] = acc[t][u][q2];
}

// ------------------------------------------------------------------------------------------------ reductions
// grads[net] = [gW1 (H D) | gb1 (H) | gW2 (H H) | gb2 (H) | gW3 (k H) | gb3 (k)]: element e of the vector is the
// fixed-order sum of its partials.  A lane owns 4 consecutive elements (float4 loads of the partial rows); the 4
// waves of a workgroup take every 4th partial row, 8 loads in flight per lane, and are summed in wave order.
// (The small gradients come from the backward's partial rows [gW1 | gb1 | gb2 | gW3 | gb3], the hidden weight
// gradient from mlp_wgrad's split partials.)
constexpr int MF_WAVES = 4;
__global__ __launch_bounds__(MF_WAVES * 64) void mlp_final(gr_mlp_args a, int bwd_rows, int bwd_ld, int splits,
                                                          const float* __restrict__ wpart) {
  __shared__ m4 sm[MF_WAVES * 64];
  const gr_mlp_net& net = a.net[blockIdx.y];
  const int H = a.hidden, D = net.d, K = net.k;
  const int n_small = H * D + 2 * H + K * H + K;
  const int q_small = (n_small + 3) / 4, q_total = q_small + H * H / 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int q = blockIdx.x * 64 + lane;  // the lane's float4 of the (padded) small part, then of gW2
  const float* src;
  int rows, ldr;
  if (q < q_small) {
    src = a.partial + (size_t)blockIdx.y * bwd_rows * bwd_ld + 4 * q;
    rows = bwd_rows;
    ldr = bwd_ld;
  } else if (q < q_total) {
    src = wpart + (size_t)blockIdx.y * splits * H * H + 4 * (q - q_small);
    rows = splits;
    ldr = H * H;
  } else {
    src = nullptr;
    rows = 0;
    ldr = 0;
  }
  m4 acc0 = zero4(), acc1 = zero4();
  if (src) {
    int b = wv;
    for (; b + 7 * MF_WAVES < rows; b += 8 * MF_WAVES) {
      m4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld4(src + (size_t)(b + u * MF_WAVES) * ldr);
#pragma unroll
      for (int u = 0; u < 8; u += 2) {
        acc0 += v[u];
        acc1 += v[u + 1];
      }
    }
    for (; b < rows; b += MF_WAVES) acc0 += ld4(src + (size_t)b * ldr);
  }
  sm[threadIdx.x] = acc0 + acc1;
  __syncthreads();
  if (wv == 0 && src) {
    m4 t = sm[lane];
#pragma unroll
    for (int w = 1; w < MF_WAVES; ++w) t += sm[w * 64 + lane];
    if (q < q_small) {
      // partial layout [gW1 | gb1 | gb2 | gW3 | gb3] -> grads [gW1 | gb1 | gW2 | gb2 | gW3 | gb3] (the boundary at
      // H D + H is a multiple of 4: a float4 lies on one side)
      const int e = 4 * q;
      const int out = e < H * D + H ? e : e + H * H;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (e + r < n_small) net.grads[out + r] = t[r];
    } else {
      const int f = 4 * (q - q_small);
#pragma unroll
      for (int r = 0; r < 4; ++r) net.grads[H * D + H + f + r] = t[r];
    }
  }
}

// ------------------------------------------------------------------------------------------------ launchers
static int mlp_grid_x(long long rows, int nets, int tile = ME) {
  const int t = (int)((rows + tile - 1) / tile), per = M_BLOCKS / nets;
  return t < per ? (t < 1 ? 1 : t) : per;
}
// gW2 split count: enough workgroups for every CU (nets x blocks x splits >= 256), rows per split a multiple of the
// stage, splits a multiple of 8 / (nets) so the XCD grouping is exact
static int mlp_splits(long long rows, int hidden, int nets) {
  const int nb = (hidden / WG_BLK) * (hidden / WG_BLK);
  int s = (M_BLOCKS + nets * nb - 1) / (nets * nb);
  const long long max_s = (rows + WG_R - 1) / WG_R;
  if (s > max_s) s = (int)max_s;
  if (s < 1) s = 1;
  // (nets * s) must be a multiple of 8 for the b -> (grp, blk) mapping: round up
  while ((nets * s) % 8) ++s;
  return s;
}
static long long mlp_rows_per_split(long long rows, int splits) {
  long long r = (rows + splits - 1) / splits;
  return (r + WG_R - 1) / WG_R * WG_R;
}

int64_t mlp_partial_floats(long long rows, int hidden, int nets, int max_d, int max_k) {
  const int bwd = mlp_grid_x(rows, nets, BE);
  const int row = mlp_bwd_row(hidden, max_d, max_k);
  const int s = mlp_splits(rows, hidden, nets);
  return (int64_t)nets * bwd * row + (int64_t)nets * s * hidden * hidden;
}

template <typename F>
static hipError_t set_lds(F* k, size_t bytes) {
  return hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <int H, int Q1>
static hipError_t launch_fwd_t(const gr_mlp_args& a, hipStream_t s) {
  static bool attr = false;
  const size_t lds = mlp_fwd_lds_bytes(H);
  if (!attr) {
    const hipError_t e = set_lds(&mlp_fwd<H, Q1>, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((mlp_fwd<H, Q1>), dim3(mlp_grid_x(a.rows, a.nets), a.nets), dim3(MW * 64), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_mlp_forward(const gr_mlp_args& a, hipStream_t s) {
  int d = a.net[0].d;
  if (a.nets > 1 && a.net[1].d > d) d = a.net[1].d;
  if (a.hidden == 256) return d <= 16 ? launch_fwd_t<256, 1>(a, s) : launch_fwd_t<256, 2>(a, s);
  return d <= 16 ? launch_fwd_t<128, 1>(a, s) : launch_fwd_t<128, 2>(a, s);
}

template <int H, int DT>
static hipError_t launch_bwd_t(const gr_mlp_args& a, int row, hipStream_t s) {
  static bool attr = false;
  const size_t lds = mlp_bwd_lds_bytes(H);
  if (!attr) {
    const hipError_t e = set_lds(&mlp_bwd<H, DT>, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((mlp_bwd<H, DT>), dim3(mlp_grid_x(a.rows, a.nets, BE), a.nets), dim3(MW * 64), lds, s, a, row);
  return hipGetLastError();
}

template <int DT>
static hipError_t launch_bwd256_t(const gr_mlp_args& a, int row, hipStream_t s) {
  static bool attr = false;
  const size_t lds = mlp_bwd256_lds_bytes(DT);
  if (!attr) {
    const hipError_t e = set_lds(&mlp_bwd256<DT>, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((mlp_bwd256<DT>), dim3(mlp_grid_x(a.rows, a.nets, BE), a.nets), dim3(MW * 64), lds, s, a, row);
  return hipGetLastError();
}

template <int DT>
static hipError_t launch_bwd256h_t(const gr_mlp_args& a, int row, hipStream_t s) {
  static bool attr = false;
  const size_t lds = mlp_bwd256h_lds_bytes(DT);
  if (!attr) {
    const hipError_t e = set_lds(&mlp_bwd256h<DT>, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL((mlp_bwd256h<DT>), dim3(2 * mlp_grid_x(a.rows, a.nets, BE), a.nets), dim3(HWV * 64), lds, s, a,
                     row);
  return hipGetLastError();
}

template <int H>
static hipError_t launch_wgrad_t(const gr_mlp_args& a, int splits, long long rps, float* wpart, hipStream_t s) {
  static bool attr = false;
  const size_t lds = mlp_wgrad_lds_bytes();
  if (!attr) {
    const hipError_t e = set_lds(&mlp_wgrad<H>, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int nb = (H / WG_BLK) * (H / WG_BLK);
  hipLaunchKernelGGL((mlp_wgrad<H>), dim3(a.nets * splits * nb), dim3(MW * 64), lds, s, a, splits, rps, wpart);
  return hipGetLastError();
}

hipError_t launch_mlp_backward(const gr_mlp_args& a, hipStream_t s) {
  int d = a.net[0].d, k = a.net[0].k;
  if (a.nets > 1) {
    d = a.net[1].d > d ? a.net[1].d : d;
    k = a.net[1].k > k ? a.net[1].k : k;
  }
  const int row = mlp_bwd_row(a.hidden, d, k);
  const int bwd_blocks = mlp_grid_x(a.rows, a.nets, BE);
  hipError_t e;
  const bool masks = a.net[0].h1mask && (a.nets < 2 || a.net[1].h1mask);
  if (a.hidden == 256 && masks) e = d <= 16 ? launch_bwd256h_t<1>(a, row, s) : launch_bwd256h_t<2>(a, row, s);
  else if (a.hidden == 256) e = d <= 16 ? launch_bwd256_t<1>(a, row, s) : launch_bwd256_t<2>(a, row, s);
  else e = d <= 16 ? launch_bwd_t<128, 1>(a, row, s) : launch_bwd_t<128, 2>(a, row, s);
  if (e != hipSuccess) return e;
  const int splits = mlp_splits(a.rows, a.hidden, a.nets);
  const long long rps = mlp_rows_per_split(a.rows, splits);
  float* wpart = a.partial + (size_t)a.nets * bwd_blocks * row;
  e = a.hidden == 256 ? launch_wgrad_t<256>(a, splits, rps, wpart, s) : launch_wgrad_t<128>(a, splits, rps, wpart, s);
  if (e != hipSuccess) return e;
  const int q_total = (a.hidden * d + 2 * a.hidden + k * a.hidden + k + 3) / 4 + a.hidden * a.hidden / 4;
  hipLaunchKernelGGL(mlp_final, dim3((q_total + 63) / 64, a.nets), dim3(MF_WAVES * 64), 0, s, a, bwd_blocks, row,
                     splits, (const float*)wpart);
  return hipGetLastError();
}

}  // namespace gr
