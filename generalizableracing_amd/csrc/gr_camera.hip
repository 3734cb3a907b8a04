// gr_camera.hip — the front depth camera (RayCasterCamera, distance_to_image_plane) and the
// depth_image observation term, for gfx950.
//
// Reference: racing_ctbr_env.py:77-95,141-160,390-391 and mdp/observation.py:65-94 (paths under
// extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/); the math lives in gr_camera.h,
// shared with the CPU oracle.
//
// One wave per env, four envs per 256-thread workgroup.  Everything an env's rays need is
// wave-uniform (camera pose, the gates of its track), so the per-gate setup runs once per wave
// (lane g sets gate g up into LDS) and the pixel loop reads the gate slots as LDS broadcasts.
// A lane owns a pixel quad (4 consecutive pixels of one row) of an 8x32 tile: 27 tiles at 96x72,
// each store 8 full 128-byte row segments.  Waves whose sensor is not outdated skip the ray cast and
// read the persistent depth buffer instead (the Isaac Lab sensor renders every
// ceil(update_period / step_dt) steps and on reset).  Both obs rows are written every call:
// [16 state terms | image], the policy image with fresh multiplicative noise.
#include "gr_camera.h"
#include "gr_kernels.h"
#include "gr_normal_table.h"

namespace gr {

static_assert(CAM_NORMAL_FLOATS == 4 * GR_NORMAL_TABLE_ENTRIES && GR_NORMAL_TABLE_ENTRIES % 64 == 0,
              "normal table size (gr_kernels.h)");
// the image noise's inverse-CDF table (gr_rng.h gr_normal24); each workgroup copies it into LDS
__constant__ __attribute__((aligned(16))) float cam_normal_tab[4 * GR_NORMAL_TABLE_ENTRIES] = GR_NORMAL_TABLE_INIT;

#define DEV_INLINE __device__ __forceinline__

typedef float gr_v4f __attribute__((ext_vector_type(4)));
// streaming store: the obs rows (2 x 27.7 KB per env) are not re-read by this kernel
DEV_INLINE void nt_store4(float4* p, float4 v) {
  const gr_v4f x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<gr_v4f*>(p));
}

#define CAM_SLOT4 (GR_CAM_SLOT / 4)
static_assert(GR_CAM_SLOT == GR_CAM_GATE_SLOT, "gate slot size (gr_camera.h / gr_kernels.h)");
#ifndef CAM_BATCH
// reuse path: depth quads loaded per lane before any is consumed (27 = 14 + 13 at 96x72).  14 against 9: obstacle
// reuse 1.271 -> 1.253 ms, gate-only 1.129 -> 1.114 ms, two alternations on one box (gpurun_out/r6m); the obstacle
// kernel's VGPRs unchanged (98, its render path), the gate-only kernel's 69 -> 94 (7 -> 5 waves per SIMD)
#define CAM_BATCH 14
#endif

// both observation rows of one pixel quad: fresh noise (quad index q), normalisation, streaming stores
DEV_INLINE void emit_quad(const CamArgs& a, const gr_cam_const* __restrict__ cc, const float* ntab, float4* op4,
                          float4* oc4, int q, float4 d4, uint32_t gid, uint32_t cnt) {
  const float scale = cc->obs_scale, inv = cc->inv_obs_scale, nstd = cc->noise_std;
  float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (cc->add_noise) gr_cam_noise4(gid, cnt, (uint32_t)q, a.seed_lo, a.seed_hi, ntab, z);
  float4 op, oc;
  op.x = gr_cam_obs(d4.x, z[0], nstd, scale, inv); oc.x = gr_cam_obs_clean(d4.x, scale, inv);
  op.y = gr_cam_obs(d4.y, z[1], nstd, scale, inv); oc.y = gr_cam_obs_clean(d4.y, scale, inv);
  op.z = gr_cam_obs(d4.z, z[2], nstd, scale, inv); oc.z = gr_cam_obs_clean(d4.z, scale, inv);
  op.w = gr_cam_obs(d4.w, z[3], nstd, scale, inv); oc.w = gr_cam_obs_clean(d4.w, scale, inv);
  nt_store4(op4 + q, op);
  nt_store4(oc4 + q, oc);
}

DEV_INLINE void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the 16 state terms of both rows
DEV_INLINE void state_terms(const CamArgs& a, int i, int lane, size_t row) {
  if (lane < 4) {
    const float4 sp = reinterpret_cast<const float4*>(a.obs_p16)[4 * i + lane];
    const float4 sc = reinterpret_cast<const float4*>(a.obs_c16)[4 * i + lane];
    reinterpret_cast<float4*>(a.out_p + i * row)[lane] = sp;
    reinterpret_cast<float4*>(a.out_c + i * row)[lane] = sc;
  }
}

// sensor up to date: stream the depth buffer into both rows, CAM_BATCH loads in flight per lane
DEV_INLINE void reuse_rows(const CamArgs& a, const gr_cam_const* __restrict__ cc, const float* ntab, const float4* dep4,
                           float4* op4, float4* oc4, int nq, int lane, uint32_t gid, uint32_t cnt) {
  for (int q0 = 0; q0 < nq; q0 += 64 * CAM_BATCH) {
    float4 dd[CAM_BATCH];
#pragma unroll
    for (int j = 0; j < CAM_BATCH; ++j) {
      const int q = q0 + 64 * j + lane;
      dd[j] = q < nq ? dep4[q] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < CAM_BATCH; ++j) {
      const int q = q0 + 64 * j + lane;
      if (q < nq) emit_quad(a, cc, ntab, op4, oc4, q, dd[j], gid, cnt);
    }
  }
}

// obstacle slot from LDS (GR_CAM_OSLOT floats: frame, primitive and kind = slot floats 0-15, what the hit and frustum
// tests read; the window's pixel rectangle, read by the tile masks and hit passes, is a packed word beside the slots)
DEV_INLINE void load_oslot(const float4* src, float s[GR_CAM_SLOT]) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 q4 = src[k];
    s[4 * k] = q4.x; s[4 * k + 1] = q4.y; s[4 * k + 2] = q4.z; s[4 * k + 3] = q4.w;
  }
}

// the obstacle's record from global memory
DEV_INLINE void load_orec(const float* rec, float r[GR_OBST_FLOATS]) {
  const float4* r4 = reinterpret_cast<const float4*>(rec);
#pragma unroll
  for (int k = 0; k < GR_OBST_FLOATS / 4; ++k) {
    const float4 v = r4[k];
    r[4 * k] = v.x; r[4 * k + 1] = v.y; r[4 * k + 2] = v.z; r[4 * k + 3] = v.w;
  }
}

// the pixel range {i : lo <= r[i] <= hi} of a decreasing ray table r[0 .. n) (a_u over u, b_v over v): [first, last],
// empty when first > last.  Exactly the pixels a window test r[i] >= lo && r[i] <= hi admits
DEV_INLINE void window_pixels(const float* __restrict__ r, int n, float lo, float hi, int& first, int& last) {
  int a = 0, b = n;  // first i with r[i] <= hi
  while (a < b) {
    const int m = (a + b) >> 1;
    if (r[m] <= hi) b = m; else a = m + 1;
  }
  first = a;
  a = 0;
  b = n;  // first i with r[i] < lo
  while (a < b) {
    const int m = (a + b) >> 1;
    if (r[m] < lo) b = m; else a = m + 1;
  }
  last = a - 1;
}

// nearest obstacle crossing of the tile quad's four rays against one set-up slot
DEV_INLINE void quad_obst(const float* s, const float av[4], float b, float d[4]) {
  // a_u decreases with u: the quad spans [av[3], av[0]]
  if (b >= s[GR_CS_BMIN] && b <= s[GR_CS_BMAX] && av[3] <= s[GR_CS_AMAX] && av[0] >= s[GR_CS_AMIN]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (av[j] >= s[GR_CS_AMIN] && av[j] <= s[GR_CS_AMAX]) d[j] = gr_minf(d[j], gr_cam_obst_hit(s, av[j], b));
  }
}

// Dynamic LDS: the normal table (workgroup), ray tables a_u[W], b_v[H] (padded to 4), then per wave: gate slots
// [max_gates][36] and their tile masks, on obstacle tracks a.obst_slots obstacle slots of 16 floats, their pixel
// rectangles and tile masks, and an 8-row depth staging band [8][W] (camera_launch_config, gr_kernels.h).
#ifdef CAM_WAVES_PER_EU
#define CAM_ATTR __attribute__((amdgpu_waves_per_eu(CAM_WAVES_PER_EU, CAM_WAVES_PER_EU)))
#else
#define CAM_ATTR
#endif
// OBST: the track carries obstacles (a separate instantiation, so the gate-only kernel keeps its code)
template <bool OBST>
__global__ __launch_bounds__(CAM_WAVES * 64) CAM_ATTR void camera_kernel(CamArgs a) {
  extern __shared__ float4 smem4[];
  float* smem = reinterpret_cast<float*>(smem4);  // [normal table | ray tables | per-wave slots]
  const gr_cam_const* __restrict__ cc = a.cc;
  const int W = a.width, H = a.height, npix = W * H, G = a.max_gates;
  const int wpad = (W + 3) & ~3, hpad = (H + 3) & ~3;
  constexpr int nw = CAM_WAVES;
  const int S = OBST ? a.obst_slots : 0;  // obstacle slots per wave
  // the normal table in LDS, shared by the workgroup's waves (read from the constant segment instead, a gate-only
  // re-render measured 1.20 -> 1.41 ms: a per-pixel gather through the vector cache, gpurun_out/r6x)
  {
    float4* s_ntab4 = smem4;
    for (int k = threadIdx.x; k < GR_NORMAL_TABLE_ENTRIES; k += nw * 64)
      s_ntab4[k] = reinterpret_cast<const float4*>(cam_normal_tab)[k];
  }
  const float* s_ntab = smem;
  smem += CAM_NORMAL_FLOATS;
  float* s_ray_a = smem;
  float* s_ray_b = smem + wpad;
  for (int k = threadIdx.x; k < W; k += nw * 64) s_ray_a[k] = cc->ray_a[k];
  for (int k = threadIdx.x; k < H; k += nw * 64) s_ray_b[k] = cc->ray_b[k];
  __syncthreads();  // (the only workgroup barrier: everything after it is per wave)

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x * nw + w;
  const bool active = i < a.num_envs;
  const int N = a.num_envs;
  constexpr bool obst = OBST;
  const int ntx = (W + 31) / 32, nty = (H + 7) / 8;
  const int oslots = (int)camera_obst_floats(W, H, S);
  const int tmf = (int)camera_tile_mask_floats(W, H);
  float* wave_lds = smem + wpad + hpad + w * (int)camera_wave_floats(W, H, G, S);
  float4* s_slot = reinterpret_cast<float4*>(wave_lds);                               // [G][CAM_SLOT4]
  uint64_t* s_gmask = reinterpret_cast<uint64_t*>(wave_lds + G * GR_CAM_SLOT);        // [tiles]
  float* olds = wave_lds + G * GR_CAM_SLOT + tmf;
  float4* s_oslot = reinterpret_cast<float4*>(olds);                                  // [slots][GR_CAM_OSLOT / 4]
  // per slot: its window's pixel rectangle u_lo | u_hi << 8 | v_lo << 16 | v_hi << 24 (W, H <= 256)
  uint32_t* s_orect = reinterpret_cast<uint32_t*>(olds + S * GR_CAM_OSLOT);
  uint64_t* s_tmask = reinterpret_cast<uint64_t*>(olds + S * GR_CAM_OSLOT + ((S + 3) & ~3));  // [tiles]
  float4* s_stage = reinterpret_cast<float4*>(olds + oslots);                         // [8 * W / 4]

  // ---- is the sensor outdated? (SensorBase.update / reset; wave-uniform)
  int render = 0;
  if (active) {
    const int age = a.age[i];
    int outdated = age < 0;
    int aged = age < 0 ? 0 : age;
    if (a.mode == GR_CAM_STEP) {
      const int rst = (a.terminated[i] | a.time_out[i]) != 0;
      aged = aged + 1;
      outdated = outdated || rst || aged >= cc->period_steps;
    } else if (a.mode == GR_CAM_RESET) {
      outdated = outdated || a.mask == nullptr || a.mask[i] != 0;
    }
    render = __builtin_amdgcn_readfirstlane(outdated);
    if (lane == 0) a.age[i] = render ? 0 : aged;
  }

  // ---- camera pose and the gate slots of this env's track
  float o[3] = {0.0f, 0.0f, 0.0f}, c0[3] = {1.0f, 0.0f, 0.0f}, c1[3] = {0.0f, 1.0f, 0.0f},
        c2[3] = {0.0f, 0.0f, 1.0f};
  float gz = 0.0f;
  uint64_t valid_mask = 0;
  const float* orecs = nullptr;  // this track's obstacle records
  int nob = 0, ofrom = 0;         // obstacles in the track; raw index of the first one beyond the slots
  int ns = 0;                     // obstacle slots in LDS
  if (render) {
    const float4 posq = reinterpret_cast<const float4*>(a.state)[(size_t)GR_P_POSQ * N + i];
    const float4 qv = reinterpret_cast<const float4*>(a.state)[(size_t)GR_P_QV * N + i];
    const float p[3] = {posq.x, posq.y, posq.z}, q[4] = {posq.w, qv.x, qv.y, qv.z};
    gr_cam_pose(cc, p, q, o, c0, c1, c2);
    const int packed = a.istate[4 * i + GR_I_PACKED];
    const int track = ((packed >> 24) & 0xff) * a.num_levels + ((packed >> 8) & 0xff);
    const float* tb = a.table + (size_t)track * a.track_stride;
    const float* rec = tb + G * GR_GATE_FLOATS;
    gz = rec[0];
    const int ng = (int)rec[3];
    float s[GR_CAM_SLOT];
    int valid = 0;
    if (lane < ng) {
      gr_cam_gate_setup(tb + lane * GR_GATE_FLOATS, o, c0, c1, c2, cc->max_distance, s);
      valid = s[GR_CS_VALID] != 0.0f;
#pragma unroll
      for (int k = 0; k < CAM_SLOT4; ++k)
        s_slot[lane * CAM_SLOT4 + k] = make_float4(s[4 * k], s[4 * k + 1], s[4 * k + 2], s[4 * k + 3]);
    }
    valid_mask = __ballot(valid);
    if constexpr (obst) {
      // obstacles in view: the first S go to LDS slots (compacted by ballot); from the
      // next one on (rare) they are set up again per tile
      nob = a.obst_counts[track];
      orecs = a.obst + (size_t)track * a.max_obst * GR_OBST_FLOATS;
      ofrom = nob;
      int nv = 0;
      for (int base = 0; base < nob; base += 64) {
        const int k = base + lane;
        int ok = 0, u_lo = 0, u_hi = -1, v_lo = 0, v_hi = -1;
        if (k < nob) {
          float r[GR_OBST_FLOATS];
          load_orec(orecs + (size_t)k * GR_OBST_FLOATS, r);
          gr_cam_obst_setup(r, o, c0, c1, c2, cc->max_distance, s);
          ok = s[GR_CS_VALID] != 0.0f;
          if (ok) {
            // the window as the pixel rectangle it admits (a_u, b_v monotonic): the tile masks and the hit passes
            // read it instead of testing rays; a window between pixel rays can be hit by none (dropped)
            window_pixels(s_ray_a, W, s[GR_CS_AMIN], s[GR_CS_AMAX], u_lo, u_hi);
            window_pixels(s_ray_b, H, s[GR_CS_BMIN], s[GR_CS_BMAX], v_lo, v_hi);
            ok = u_lo <= u_hi && v_lo <= v_hi;
          }
        }
        const uint64_t b = __ballot(ok);
        const int pos = nv + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        if (ok && pos < S) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            s_oslot[pos * (GR_CAM_OSLOT / 4) + q] = make_float4(s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]);
          s_orect[pos] = (uint32_t)u_lo | (uint32_t)u_hi << 8 | (uint32_t)v_lo << 16 | (uint32_t)v_hi << 24;
        }
        const int nb = __popcll(b);
        if (nv + nb > S && ofrom == nob) {
          // raw index of valid obstacle number S (wave-uniform)
          const uint64_t over = __ballot(ok && pos == S);
          ofrom = base + __builtin_ctzll(over);
        }
        nv += nb;
      }
      ns = nv < S ? nv : S;
    }
    // per 8x32 tile: the gates and obstacle slots whose window meets the tile's ray range (a_u, b_v decrease
    // with u, v) and whose bounding box reaches into the tile's frustum (gr_cam_gate_outside / _obst_outside)
    wave_lds_sync();
    for (int tl = lane; tl < ntx * nty; tl += 64) {
      const int v0 = 8 * (tl / ntx), u0 = 32 * (tl % ntx);
      const int v1 = (v0 + 7 < H ? v0 + 7 : H - 1), u1 = (u0 + 31 < W ? u0 + 31 : W - 1);
      const float a_hi = s_ray_a[u0], a_lo = s_ray_a[u1], b_hi = s_ray_b[v0], b_lo = s_ray_b[v1];
      uint64_t gm = 0;
      for (uint64_t m = valid_mask; m; m &= m - 1) {
        const int g = __builtin_ctzll(m);
        float sg[GR_CAM_SLOT];
#pragma unroll
        for (int k = 0; k < CAM_SLOT4; ++k) {
          const float4 q4 = s_slot[g * CAM_SLOT4 + k];
          sg[4 * k] = q4.x; sg[4 * k + 1] = q4.y; sg[4 * k + 2] = q4.z; sg[4 * k + 3] = q4.w;
        }
        const bool meet = !(sg[GR_CS_AMAX] < a_lo || sg[GR_CS_AMIN] > a_hi || sg[GR_CS_BMAX] < b_lo ||
                            sg[GR_CS_BMIN] > b_hi) && !gr_cam_gate_outside(sg, a_lo, a_hi, b_lo, b_hi);
        gm |= (uint64_t)meet << g;
      }
      s_gmask[tl] = gm;
    }
    if constexpr (obst) {
      // the obstacle slots' tile masks on all 64 lanes when the image has <= 32 tiles (27 at 96 x 72): lane (h, tile)
      // tests slots h, h + 2, ... of its tile, then the two halves' masks are OR-ed (a lane per tile left 37 of 64
      // lanes idle through the longest loop of the set-up)
      const int ntiles = ntx * nty;
      const bool split = ntiles <= 32;
      const int kstep = split ? 2 : 1;
      for (int t0 = split ? (lane & 31) : lane; t0 < (split ? 32 : ntiles); t0 += 64) {
        const int tl = t0, k0 = split ? (lane >> 5) : 0;
        uint64_t tm = 0;
        if (tl < ntiles) {
          const int v0 = 8 * (tl / ntx), u0 = 32 * (tl % ntx);
          const int v1 = (v0 + 7 < H ? v0 + 7 : H - 1), u1 = (u0 + 31 < W ? u0 + 31 : W - 1);
          const float a_hi = s_ray_a[u0], a_lo = s_ray_a[u1], b_hi = s_ray_b[v0], b_lo = s_ray_b[v1];
          for (int k = k0; k < ns; k += kstep) {
            const uint32_t wk = s_orect[k];  // pixel rectangle u_lo, u_hi, v_lo, v_hi
            bool meet = !((int)(wk >> 8 & 0xffu) < u0 || (int)(wk & 0xffu) > u1 || (int)(wk >> 24) < v0 ||
                          (int)(wk >> 16 & 0xffu) > v1);
            if (meet) {
              float sk[GR_CAM_SLOT];
              load_oslot(s_oslot + k * (GR_CAM_OSLOT / 4), sk);
              meet = !gr_cam_obst_outside(sk, a_lo, a_hi, b_lo, b_hi);
            }
            tm |= (uint64_t)meet << k;
          }
        }
        if (split) {  // (every lane: the shuffles are wave-wide)
          const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)tm, 32);
          const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(tm >> 32), 32);
          tm |= ((uint64_t)hi << 32) | lo;
          if (lane < 32 && tl < ntiles) s_tmask[tl] = tm;
        } else if (tl < ntiles) {
          s_tmask[tl] = tm;
        }
      }
    }
  }
  wave_lds_sync();  // (this wave's slots and masks)
  if (!active) return;

  const uint32_t gid = (uint32_t)(a.env_id_offset + i);
  const uint32_t cnt = a.counters[a.counter_index];
  const size_t row = (size_t)(16 + npix);
  state_terms(a, i, lane, row);
  float4* op4 = reinterpret_cast<float4*>(a.out_p + i * row + 16);
  float4* oc4 = reinterpret_cast<float4*>(a.out_c + i * row + 16);
  float4* dep4 = reinterpret_cast<float4*>(a.depth + (size_t)i * npix);
  const int nq = npix >> 2;

  if (!render) {
    const float* ntab = s_ntab;
    reuse_rows(a, cc, ntab, dep4, op4, oc4, nq, lane, gid, cnt);
    return;
  }

  // ---- render: bands of 8 image rows.  Rays are cast in 8x32 tiles (a lane owns a quad of one tile
  // row), so a gate's screen window culls whole tiles; the band is staged in LDS and written out in
  // row-major order (full, contiguous 1 KB stores per wave instruction).
  const float maxd = cc->max_distance;
  for (int v0 = 0; v0 < H; v0 += 8) {
    const int rows = H - v0 < 8 ? H - v0 : 8;
    for (int u_t = 0; u_t < W; u_t += 32) {
      const int v = v0 + (lane >> 3), u0 = u_t + 4 * (lane & 7);
      if (v >= H || u0 >= W) continue;
      const float b = s_ray_b[v];
      const float4 a4 = *reinterpret_cast<const float4*>(&s_ray_a[u0]);
      const float av[4] = {a4.x, a4.y, a4.z, a4.w};
      float d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float dz = gr_fmaf(b, c2[2], gr_fmaf(av[j], c1[2], c0[2]));
        d[j] = gr_cam_ground_hit(o[2], gz, dz);
      }
      uint64_t m = s_gmask[(v0 >> 3) * ntx + (u_t >> 5)];
      while (m) {
        const int g = __builtin_ctzll(m);
        m &= m - 1;
        float s[GR_CAM_SLOT];
#pragma unroll
        for (int k = 0; k < CAM_SLOT4; ++k) {
          const float4 q4 = s_slot[g * CAM_SLOT4 + k];
          s[4 * k] = q4.x; s[4 * k + 1] = q4.y; s[4 * k + 2] = q4.z; s[4 * k + 3] = q4.w;
        }
        if (b >= s[GR_CS_BMIN] && b <= s[GR_CS_BMAX] && av[3] <= s[GR_CS_AMAX] && av[0] >= s[GR_CS_AMIN]) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (av[j] >= s[GR_CS_AMIN] && av[j] <= s[GR_CS_AMAX]) d[j] = gr_minf(d[j], gr_cam_gate_hit(s, av[j], b));
        }
      }
      if constexpr (obst) {
        for (int k = ofrom; k < nob; ++k) {  // beyond the slots: set up again (identical slot values)
          float r[GR_OBST_FLOATS], s[GR_CAM_SLOT];
          load_orec(orecs + (size_t)k * GR_OBST_FLOATS, r);
          gr_cam_obst_setup(r, o, c0, c1, c2, maxd, s);
          if (s[GR_CS_VALID] != 0.0f) quad_obst(s, av, b, d);
        }
      }
      s_stage[((v - v0) * W + u0) >> 2] =
          make_float4(gr_cam_clip(d[0], maxd), gr_cam_clip(d[1], maxd), gr_cam_clip(d[2], maxd), gr_cam_clip(d[3], maxd));
    }
    if constexpr (obst) {
      // the obstacles of the LDS slots, per tile of the band: only the pixels inside a slot's window (a column
      // range times a row range: a_u and b_v are monotonic), packed onto the lanes across slots and tiles of
      // the band (one hit per lane and batch of 64 pixels) and min-ed into the staged band (clip(min) =
      // min(clip): the clip is monotonic). Two slots of one batch may share a pixel, so the min is an LDS
      // integer atomic: a hit is > 0 and never NaN, the staged depth is clipped (not NaN), so the signed
      // order of the bit patterns is the float order of the pairs compared and the result is the sequential
      // min's bits whatever the order
      int* sti = reinterpret_cast<int*>(s_stage);
      int fill = 0;                      // lanes holding a pixel of the current batch (wave-uniform)
      int my_k = 0, my_u = 0, my_r = 0;  // this lane's slot, column and band row
      auto batch = [&](int nfill) {
        if (lane < nfill) {
          float s[GR_CAM_SLOT];
          load_oslot(s_oslot + my_k * (GR_CAM_OSLOT / 4), s);
          const float h = gr_cam_clip(gr_cam_obst_hit(s, s_ray_a[my_u], s_ray_b[v0 + my_r]), maxd);
          __hip_atomic_fetch_min(sti + my_r * W + my_u, __float_as_int(h), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
      };
      wave_lds_sync();
      for (int u_t = 0; u_t < W; u_t += 32) {
        uint64_t mo = s_tmask[(v0 >> 3) * ntx + (u_t >> 5)];
        while (mo) {
          const int k = __builtin_ctzll(mo);
          mo &= mo - 1;
          // the slot's pixel rectangle within this tile of the band (wave-uniform integer ranges)
          const uint32_t wk = s_orect[k];
          const int ulo = (int)(wk & 0xffu), uhi = (int)(wk >> 8 & 0xffu), vlo = (int)(wk >> 16 & 0xffu),
                    vhi = (int)(wk >> 24);
          const int cu = ulo > u_t ? ulo : u_t, cu1 = uhi < u_t + 31 ? uhi : u_t + 31;
          const int rv = (vlo > v0 ? vlo : v0) - v0, rv1 = (vhi < v0 + 7 ? vhi : v0 + 7) - v0;
          if (cu > cu1 || rv > rv1) continue;
          const int wc = cu1 - cu + 1, area = wc * (rv1 - rv + 1);
          // (idx / wc below exact for idx < 256, wc <= 32 with a 1-ulp reciprocal: see the 1e-3 margin)
          const float inv_wc = __builtin_amdgcn_rcpf((float)wc);
          for (int done = 0; done < area;) {
            const int take = area - done < 64 - fill ? area - done : 64 - fill;
            if (lane >= fill && lane < fill + take) {
              // idx / wc exactly for idx < 256, wc <= 32 (the fraction of a non-integer quotient is <= 31/32)
              const int idx = done + lane - fill;
              const int r = (int)((float)idx * inv_wc + 1.0e-3f);
              my_k = k;
              my_u = cu + idx - r * wc;
              my_r = rv + r;
            }
            fill += take;
            done += take;
            if (fill == 64) {
              batch(64);
              fill = 0;
            }
          }
        }
      }
      if (fill) batch(fill);
    }
    wave_lds_sync();
    const int qb = (v0 * W) >> 2, nqb = (rows * W) >> 2;
    for (int qq = lane; qq < nqb; qq += 64) {
      const float4 d4 = s_stage[qq];
      nt_store4(dep4 + qb + qq, d4);
      emit_quad(a, cc, s_ntab, op4, oc4, qb + qq, d4, gid, cnt);
    }
    wave_lds_sync();
  }
}

template <bool OBST>
static hipError_t camera_launch_t(const CamArgs& b, const CamLaunch& L, hipStream_t s) {
  if (L.lds > (size_t)CAM_LDS_PER_CU) return hipErrorInvalidValue;
  static bool attr = false;  // (dynamic LDS above 64 KB: many gates)
  if (L.lds > 65536 && !attr) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&camera_kernel<OBST>),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, CAM_LDS_PER_CU);
    if (e != hipSuccess) return e;
    attr = true;
  }
  hipLaunchKernelGGL(camera_kernel<OBST>, dim3((b.num_envs + L.waves - 1) / L.waves), dim3(L.waves * 64), L.lds, s, b);
  return hipGetLastError();
}

hipError_t launch_camera(const CamArgs& a, hipStream_t s) {
  const bool obst = a.obst != nullptr;
  const CamLaunch L = camera_launch_config(a.width, a.height, a.max_gates, obst, obst ? a.obst_slots : 0);
  CamArgs b = a;
  b.obst_slots = L.slots;
  return obst ? camera_launch_t<true>(b, L, s) : camera_launch_t<false>(b, L, s);
}

}  // namespace gr
