// gr_kernels.hip — fused racing-env step for MI355X (gfx950, CDNA4).
//
// One lane per env, 256-lane workgroups (4 wave64).  Env state is
// struct-of-float4-planes in HBM (GR_P_* in include/gr.h): every field group
// is one coalesced 16-B-per-lane load / store (1 KiB per wave instruction).
// The gate geometry of the tracks a workgroup's envs can reference (its
// terrain-type range x all levels) is staged into LDS once per launch.
//
// Kernel == the reference step (manager_based_diff_rl_env.py:160-267) in the
// reference's op order, bit-identical to oracle/gr_oracle.c (built with
// -ffp-contract=off and the shared gr_math.h / gr_rng.h).  Reset is mask-based
// and in-lane: no host synchronisation, hipGraph-capturable.
#include <hip/hip_runtime.h>

#include "../../include/gr.h"
#include "gr_kernels.h"
#include "gr_normal_table.h"
#include "gr_math.h"
#include "gr_obstacles.h"
#include "gr_rng.h"

namespace gr {

// the observation noise's inverse-CDF normals (gr_rng.h gr_normal21; gr_normal_table.h)
__constant__ __attribute__((aligned(16))) float obs_normal_tab[4 * GR_NORMAL_TABLE_ENTRIES] = GR_NORMAL_TABLE_INIT;

#define DEV __device__ __forceinline__

// 16-byte stores of the step's outputs (state planes, istate, obs rows).  GR_STORE_POLICY: 0 plain;
// 1 non-temporal (`nt`, the default: the step's ~19 MB of outputs are not re-read by this launch);
// 2 write-through (`sc1`, buffer store on the uniform base); 3 `sc1 nt`.  `base` must be wave-uniform (a kernel-argument pointer).
#ifndef GR_STORE_POLICY
#define GR_STORE_POLICY 1  // nt measured 0.8 us (7 %) faster per step than plain; sc1 and nt loads slower
#endif
#ifndef GR_SCALAR_NT
#define GR_SCALAR_NT 1  // nt for the scalar outputs as well (measured 0.1 us faster)
#endif
template <typename T>
DEV void st1(T* p, T v) {  // the per-env scalar outputs (reward, flags, dones, aux)
#if GR_SCALAR_NT
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}
// 16-byte loads of planes only the physics waves read (GR_LOAD_POLICY 1: non-temporal).
#ifndef GR_LOAD_POLICY
#define GR_LOAD_POLICY 0
#endif
DEV float4 ld4(const float4* base, size_t idx) {
#if GR_LOAD_POLICY == 1
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4 w = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(base) + idx);
  return make_float4(w[0], w[1], w[2], w[3]);
#else
  return base[idx];
#endif
}
// GR_STATE_STORE_POLICY: the same choice for the state planes and istate alone (the only outputs the next step
// re-reads, on the same XCD: workgroup b runs on XCD b % 8 in every launch).
#ifndef GR_STATE_STORE_POLICY
#define GR_STATE_STORE_POLICY GR_STORE_POLICY
#endif
template <int POL = GR_STORE_POLICY, typename T4>
DEV void st4(T4* base, size_t idx, const T4& v) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 w = {__builtin_bit_cast(unsigned, v.x), __builtin_bit_cast(unsigned, v.y),
                   __builtin_bit_cast(unsigned, v.z), __builtin_bit_cast(unsigned, v.w)};
  if constexpr (POL == 1) {
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(base) + idx);
  } else if constexpr (POL >= 2) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(w, r, (int)(idx * 16), 0, POL == 2 ? 16 : 18);
  } else {
    *reinterpret_cast<u32x4*>(base + idx) = w;
  }
}
template <typename T4>
DEV void st4s(T4* base, size_t idx, const T4& v) {  // state planes and istate
  st4<GR_STATE_STORE_POLICY>(base, idx, v);
}

// ------------------------------------------------------------- IL math
// Isaac Lab omni.isaac.lab.utils.math restated (see oracle/gr_oracle.c).
DEV void quat_rotate(const float q[4], const float v[3], float o[3]) {
  float s = 2.0f * (q[0] * q[0]) - 1.0f;
  float cx = q[2] * v[2] - q[3] * v[1];
  float cy = q[3] * v[0] - q[1] * v[2];
  float cz = q[1] * v[1] - q[2] * v[0];
  float d = (q[1] * v[0] + q[2] * v[1]) + q[3] * v[2];
  o[0] = (v[0] * s + (cx * q[0]) * 2.0f) + (q[1] * d) * 2.0f;
  o[1] = (v[1] * s + (cy * q[0]) * 2.0f) + (q[2] * d) * 2.0f;
  o[2] = (v[2] * s + (cz * q[0]) * 2.0f) + (q[3] * d) * 2.0f;
}
DEV void quat_rotate_inverse(const float q[4], const float v[3], float o[3]) {
  float s = 2.0f * (q[0] * q[0]) - 1.0f;
  float cx = q[2] * v[2] - q[3] * v[1];
  float cy = q[3] * v[0] - q[1] * v[2];
  float cz = q[1] * v[1] - q[2] * v[0];
  float d = (q[1] * v[0] + q[2] * v[1]) + q[3] * v[2];
  o[0] = (v[0] * s - (cx * q[0]) * 2.0f) + (q[1] * d) * 2.0f;
  o[1] = (v[1] * s - (cy * q[0]) * 2.0f) + (q[2] * d) * 2.0f;
  o[2] = (v[2] * s - (cz * q[0]) * 2.0f) + (q[3] * d) * 2.0f;
}
DEV void quat_mul(const float a[4], const float b[4], float o[4]) {
  float ww = (a[3] + a[1]) * (b[1] + b[2]);
  float yy = (a[0] - a[2]) * (b[0] + b[3]);
  float zz = (a[0] + a[2]) * (b[0] - b[3]);
  float xx = (ww + yy) + zz;
  float qq = 0.5f * (xx + (a[3] - a[1]) * (b[1] - b[2]));
  o[0] = (qq - ww) + (a[3] - a[2]) * (b[2] - b[3]);
  o[1] = (qq - xx) + (a[1] + a[0]) * (b[1] + b[0]);
  o[2] = (qq - yy) + (a[0] - a[1]) * (b[2] + b[3]);
  o[3] = (qq - zz) + (a[3] + a[2]) * (b[0] - b[1]);
}
// sin / cos with a wave-uniform fast path: when every lane's |x| < pi/4 the Cody-Waite reduction is the
// identity (k = 0, r = x exactly), so skipping it gives the same bits as gr_sincosf
DEV void sincos_w(float x, float* s, float* c) {
  if (__all(gr_fabsf(x) < 0.78f)) {
    const float r2 = x * x;
    float sp = 2.75573192e-06f;
    sp = gr_fmaf(sp, r2, -1.98412698e-04f);
    sp = gr_fmaf(sp, r2, 8.33333333e-03f);
    sp = gr_fmaf(sp, r2, -1.66666667e-01f);
    *s = gr_fmaf(x, r2 * sp, x);
    float cp = -2.75573192e-07f;
    cp = gr_fmaf(cp, r2, 2.48015873e-05f);
    cp = gr_fmaf(cp, r2, -1.38888889e-03f);
    cp = gr_fmaf(cp, r2, 4.16666667e-02f);
    cp = gr_fmaf(cp, r2, -0.5f);
    *c = gr_fmaf(r2, cp, 1.0f);
    return;
  }
  gr_sincosf(x, s, c);
}
DEV void quat_from_euler_xyz(float roll, float pitch, float yaw, float o[4]) {
  float sy, cy, sr, cr, sp, cp;
  sincos_w(yaw * 0.5f, &sy, &cy);
  sincos_w(roll * 0.5f, &sr, &cr);
  sincos_w(pitch * 0.5f, &sp, &cp);
  o[0] = (cy * cr) * cp + (sy * sr) * sp;
  o[1] = (cy * sr) * cp - (sy * cr) * sp;
  o[2] = (cy * cr) * sp + (sy * sr) * cp;
  o[3] = (sy * cr) * cp - (cy * sr) * sp;
}
DEV void matrix_row2(const float q[4], float o[3]) {
  float two_s = 2.0f / (((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  o[0] = two_s * (q[1] * q[3] - q[2] * q[0]);
  o[1] = two_s * (q[2] * q[3] + q[1] * q[0]);
  o[2] = 1.0f - two_s * (q[1] * q[1] + q[2] * q[2]);
}
DEV void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
DEV float norm3(const float a[3]) { return gr_sqrtf((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]); }
DEV float cosine_similarity(const float a[3], const float b[3]) {
  float na = gr_maxf(norm3(a), 1e-8f), nb = gr_maxf(norm3(b), 1e-8f);
  return ((a[0] / na) * (b[0] / nb) + (a[1] / na) * (b[1] / nb)) + (a[2] / na) * (b[2] / nb);
}

// ------------------------------------------------------------- env registers
struct Env {
  float p[3], q[4], v[3], w[3], al[3], T, tau[3], lag[4];
  float thr, nl, k2[3], k1[3], es[7], mar;
  float Kp[3], cT, Kd[3], mp, ct[3], mc, J[3], mw[4];
  int ep, acc, epoch, gate, lvl, type, azero;
};

DEV void load_env(const KArgs& a, int i, Env& e) {
  // issue order = order of first use (the waitcnt counters retire in order)
  const float4* S = reinterpret_cast<const float4*>(a.buf.state);
  const size_t n = (size_t)a.h.num_envs;
  int4 ii = reinterpret_cast<const int4*>(a.buf.istate)[i];
  float4 s5 = ld4(S, GR_P_LAG * n + i), s6 = S[GR_P_RST0 * n + i], p2 = S[GR_P_PAR2 * n + i];
  float4 s2 = ld4(S, GR_P_VW * n + i), s3 = ld4(S, GR_P_WA * n + i), s4 = ld4(S, GR_P_CTRL * n + i);
  float4 p0 = ld4(S, GR_P_PAR0 * n + i), p1 = ld4(S, GR_P_PAR1 * n + i), p3 = ld4(S, GR_P_PAR3 * n + i);
  float4 s0 = ld4(S, GR_P_POSQ * n + i), s1 = ld4(S, GR_P_QV * n + i), s7 = S[GR_P_RST1 * n + i];
  float4 s8 = ld4(S, GR_P_EP0 * n + i), s9 = ld4(S, GR_P_EP1 * n + i);
  e.p[0] = s0.x; e.p[1] = s0.y; e.p[2] = s0.z; e.q[0] = s0.w;
  e.q[1] = s1.x; e.q[2] = s1.y; e.q[3] = s1.z; e.v[0] = s1.w;
  e.v[1] = s2.x; e.v[2] = s2.y; e.w[0] = s2.z; e.w[1] = s2.w;
  e.w[2] = s3.x; e.al[0] = s3.y; e.al[1] = s3.z; e.al[2] = s3.w;
  e.T = s4.x; e.tau[0] = s4.y; e.tau[1] = s4.z; e.tau[2] = s4.w;
  e.lag[0] = s5.x; e.lag[1] = s5.y; e.lag[2] = s5.z; e.lag[3] = s5.w;
  e.thr = s6.x; e.nl = s6.y; e.k2[0] = s6.z; e.k2[1] = s6.w;
  e.k2[2] = s7.x; e.k1[0] = s7.y; e.k1[1] = s7.z; e.k1[2] = s7.w;
  e.es[0] = s8.x; e.es[1] = s8.y; e.es[2] = s8.z; e.es[3] = s8.w;
  e.es[4] = s9.x; e.es[5] = s9.y; e.es[6] = s9.z; e.mar = s9.w;
  e.Kp[0] = p0.x; e.Kp[1] = p0.y; e.Kp[2] = p0.z; e.cT = p0.w;
  e.Kd[0] = p1.x; e.Kd[1] = p1.y; e.Kd[2] = p1.z; e.mp = p1.w;
  e.ct[0] = p2.x; e.ct[1] = p2.y; e.ct[2] = p2.z; e.mc = p2.w;
  e.J[0] = p3.x; e.J[1] = p3.y; e.J[2] = p3.z;
  if (a.h.use_motor_model) {
    float4 m = S[GR_P_MOTOR * n + i];
    e.mw[0] = m.x; e.mw[1] = m.y; e.mw[2] = m.z; e.mw[3] = m.w;
  } else {
    e.mw[0] = e.mw[1] = e.mw[2] = e.mw[3] = 0.0f;
  }
  e.ep = ii.x; e.acc = ii.y; e.epoch = ii.z;
  e.gate = ii.w & 0xff; e.lvl = (ii.w >> 8) & 0xff; e.azero = (ii.w >> 16) & 1; e.type = (ii.w >> 24) & 0xff;
}

// Per-step planes: kinematics, controller filters, lag (+ motor speeds) ...
DEV void store_kin(const KArgs& a, int i, const Env& e) {
  float4* S = reinterpret_cast<float4*>(a.buf.state);
  const size_t n = (size_t)a.h.num_envs;
  st4s(S, GR_P_POSQ * n + i, make_float4(e.p[0], e.p[1], e.p[2], e.q[0]));
  st4s(S, GR_P_QV * n + i, make_float4(e.q[1], e.q[2], e.q[3], e.v[0]));
  st4s(S, GR_P_VW * n + i, make_float4(e.v[1], e.v[2], e.w[0], e.w[1]));
  st4s(S, GR_P_WA * n + i, make_float4(e.w[2], e.al[0], e.al[1], e.al[2]));
  st4s(S, GR_P_CTRL * n + i, make_float4(e.T, e.tau[0], e.tau[1], e.tau[2]));
  st4s(S, GR_P_LAG * n + i, make_float4(e.lag[0], e.lag[1], e.lag[2], e.lag[3]));
  if (a.h.use_motor_model) st4s(S, GR_P_MOTOR * n + i, make_float4(e.mw[0], e.mw[1], e.mw[2], e.mw[3]));
}
// ... and episode sums
DEV void store_eps(const KArgs& a, int i, const Env& e) {
  float4* S = reinterpret_cast<float4*>(a.buf.state);
  const size_t n = (size_t)a.h.num_envs;
  st4s(S, GR_P_EP0 * n + i, make_float4(e.es[0], e.es[1], e.es[2], e.es[3]));
  st4s(S, GR_P_EP1 * n + i, make_float4(e.es[4], e.es[5], e.es[6], e.mar));
}
DEV void store_dyn(const KArgs& a, int i, const Env& e) {
  store_kin(a, i, e);
  store_eps(a, i, e);
}

// Per-episode domain-randomisation planes (written at reset only).
DEV void store_rst(const KArgs& a, int i, const Env& e) {
  float4* S = reinterpret_cast<float4*>(a.buf.state);
  const size_t n = (size_t)a.h.num_envs;
  st4s(S, GR_P_RST0 * n + i, make_float4(e.thr, e.nl, e.k2[0], e.k2[1]));
  st4s(S, GR_P_RST1 * n + i, make_float4(e.k2[2], e.k1[0], e.k1[1], e.k1[2]));
}

DEV void store_istate(const KArgs& a, int i, const Env& e) {
  int packed = (e.gate & 0xff) | ((e.lvl & 0xff) << 8) | ((e.azero & 1) << 16) | ((e.type & 0xff) << 24);
  st4s(reinterpret_cast<int4*>(a.buf.istate), (size_t)i, make_int4(e.ep, e.acc, e.epoch, packed));
}

// ------------------------------------------------------------- track table view
// Packed table: per track [max_gates * GR_GATE_FLOATS gate records | GR_TRACK_FLOATS track record].
// `base` points at the first track of type t0 (LDS copy or the global table).
struct Tab {
  const float* base;
  int t0, L, G, stride;
  DEV const float* track_base(int type, int lvl) const { return base + ((type - t0) * L + lvl) * stride; }
  DEV const float* gate(int type, int lvl, int g) const { return track_base(type, lvl) + g * GR_GATE_FLOATS; }
  DEV const float* rec(int type, int lvl) const { return track_base(type, lvl) + G * GR_GATE_FLOATS; }
};

DEV uint32_t gid_of(const KArgs& a, int i) { return (uint32_t)(a.h.env_id_offset + i); }
DEV gr_u32x4 draw(const KArgs& a, uint32_t gid, uint32_t c1, uint32_t tag, uint32_t c3) {
  return gr_philox4x32_10(gid, c1, tag, c3, a.h.seed_lo, a.h.seed_hi);
}

DEV void action_scale(const KArgs& a, float m_ctrl, float sc[4], float of[4]) {
  float weight = m_ctrl * a.kc->cfg.gravity;
  float s0 = (weight * a.kc->cfg.max_thrust_weight_ratio) / 2.0f;
  sc[0] = s0; of[0] = s0;
  for (int k = 1; k < 4; ++k) { sc[k] = a.kc->cfg.body_rate_bound; of[k] = 0.0f; }
}

// ------------------------------------------------------------- collision
// Lattice of the drone box (diff.lab/utils/__init__.py:19-37): offsets
// (lx*hx, ly*hy, lz*hz) with l in {0, +-1, +-0.5}.  quat_rotate is linear, so a
// lattice point is p + (lx*A + ly*B) + lz*C with A, B, C the rotated scaled body
// axes (3 rotations instead of 17); in a gate frame M (rows of R_gate^T) the same
// point is d_g + (lx*A_g + ly*B_g) + lz*C_g with d_g = M(p - c), A_g = M A, ...
// Oracle and kernel evaluate exactly these expressions; the kernel adds
// conservative culls (sphere, plane slab, outer box, hole) that can only skip
// gates where no lattice point can be inside, so the count is unchanged.
// compile-time lattice: after unrolling every offset is an inline constant (0, +-1, +-0.5)
constexpr float c_lattice[17][3] = GR_LATTICE_INIT;
#ifndef GR_OBST_BATCH
#define GR_OBST_BATCH 8  // obstacle cull spheres loaded per batch (8: -0.15 us on obstacle tracks vs 4; 16 spills)
#endif

// ------------------------------------------------------------- obstacles
// Per track a uniform xy grid; cell lists hold copies of every record whose cull sphere reaches into
// the cell grown by `margin` per axis (gr.h gr_obstacles, tracks.py pack_obstacles).  Per env, the
// GR_P_OHINT plane carries the list of the cell its position lies in (first item, count + 1, and the
// lower corner of the grown cell; 0 = no hint), written at the end of every step for the next one: so
// the records can be fetched at kernel entry, and the list serves the post-step test whenever the drone
// stayed within the grown cell (a step moves it a few cm).  Otherwise (no hint, left the grown cell) the
// post-step cell is looked up.
struct ObstGrid {
  float4 f;  // x0, y0, 1/cell, margin / cell
  int4 i;    // nx, ny, first cell, 0
};
DEV ObstGrid obst_grid(const KArgs& a, int type, int lvl) {
  const int tk = type * a.h.num_levels + lvl;
  return ObstGrid{a.obst_grid_f[tk], a.obst_grid_i[tk]};
}
// the cell of p: linear cell index, or -1 outside the grid; (cx, cy) its coordinates
DEV int obst_cell(const ObstGrid& og, const float p[3], int& cx, int& cy) {
  const float fx = (p[0] - og.f.x) * og.f.z, fy = (p[1] - og.f.y) * og.f.z;
  cx = cy = 0;
  if (!(fx >= 0.0f && fy >= 0.0f && fx < (float)og.i.x && fy < (float)og.i.y)) return -1;
  cx = (int)fx;
  cy = (int)fy;
  return og.i.z + cy * og.i.x + cx;
}
// lattice mask of one record (cull sphere first)
// (cull sphere, then the primitive grown by the lattice reach, then the 17 points)
DEV uint32_t obst_one(const KArgs& a, const float4 r4[GR_OBST_FLOATS / 4], const float p[3], const float A[3],
                      const float B[3], const float C[3]) {
  float r[GR_OBST_FLOATS];
#pragma unroll
  for (int k = 0; k < GR_OBST_FLOATS / 4; ++k) {
    r[4 * k] = r4[k].x; r[4 * k + 1] = r4[k].y; r[4 * k + 2] = r4[k].z; r[4 * k + 3] = r4[k].w;
  }
  if (!(gr_obst_near(r, p) && gr_obst_maybe(r, p, a.kc->lat_reach))) return 0u;
  return gr_obst_lattice_mask(r, p, A, B, C, c_lattice);
}
// the cull spheres of list items [first + j0, first + j0 + GR_OBST_BATCH) (w = -1 past the end)
DEV void obst_spheres(const KArgs& a, int first, int j0, int count, float4 sp[GR_OBST_BATCH]) {
#pragma unroll
  for (int j = 0; j < GR_OBST_BATCH; ++j)
    sp[j] = j0 + j < count ? a.obst_items[(size_t)(first + j0 + j) * (GR_OBST_FLOATS / 4)]
                           : make_float4(0.0f, 0.0f, 0.0f, -1.0f);
}
// lattice mask of the list items [first, first + count): cull spheres in batches of independent loads (the
// first batch may come prefetched), full records only for the spheres that hold p
DEV uint32_t obst_list(const KArgs& a, int first, int count, const float4* pre, const float p[3], const float A[3],
                       const float B[3], const float C[3]) {
  uint32_t m = 0u;
  for (int j0 = 0; j0 < count; j0 += GR_OBST_BATCH) {
    float4 sp[GR_OBST_BATCH];
    if (pre != nullptr && j0 == 0) {
#pragma unroll
      for (int j = 0; j < GR_OBST_BATCH; ++j) sp[j] = pre[j];
    } else {
      obst_spheres(a, first, j0, count, sp);
    }
    uint32_t near = 0u;
#pragma unroll
    for (int j = 0; j < GR_OBST_BATCH; ++j) {
      const float r[4] = {sp[j].x, sp[j].y, sp[j].z, sp[j].w};
      near |= (uint32_t)gr_obst_near(r, p) << j;
    }
    while (near) {
      const int j = __builtin_ctz(near);
      near &= near - 1u;
      const float4* r4 = a.obst_items + (size_t)(first + j0 + j) * (GR_OBST_FLOATS / 4);
      float4 rr[GR_OBST_FLOATS / 4];
#pragma unroll
      for (int k = 0; k < GR_OBST_FLOATS / 4; ++k) rr[k] = r4[k];
      m |= obst_one(a, rr, p, A, B, C);
    }
  }
  return m;
}
// full lookup from the grid (no hint)
DEV uint32_t obst_lookup(const KArgs& a, const ObstGrid& og, const float p[3], const float A[3], const float B[3],
                         const float C[3]) {
  int cx, cy;
  const int c = obst_cell(og, p, cx, cy);
  if (c < 0) return 0u;
  const int2 ce = a.obst_cells[c];
  return obst_list(a, ce.x, ce.y, nullptr, p, A, B, C);
}
// the hint of a position: its cell's list and the grown cell's lower corner (0: outside the grid)
DEV float4 obst_hint_of(const KArgs& a, const ObstGrid& og, const float p[3]) {
  int cx, cy;
  const int c = obst_cell(og, p, cx, cy);
  if (c < 0) return make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const int2 ce = a.obst_cells[c];
  const float cell = 1.0f / og.f.z, margin = og.f.w * cell;
  return make_float4(__int_as_float(ce.x), __int_as_float(ce.y + 1), og.f.x + (float)cx * cell - margin,
                     og.f.y + (float)cy * cell - margin);
}
// is p inside the hinted grown cell?  (span = cell + 2 margin)
DEV bool obst_hint_holds(const float4& h, const float p[3], float span) {
  return __float_as_int(h.y) > 0 && p[0] >= h.z && p[0] <= h.z + span && p[1] >= h.w && p[1] <= h.w + span;
}

DEV void body_axes(const KArgs& a, const float q[4], float A[3], float B[3], float Cz[3]) {
  const float ex[3] = {a.kc->cfg.collider_half[0], 0.0f, 0.0f}, ey[3] = {0.0f, a.kc->cfg.collider_half[1], 0.0f},
              ez[3] = {0.0f, 0.0f, a.kc->cfg.collider_half[2]};
  quat_rotate(q, ex, A);
  quat_rotate(q, ey, B);
  quat_rotate(q, ez, Cz);
}

DEV void gate_frame(const float* g, const float v[3], float o[3]) {
  o[0] = (g[4] * v[0] + g[5] * v[1]) + g[6] * v[2];
  o[1] = (g[8] * v[0] + g[9] * v[1]) + g[10] * v[2];
  o[2] = (g[12] * v[0] + g[13] * v[1]) + g[14] * v[2];
}

// lattice mask (17 bits) of the points inside a gate frame or under the ground, and with OBST inside
// an obstacle looked up from the grid (the substep integrator; the explicit step hands obstacles to the
// policy waves instead).  Replaces PhysX contact / Warp mesh_tools.py:128-233; see oracle.
// MAXG > 0: tracks of at most MAXG gates (the launch checks max_gates), the sphere pass a fixed predicated sequence
template <bool OBST, int MAXG = 0>
DEV uint32_t collision_mask(const KArgs& a, const Tab& tab, int type, int lvl, const float p[3], const float q[4],
                            const ObstGrid& og) {
  const float* rec = tab.rec(type, lvl);
  const float ground = rec[0];
  const int ng = (int)rec[3];
  const float reach = a.kc->lat_reach;  // > max |lattice offset| incl. rounding
  // ---- pass 1: bounding-sphere cull, one 16-byte read (centre, r^2) per gate ----
  uint32_t sph = 0u;
  if constexpr (MAXG > 0) {
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      if (g < ng) {
        const float4 c4 = *reinterpret_cast<const float4*>(tab.gate(type, lvl, g));
        const float dx = p[0] - c4.x, dy = p[1] - c4.y, dz = p[2] - c4.z;
        if ((dx * dx + dy * dy) + dz * dz <= c4.w) sph |= 1u << g;
      }
    }
  } else {
#pragma unroll 8
    for (int g = 0; g < ng; ++g) {
      const float4 c4 = *reinterpret_cast<const float4*>(tab.gate(type, lvl, g));
      const float dx = p[0] - c4.x, dy = p[1] - c4.y, dz = p[2] - c4.z;
      if ((dx * dx + dy * dy) + dz * dz <= c4.w) sph |= 1u << g;
    }
  }
  const bool ground_near = p[2] - ground < reach;
  int ocount = 0;
  if (OBST) {
    int cx, cy;
    ocount = obst_cell(og, p, cx, cy) >= 0;
  }
  if (!sph && !ground_near && !ocount) return 0u;
  float A[3], B[3], Cz[3];
  body_axes(a, q, A, B, Cz);
  uint32_t inside = 0u;
  if (ground_near) {
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      float oz = (c_lattice[k][0] * A[2] + c_lattice[k][1] * B[2]) + c_lattice[k][2] * Cz[2];
      if (p[2] + oz < ground) inside |= 1u << k;
    }
  }
  // ---- pass 2: gates inside the sphere: plane-slab / outer-box / hole culls (2a), then the lattice of the
  // survivors (2b).  Two loops, so a wave runs the lattice as often as its worst lane has survivors, not as
  // often as its worst lane has sphere hits (dense tracks: several spheres per env) ----
  uint32_t cand = 0u;
  while (sph) {
    const int g = __builtin_ctz(sph);
    sph &= sph - 1u;
    const float* gr = tab.gate(type, lvl, g);
    float d[3] = {p[0] - gr[0], p[1] - gr[1], p[2] - gr[2]};
    float dg[3];
    gate_frame(gr, d, dg);
    const float x = gr_fabsf(dg[0]), y = gr_fabsf(dg[1]), z = gr_fabsf(dg[2]);
    const bool slab = z <= gr[15] + reach;
    const bool outer = (x <= gr[16] + reach) & (y <= gr[17] + reach);
    const bool hole = (x < gr[7] - reach) & (y < gr[11] - reach);
    if (slab & outer & !hole) cand |= 1u << g;
  }
  while (cand) {
    const int g = __builtin_ctz(cand);
    cand &= cand - 1u;
    const float* gr = tab.gate(type, lvl, g);
    float d[3] = {p[0] - gr[0], p[1] - gr[1], p[2] - gr[2]};
    float dg[3];
    gate_frame(gr, d, dg);
    float Ag[3], Bg[3], Cg[3];
    gate_frame(gr, A, Ag);
    gate_frame(gr, B, Bg);
    gate_frame(gr, Cz, Cg);
#pragma unroll
    for (int k = 0; k < 17; ++k) {
      const float lx = c_lattice[k][0], ly = c_lattice[k][1], lz = c_lattice[k][2];
      float l0 = dg[0] + ((lx * Ag[0] + ly * Bg[0]) + lz * Cg[0]);
      float l1 = dg[1] + ((lx * Ag[1] + ly * Bg[1]) + lz * Cg[1]);
      float l2 = dg[2] + ((lx * Ag[2] + ly * Bg[2]) + lz * Cg[2]);
      float a0 = gr_fabsf(l0), a1 = gr_fabsf(l1), a2 = gr_fabsf(l2);
      bool in_outer = (a0 <= gr[16]) & (a1 <= gr[17]) & (a2 <= gr[15]);
      bool in_hole = (a0 < gr[7]) & (a1 < gr[11]);
      if (in_outer & !in_hole) inside |= 1u << k;
    }
  }
  if (OBST) inside |= obst_lookup(a, og, p, A, B, Cz);
  return inside;
}

// ------------------------------------------------------------- controller
// Rotor constants of one env: the config's (derived once on the host, KConst) or, with config C5's rotor-
// constant DR, the env's own thrust map and kappa (GR_P_ROTOR: k2 k1 k0 kappa), through the same double-
// precision expressions as derive() (gr_capi.cpp) and the oracle.
struct MotorK {
  float lo, hi;                                  // gross-thrust clamp 4 f(w_min), 4 f(w_max) (controller_diff.py:96-99)
  float fmax;                                    // rotor thrust cap f(w_max) (:142)
  float kap, kap_inv4;                           // kappa, 1 / (4 kappa): allocation row / column 3
  float k2, k1, k0, k1sq, k4k2, inv2k2, negk1;   // thrust map, Thrust2Omega (thrust_controller_diff.py:167-179)
  bool own;
};
DEV void motor_consts(const KArgs& a, const float4* rk, MotorK& m) {
  m.own = rk != nullptr;
  if (!rk) {
    m.lo = a.kc->thrust_lo; m.hi = a.kc->thrust_hi; m.fmax = a.kc->motor_fmax;
    m.kap = 0.0f; m.kap_inv4 = 0.0f;  // (the KConst matrices are used)
    m.k2 = a.kc->tm_k2; m.k1 = a.kc->tm_k1; m.k0 = a.kc->tm_k0;
    m.k1sq = a.kc->tm_k1sq; m.k4k2 = a.kc->tm_4k2; m.inv2k2 = a.kc->tm_inv2k2; m.negk1 = a.kc->tm_negk1;
    return;
  }
  const double k2 = rk->x, k1 = rk->y, k0 = rk->z;
  const double w0 = a.kc->cfg.motor_omega[0], w1 = a.kc->cfg.motor_omega[1];
  const double tmin = k2 * w0 * w0 + k1 * w0 + k0, tmax = k2 * w1 * w1 + k1 * w1 + k0;
  m.lo = (float)(tmin * 4.0); m.hi = (float)(tmax * 4.0); m.fmax = (float)tmax;
  m.kap = rk->w; m.kap_inv4 = 1.0f / (4.0f * rk->w);
  m.k2 = (float)k2; m.k1 = (float)k1; m.k0 = (float)k0;
  m.k1sq = (float)(k1 * k1); m.k4k2 = (float)(4.0 * k2); m.inv2k2 = (float)(1.0 / (2.0 * k2)); m.negk1 = (float)(-k1);
}

// ThrustController.update (thrust_controller_diff.py:182-186): desired rotor thrusts -> motor speeds
// (Thrust2Omega :167-176) -> first-order motor lag -> realised thrusts (Omega2Thrust :178-179), in place
DEV void motor_update(const KArgs& a, const MotorK& m, float f[4], float mw[4]) {
  for (int i = 0; i < 4; ++i) {
    float t3 = m.k1sq - m.k4k2 * (m.k0 - f[i]);
    float wdes = m.inv2k2 * (m.negk1 + gr_sqrtf(t3));
    mw[i] = a.kc->motor_c * mw[i] + (1.0f - a.kc->motor_c) * wdes;
    f[i] = (m.k2 * mw[i] * mw[i] + m.k1 * mw[i]) + m.k0;
  }
}

// CTBRController.compute (controller_diff.py:120-144); rk: the env's rotor constants (dr_rotor) or null
// NO_MOTOR: compiled for configurations without the motor model (the lean step kernel)
template <bool NO_MOTOR = false>
DEV void ctbr_compute(const KArgs& a, const float cmd[4], const float wb[3], const float ab[3], const float Kp[3],
                      const float Kd[3], float cT, const float ct[3], float& T, float tau[3], float mw[4],
                      float tt[4], const float4* rk = nullptr) {
  MotorK mk;
  motor_consts(a, rk, mk);
  float T_des = gr_clampf(cmd[0], mk.lo, mk.hi);
  T = (1.0f - cT) * T_des + cT * T;
  const float* J = a.kc->cfg.inertia;
  float err[3], Jw[3], cr[3];
  for (int i = 0; i < 3; ++i) err[i] = gr_clampf(cmd[i + 1], -a.kc->cfg.body_rate_bound, a.kc->cfg.body_rate_bound) - wb[i];
  for (int i = 0; i < 3; ++i) Jw[i] = J[i] * wb[i];
  cross3(wb, Jw, cr);
  for (int i = 0; i < 3; ++i) {
    float tdes = (J[i] * (Kp[i] * err[i]) + cr[i]) - Kd[i] * ab[i];
    tau[i] = (1.0f - ct[i]) * tdes + ct[i] * tau[i];
  }
  tt[0] = T; tt[1] = tau[0]; tt[2] = tau[1]; tt[3] = tau[2];
  if (NO_MOTOR || !a.h.use_motor_model) return;
  // allocation (controller_diff.py:56-69): rows 0-2 / columns 0-2 do not involve kappa; row / column 3 is
  // kappa * (1 -1 1 -1) and its inverse (1 -1 1 -1) / (4 kappa)
  const float sz[4] = {1.0f, -1.0f, 1.0f, -1.0f};
  float f[4];
  for (int r = 0; r < 4; ++r) {
    const float bi3 = mk.own ? sz[r] * mk.kap_inv4 : a.kc->Bi[r][3];
    f[r] = ((tt[0] * a.kc->Bi[r][0] + tt[1] * a.kc->Bi[r][1]) + tt[2] * a.kc->Bi[r][2]) + tt[3] * bi3;
  }
  for (int i = 0; i < 4; ++i) f[i] = gr_clampf(f[i], 0.0f, mk.fmax);  // controller_diff.py:142
  motor_update(a, mk, f, mw);
  for (int r = 0; r < 3; ++r) tt[r] = ((f[0] * a.kc->B[r][0] + f[1] * a.kc->B[r][1]) + f[2] * a.kc->B[r][2]) + f[3] * a.kc->B[r][3];
  if (mk.own) tt[3] = ((f[0] * (mk.kap * sz[0]) + f[1] * (mk.kap * sz[1])) + f[2] * (mk.kap * sz[2])) + f[3] * (mk.kap * sz[3]);
  else tt[3] = ((f[0] * a.kc->B[3][0] + f[1] * a.kc->B[3][1]) + f[2] * a.kc->B[3][2]) + f[3] * a.kc->B[3][3];
}

// ------------------------------------------------------------- integrators
// DroneDynamics.step (droneDynamics.py:119-135)
DEV void dd_explicit(float m, const float J[3], const float k2[3], const float k1[3], const float tt[4], float dt,
                     float gz, float p[3], float q[4], float v[3], float w[3], float a_out[3], float al_out[3]) {
  float vb[3];
  quat_rotate_inverse(q, v, vb);
  float thr[3] = {0.0f, 0.0f, tt[0]};
  for (int i = 0; i < 3; ++i) thr[i] = (thr[i] - (k2[i] * vb[i]) * gr_fabsf(vb[i])) - k1[i] * vb[i];
  float tw[3];
  quat_rotate(q, thr, tw);
  float acc[3] = {0.0f + tw[0] / m, 0.0f + tw[1] / m, -gz + tw[2] / m};
  float Jw[3] = {J[0] * w[0], J[1] * w[1], J[2] * w[2]}, cr[3];
  cross3(w, Jw, cr);
  float al[3];
  for (int i = 0; i < 3; ++i) {
    float ji = 1.0f / J[i];
    al[i] = ji * tt[i + 1] - ji * cr[i];
  }
  for (int i = 0; i < 3; ++i) p[i] = (p[i] + v[i] * dt) + ((0.5f * acc[i]) * dt) * dt;
  float wq[4] = {0.0f, w[0], w[1], w[2]}, qd[4];
  quat_mul(q, wq, qd);
  for (int i = 0; i < 4; ++i) q[i] = q[i] + (0.5f * qd[i]) * dt;
  float nq = gr_sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / nq;
  for (int i = 0; i < 3; ++i) v[i] = v[i] + acc[i] * dt;
  for (int i = 0; i < 3; ++i) w[i] = w[i] + al[i] * dt;
  for (int i = 0; i < 3; ++i) { a_out[i] = acc[i]; al_out[i] = al[i]; }
}

// semi-implicit Euler substep (PhysX role), wrench held over the substep
DEV void si_substep(float m, const float J[3], const float fb[3], const float tb[3], float h, float gz, float p[3],
                    float q[4], float v[3], float w[3], float a_out[3], float al_out[3]) {
  float tw[3];
  quat_rotate(q, fb, tw);
  float acc[3] = {0.0f + tw[0] / m, 0.0f + tw[1] / m, -gz + tw[2] / m};
  float Jw[3] = {J[0] * w[0], J[1] * w[1], J[2] * w[2]}, cr[3];
  cross3(w, Jw, cr);
  float al[3];
  for (int i = 0; i < 3; ++i) al[i] = (tb[i] - cr[i]) / J[i];
  for (int i = 0; i < 3; ++i) v[i] = v[i] + acc[i] * h;
  for (int i = 0; i < 3; ++i) w[i] = w[i] + al[i] * h;
  for (int i = 0; i < 3; ++i) p[i] = p[i] + v[i] * h;
  float wq[4] = {0.0f, w[0], w[1], w[2]}, qd[4];
  quat_mul(q, wq, qd);
  for (int i = 0; i < 4; ++i) q[i] = q[i] + (0.5f * qd[i]) * h;
  float nq = gr_sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / nq;
  for (int i = 0; i < 3; ++i) { a_out[i] = acc[i]; al_out[i] = al[i]; }
}

// ------------------------------------------------------------- reset
// reset_root_state_racing (events.py:139-177) + drag DR (droneDynamics.py:50-57) +
// thrust-estimate error (diff_action.py:223-233) + curriculum (curriculums.py:25-54).
// Split in two: everything that depends only on (env, next episode) — the four
// Philox blocks, uniforms, Box-Muller, drag — can be drawn before it is known
// whether the env resets; the rest (level, yaw to the start gate) is applied then.
struct ResetDraws {
  float p[3], att[3], v[3], wv[3];  // spawn position, roll/pitch/yaw offsets, linear / angular velocity
  float k2[3], k1[3];               // drag (random_drag)
  float lvl_u, thr;                 // random level for "beyond the last level", thrust-estimate error
  float sr, cr, sp, cp;             // sin/cos of roll/2 and pitch/2 (quat_from_euler_xyz)
};

// 24 x 21-bit fields: pos 0-2, att 3-5, vel 6-11, z-drag 12, k2 13-15, k1 16-18, level 19, thr 20-21
DEV void reset_draws(const KArgs& a, uint32_t gid, uint32_t ep, float m_ctrl, ResetDraws& r) {
  const gr_config& c = a.kc->cfg;
  uint32_t f[24];
  gr_u32x4 w4[4];
  gr_philox4x32_10_x4(gid, ep, GR_TAG_RESET, 0u, a.h.seed_lo, a.h.seed_hi, w4);
  for (int j = 0; j < 4; ++j) gr_fields6(w4[j], f + 6 * j);
  r.lvl_u = gr_f21(f[19]);
  for (int k = 0; k < 3; ++k) {
    r.p[k] = c.spawn_pos[k] + gr_uniform21(f[k], -c.reset_pos_half[k], c.reset_pos_half[k]);
    r.att[k] = gr_uniform21(f[3 + k], -c.reset_att_half[k], c.reset_att_half[k]);
    r.v[k] = 0.0f + gr_uniform21(f[6 + k], -c.reset_vel_half[k], c.reset_vel_half[k]);
    r.wv[k] = 0.0f + gr_uniform21(f[9 + k], -c.reset_vel_half[3 + k], c.reset_vel_half[3 + k]);
  }
  {  // drag DR (applied only with random_drag; computed unconditionally to keep one basic block)
    float z = c.z_drag + gr_f21(f[12]) * c.z_drag_rand;
    for (int k = 0; k < 3; ++k) {
      r.k2[k] = c.drag2[k] * m_ctrl + gr_f21(f[13 + k]) * c.drag2_rand;
      r.k1[k] = c.drag1[k] * m_ctrl + gr_f21(f[16 + k]) * c.drag1_rand;
    }
    r.k2[2] = r.k2[2] * z;
    r.k1[2] = r.k1[2] * z;
  }
  float z0, z1;
  gr_box_muller21(f[20], f[21], &z0, &z1);
  r.thr = 1.0f + z0 * 0.01f;
  sincos_w(r.att[0] * 0.5f, &r.sr, &r.cr);
  sincos_w(r.att[1] * 0.5f, &r.sp, &r.cp);
}

DEV void reset_apply(const KArgs& a, const Tab& tab, Env& e, const ResetDraws& r) {
  const gr_config& c = a.kc->cfg;
  int up = e.acc >= c.level_up_threshold, down = e.acc < c.level_down_threshold;
  int lvl = e.lvl + up - down;
  if (lvl >= c.num_levels) lvl = (int)gr_floorf(r.lvl_u * (float)c.num_levels);
  else if (lvl < 0) lvl = 0;
  {
    float upf = e.acc >= c.noise_enhance_threshold ? 1.0f + c.noise_enhance : 1.0f;
    float dnf = e.acc < c.noise_decay_threshold ? 1.0f - c.noise_decay : 1.0f;
    float nl = e.nl * upf;
    nl = nl * dnf;
    e.nl = c.noise_curriculum ? nl : e.nl;
  }
  e.lvl = lvl;
  for (int k = 0; k < 3; ++k) e.p[k] = r.p[k];
  const float* rec = tab.rec(e.type, lvl);
  int start = (int)rec[2];
  const float* g0 = tab.gate(e.type, lvl, start);
  float tx = g0[0] - e.p[0], ty = g0[1] - e.p[1];
  float yaw = gr_wrap_to_pi(gr_atan2f(ty, tx)) + r.att[2];
  float qd[4], qid[4] = {1.0f, 0.0f, 0.0f, 0.0f};
  {  // quat_from_euler_xyz(roll, pitch, yaw) with the roll/pitch half-angle sincos drawn ahead
    float sy, cy;
    gr_sincosf(yaw * 0.5f, &sy, &cy);
    const float sr = r.sr, cr = r.cr, sp = r.sp, cp = r.cp;
    qd[0] = (cy * cr) * cp + (sy * sr) * sp;
    qd[1] = (cy * sr) * cp - (sy * cr) * sp;
    qd[2] = (cy * cr) * sp + (sy * sr) * cp;
    qd[3] = (sy * cr) * cp - (cy * sr) * sp;
  }
  quat_mul(qid, qd, e.q);
  for (int k = 0; k < 3; ++k) e.v[k] = r.v[k];
  quat_rotate_inverse(e.q, r.wv, e.w);
  e.azero = 1;
  e.T = 0.0f;
  for (int k = 0; k < 3; ++k) { e.tau[k] = 0.0f; e.al[k] = 0.0f; }
  for (int k = 0; k < 4; ++k) e.mw[k] = 0.0f;
  for (int k = 0; k < 3; ++k) {
    e.k2[k] = c.random_drag ? r.k2[k] : e.k2[k];
    e.k1[k] = c.random_drag ? r.k1[k] : e.k1[k];
  }
  e.thr = r.thr;
  for (int k = 0; k < 7; ++k) e.es[k] = 0.0f;
  e.mar = 0.0f;
  e.acc = 0;
  e.gate = start;
  e.ep = 0;
  e.epoch = e.epoch + 1;
}

DEV void reset_env(const KArgs& a, const Tab& tab, Env& e, uint32_t gid) {
  ResetDraws r;
  reset_draws(a, gid, (uint32_t)e.epoch + 1u, e.mc, r);
  reset_apply(a, tab, e, r);
}

// ------------------------------------------------------------- observations
// gate-pose noise of the current (out[0..2]) and next (out[3..5]) gate: one draw
// per (episode, gates passed), commands.py:287-289,329-350
DEV void gate_noise(const KArgs& a, const Env& e, uint32_t gid, float out[6]) {
  if (!a.kc->cfg.add_gate_noise) { for (int k = 0; k < 6; ++k) out[k] = 0.0f; return; }
  uint32_t f[6];
  gr_fields6(draw(a, gid, (uint32_t)e.epoch, GR_TAG_GATE, (uint32_t)e.acc), f);
  for (int k = 0; k < 6; ++k) {
    float lo = (-a.kc->cfg.gate_noise_pos[k % 3]) * e.nl, hi = a.kc->cfg.gate_noise_pos[k % 3] * e.nl;
    out[k] = lo + gr_f21(f[k]) * (hi - lo);
  }
}

// Observation noise depends only on (env, call counter): drawn before the state
// loads land, so its Philox / Box-Muller work hides under the load latency.
struct ObsNoise {
  float vfac[3];  // 1 + N(0,1) * 0.03        (observation.py:52)
  float qn[4];    // quat_from_euler_xyz(N(0,1) * 0.05) (observation.py:27-28)
};

DEV void obs_noise(const KArgs& a, uint32_t gid, uint32_t cnt, ObsNoise& on) {
  float nz[6];
  {  // drawn unconditionally (one basic block for the scheduler), zeroed without obs noise
    uint32_t f[6];
    gr_fields6(draw(a, gid, cnt, GR_TAG_OBS, 0), f);
    for (int k = 0; k < 6; ++k) nz[k] = gr_normal21(f[k], obs_normal_tab);
    for (int k = 0; k < 6; ++k) nz[k] = a.h.obs_noise ? nz[k] : 0.0f;
  }
  for (int k = 0; k < 3; ++k) on.vfac[k] = 1.0f + nz[k] * a.h.obs_lin_vel_noise;
  quat_from_euler_xyz(nz[3] * a.h.obs_att_noise, nz[4] * a.h.obs_att_noise, nz[5] * a.h.obs_att_noise, on.qn);
}

// policy / critic observation rows of one env (observation.py:22-63, commands.py:208-245;
// group order racing_ctbr_env.py:141-169)
struct ObsRows {
  float4 c[4], p[4];
};

// the gates an observation refers to: current and next of the env's track
DEV void obs_gates(const Tab& tab, const Env& e, float g0[3], float gn0[3]) {
  const float* rec = tab.rec(e.type, e.lvl);
  int ng = (int)rec[3];
  const float* g = tab.gate(e.type, e.lvl, e.gate);
  int gnext = e.gate + 1;
  if (gnext >= ng) gnext -= ng;
  const float* gn = tab.gate(e.type, e.lvl, gnext);
  for (int k = 0; k < 3; ++k) { g0[k] = g[k]; gn0[k] = gn[k]; }
}

// critic row: noise-free (observation.py:97-104, commands.py:233-245)
DEV void compute_critic(const Tab& tab, const Env& e, const float lc[4], float4 c[4]) {
  float g0[3], gn0[3];
  obs_gates(tab, e, g0, gn0);
  float vb[3], r2[3];
  quat_rotate_inverse(e.q, e.v, vb);
  matrix_row2(e.q, r2);
  float d[3] = {g0[0] - e.p[0], g0[1] - e.p[1], g0[2] - e.p[2]};
  float dn[3] = {gn0[0] - g0[0], gn0[1] - g0[1], gn0[2] - g0[2]};
  float cg[3], cn[3];
  quat_rotate_inverse(e.q, d, cg);
  quat_rotate_inverse(e.q, dn, cn);
  c[0] = make_float4(vb[0], vb[1], vb[2], r2[0]);
  c[1] = make_float4(r2[1], r2[2], cg[0], cg[1]);
  c[2] = make_float4(cg[2], cn[0], cn[1], cn[2]);
  c[3] = make_float4(lc[0], lc[1], lc[2], lc[3]);
}

// policy row: velocity and attitude noise (observation.py:22-63), noisy gate poses (commands.py:208-221)
DEV void compute_policy(const KArgs& a, const Tab& tab, const Env& e, uint32_t gid, const ObsNoise& on,
                        const float lc[4], float4 p[4]) {
  float g0[3], gn0[3];
  obs_gates(tab, e, g0, gn0);
  float vb[3];
  quat_rotate_inverse(e.q, e.v, vb);
  float qq[4], r2n[3];
  quat_mul(e.q, on.qn, qq);
  matrix_row2(qq, r2n);
  float gnz[6];
  gate_noise(a, e, gid, gnz);
  float gw[3] = {g0[0] + gnz[0], g0[1] + gnz[1], g0[2] + gnz[2]};
  float gnw[3] = {gn0[0] + gnz[3], gn0[1] + gnz[4], gn0[2] + gnz[5]};
  float dp[3] = {gw[0] - e.p[0], gw[1] - e.p[1], gw[2] - e.p[2]};
  float dnp[3] = {gnw[0] - gw[0], gnw[1] - gw[1], gnw[2] - gw[2]};
  float pg[3], pn[3];
  quat_rotate_inverse(e.q, dp, pg);
  quat_rotate_inverse(e.q, dnp, pn);
  float vn[3];
  for (int k = 0; k < 3; ++k) vn[k] = vb[k] * on.vfac[k];
  p[0] = make_float4(vn[0], vn[1], vn[2], r2n[0]);
  p[1] = make_float4(r2n[1], r2n[2], pg[0], pg[1]);
  p[2] = make_float4(pg[2], pn[0], pn[1], pn[2]);
  p[3] = make_float4(lc[0], lc[1], lc[2], lc[3]);
}

DEV void compute_obs(const KArgs& a, const Tab& tab, const Env& e, uint32_t gid, const ObsNoise& on,
                     const float lc[4], ObsRows& o) {
  compute_critic(tab, e, lc, o.c);
  compute_policy(a, tab, e, gid, on, lc, o.p);
}

// command compute: _update_metrics + _update_command (commands.py:247-260, 308-350)
DEV void gate_advance(const KArgs& a, const Tab& tab, Env& e) {
  const float* gg = tab.gate(e.type, e.lvl, e.gate);
  float dd[3] = {gg[0] - e.p[0], gg[1] - e.p[1], gg[2] - e.p[2]};
  const bool pass = norm3(dd) < a.kc->cfg.gate_threshold;
  const int ngt = (int)tab.rec(e.type, e.lvl)[3];
  int g = e.gate + 1;
  if (g >= ngt) g -= ngt;
  e.acc = pass ? e.acc + 1 : e.acc;
  e.gate = pass ? g : e.gate;
}

// one lane writes its env's 64-byte rows (4 x 16 B, 64-byte lane stride)
DEV void store_obs_direct(const KArgs& a, int i, const ObsRows& o, float aux) {
  float4* C = reinterpret_cast<float4*>(a.buf.obs_critic) + (size_t)i * 4;
  float4* P = reinterpret_cast<float4*>(a.buf.obs_policy) + (size_t)i * 4;
  for (int k = 0; k < 4; ++k) C[k] = o.c[k];
  for (int k = 0; k < 4; ++k) P[k] = o.p[k];
  a.buf.obs_aux[i] = aux;
}

// The same rows written by a whole wave through an LDS transpose, so each store
// instruction covers 1 KiB of consecutive bytes (16 envs x 64 B) instead of 64
// scattered 16-byte pieces: the store path of a CU is the tail of the step.
// `stage` = this wave's 4 x 64 float4 LDS slots (quad-major: conflict-free writes).
DEV void store_rows_staged(float4* dst, int env0, int n, const float4 rows[4], float4* stage) {
  const int l = threadIdx.x & 63;
  for (int q = 0; q < 4; ++q) stage[q * GR_BLOCK + l] = rows[q];
  __asm__ volatile("" ::: "memory");  // LDS ops of a wave retire in order; keep the compiler from reordering
  for (int j = 0; j < 4; ++j) {
    const int env = 16 * j + (l >> 2), q = l & 3;
    const float4 v = stage[q * GR_BLOCK + env];
    if (env0 + env < n) st4(dst, (size_t)(env0 + env) * 4 + q, v);
  }
  __asm__ volatile("" ::: "memory");
}

// Observation sink (gr_bind_obs_sink): the same rows again into the rollout storage's slot, fp32 or bf16.
// bf16: round to nearest even on the fp32 bits, NaN -> 0x7FC0 (c10::BFloat16's round_to_nearest_even).
DEV uint32_t bf16_rne(float x) {
  const uint32_t u = __float_as_uint(x);
  return (x != x) ? 0x7FC0u : ((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
DEV uint32_t bf16x2(float lo, float hi) { return bf16_rne(lo) | (bf16_rne(hi) << 16); }
DEV uint4 bf16x8(const float4& u, const float4& v) {
  return make_uint4(bf16x2(u.x, u.y), bf16x2(u.z, u.w), bf16x2(v.x, v.y), bf16x2(v.z, v.w));
}
// from the LDS stage of store_rows_staged (call right after it): bf16 rows are 32 B, two lanes per env, so
// each store instruction again covers 1 KiB of consecutive bytes
DEV void store_rows_sink(const KArgs& a, void* dst, int env0, int n, const float4* stage) {
  const int l = threadIdx.x & 63;
  if (a.sink_dtype == GR_DTYPE_BF16) {
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (int j = 0; j < 2; ++j) {
      const int env = 32 * j + (l >> 1), h = l & 1;
      const uint4 w = bf16x8(stage[(2 * h) * GR_BLOCK + env], stage[(2 * h + 1) * GR_BLOCK + env]);
      if (env0 + env < n) st4(d, (size_t)(env0 + env) * 2 + h, w);
    }
  } else {
    float4* d = reinterpret_cast<float4*>(dst);
    for (int j = 0; j < 4; ++j) {
      const int env = 16 * j + (l >> 2), q = l & 3;
      const float4 v = stage[q * GR_BLOCK + env];
      if (env0 + env < n) st4(d, (size_t)(env0 + env) * 4 + q, v);
    }
  }
  __asm__ volatile("" ::: "memory");
}
// one env's rows (gr_reset / gr_observe)
DEV void store_obs_sink(const KArgs& a, int i, const ObsRows& o) {
  if (a.sink_dtype == GR_DTYPE_BF16) {
    uint4* P = reinterpret_cast<uint4*>(a.sink_policy) + (size_t)i * 2;
    uint4* C = reinterpret_cast<uint4*>(a.sink_critic) + (size_t)i * 2;
    P[0] = bf16x8(o.p[0], o.p[1]); P[1] = bf16x8(o.p[2], o.p[3]);
    C[0] = bf16x8(o.c[0], o.c[1]); C[1] = bf16x8(o.c[2], o.c[3]);
  } else {
    float4* P = reinterpret_cast<float4*>(a.sink_policy) + (size_t)i * 4;
    float4* C = reinterpret_cast<float4*>(a.sink_critic) + (size_t)i * 4;
    for (int k = 0; k < 4; ++k) { P[k] = o.p[k]; C[k] = o.c[k]; }
  }
}

// ------------------------------------------------------------- log reduction
// Per-wave partial sums into log_partial[row][GR_LOG_SLOTS] (no workgroup
// barrier); a workgroup owns GR_LOG_ROWS_PER_BLOCK rows.  Resets are sparse
// (~1 % of envs per step): the reset slots are accumulated over the set bits of
// the wave's reset ballot with wave-uniform lane reads; the two all-env sums
// (terrain level, noise level) use a butterfly.  Means are formed on demand.

// a wave-uniform row of GR_LOG_SLOTS floats, written by lane 0 (five 16-byte stores).  (Spreading
// the row over lanes 0-4 in one store instruction measured 2 us SLOWER per step on gfx950.)
DEV void log_row_store(const KArgs& a, int row, const float v[GR_LOG_SLOTS]) {
  if ((threadIdx.x & 63) != 0) return;
  float4* r = reinterpret_cast<float4*>(a.buf.log_partial + ((size_t)blockIdx.x * GR_LOG_ROWS_PER_BLOCK + row) *
                                                                GR_LOG_SLOTS);
  r[0] = make_float4(v[0], v[1], v[2], v[3]);
  r[1] = make_float4(v[4], v[5], v[6], v[7]);
  r[2] = make_float4(v[8], v[9], v[10], v[11]);
  r[3] = make_float4(v[12], v[13], v[14], v[15]);
  r[4] = make_float4(v[16], v[17], v[18], v[19]);
}

// reset-lane slots (GR_LOG_NRESET .. GR_LOG_T_BADPOSE) of this wave -> row
// wave-wide float sum by DPP (no LDS round trips); the total lands in lane 63
template <int CTRL, int ROWS>
DEV float dpp_term(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
DEV float wave_sum63(float v) {
  v = v + dpp_term<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = v + dpp_term<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = v + dpp_term<0x141, 0xF>(v);  // row_half_mirror
  v = v + dpp_term<0x140, 0xF>(v);  // row_mirror: every lane of a row holds the row sum
  v = v + dpp_term<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = v + dpp_term<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return v;
}

// one row per wave: the reset slots summed over the wave's resetting lanes, and the all-env slots
// (terrain level, noise level of the post-reset state) summed over its live lanes
DEV void wave_log(const KArgs& a, int row, const float lg[GR_LOG_SLOTS], bool reset_lane, float level, float noise) {
  float acc[GR_LOG_SLOTS];
  for (int s = 0; s < GR_LOG_SLOTS; ++s) acc[s] = 0.0f;
  uint64_t m = __ballot(reset_lane);
  while (m) {
    const int l = __builtin_ctzll(m);
    m &= m - 1;
    for (int s = 0; s < GR_LOG_LEVEL; ++s) acc[s] += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lg[s]), l));
  }
  acc[GR_LOG_LEVEL] = __shfl(wave_sum63(level), 63, 64);
  acc[GR_LOG_NOISE] = __shfl(wave_sum63(noise), 63, 64);
  log_row_store(a, row, acc);
}

// ------------------------------------------------------------- gate table staging
// The workgroup's slice of the track table (its terrain types x all levels) is
// loaded into registers together with the state loads, and written to LDS only
// when the collision test needs it: the barrier then waits for loads that have
// long landed, while the controller and integrator run under the load latency.
constexpr int GR_TREG = 2;  // float4 per thread held in registers (one 8-gate type: 410 float4)

__device__ __forceinline__ void table_commit(const float4* src, int nvec, float4 r0, float4 r1, float4* lds) {
  const int t = threadIdx.x;
  if (t < nvec) lds[t] = r0;
  if (t + GR_BLOCK < nvec) lds[t + GR_BLOCK] = r1;
  for (int idx = t + GR_TREG * GR_BLOCK; idx < nvec; idx += GR_BLOCK) lds[idx] = src[idx];
  __syncthreads();
}

// ------------------------------------------------------------- diagnostic stamps
// -DGR_STAMPS (diagnostic build only, scripts/stamps.py): lane 0 of every wave
// records s_memtime at phase boundaries and s_memrealtime at entry/exit into a
// buffer nothing else reads.  The product build compiles these away.
#ifdef GR_STAMPS
__device__ unsigned long long g_stamps[GR_STAMP_WAVES * GR_STAMP_SLOTS];
#define STAMP(k)                                                                              \
  do {                                                                                        \
    unsigned long long t_ = __builtin_amdgcn_s_memtime();                                    \
    const unsigned w_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                  \
    if ((threadIdx.x & 63) == 0 && w_ < GR_STAMP_WAVES) g_stamps[w_ * GR_STAMP_SLOTS + (k)] = t_; \
  } while (0)
#define RSTAMP(k)                                                                             \
  do {                                                                                        \
    unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                \
    const unsigned w_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);                  \
    if ((threadIdx.x & 63) == 0 && w_ < GR_STAMP_WAVES) g_stamps[w_ * GR_STAMP_SLOTS + (k)] = t_; \
  } while (0)
#else
#define STAMP(k)
#define RSTAMP(k)
#endif

// ------------------------------------------------------------- table slice view
struct Slice {
  Tab tab;
  const float4* src;  // global copy of this workgroup's slice
  int nvec;           // float4 in the slice
};

template <bool USE_LDS>
DEV Slice block_slice(const KArgs& a, const float4* lds) {
  // terrain types of this workgroup (type = floor(i / (N / T)), IL TerrainImporter layout),
  // derived on the host per workgroup: one scalar load
  const int bt = a.blk_types[blockIdx.x];
  const int t0 = bt & 0xffff, t1 = bt >> 16;
  Slice s;
  s.tab.L = a.h.num_levels;
  s.tab.G = a.h.max_gates;
  s.tab.stride = a.h.track_stride;
  s.tab.t0 = t0;
  s.src = reinterpret_cast<const float4*>(a.table + (size_t)t0 * s.tab.L * s.tab.stride);
  s.nvec = (t1 - t0 + 1) * s.tab.L * s.tab.stride / 4;
  s.tab.base = USE_LDS ? reinterpret_cast<const float*>(lds) : reinterpret_cast<const float*>(s.src);
  return s;
}

// ------------------------------------------------------------- reset / observe kernel
// gr_reset / gr_observe: observations for every env, reset for the masked ones.
template <int MODE, bool USE_LDS>
__global__ __launch_bounds__(GR_BLOCK) void env_kernel(KArgs a, const KConst* __restrict__ kc,
                                                        const uint8_t* __restrict__ mask) {
  a.kc = kc;
  extern __shared__ __attribute__((aligned(16))) float4 lds_tab[];
  const int n = a.h.num_envs;
  const int i = blockIdx.x * GR_BLOCK + threadIdx.x;
  const bool live = i < n;
  const int ii = live ? i : n - 1;  // dead lanes mirror the last env (loads stay in bounds, no stores)
  const uint32_t gid = gid_of(a, ii);
  const uint32_t cnt = a.buf.counters[a.buf.counter_index];
  Env e;
  load_env(a, ii, e);
  const Slice sl = block_slice<USE_LDS>(a, lds_tab);
  if (USE_LDS) {
    for (int idx = threadIdx.x; idx < sl.nvec; idx += GR_BLOCK) lds_tab[idx] = sl.src[idx];
    __syncthreads();
  }
  ObsNoise on;
  obs_noise(a, gid, cnt, on);
  if (threadIdx.x == 0 && blockIdx.x == 0) a.buf.counters[a.buf.counter_index ^ 1] = cnt + 1u;
  float lg[GR_LOG_SLOTS];
  for (int s = 0; s < GR_LOG_SLOTS; ++s) lg[s] = 0.0f;
  bool reset_lane = false;
  // last action and aux carry over from the previous observation
  const float4 lcv = reinterpret_cast<const float4*>(a.buf.prev_obs_critic)[(size_t)ii * 4 + 3];
  const float lc[4] = {lcv.x, lcv.y, lcv.z, lcv.w};
  const float aux = a.buf.prev_obs_aux[ii];
  if (MODE == KMODE_RESET && live && (mask == nullptr || mask[i])) {
    reset_lane = true;
    lg[GR_LOG_NRESET] = 1.0f;
    for (int k = 0; k < 7; ++k) lg[GR_LOG_EPSUM0 + k] = e.es[k];
    lg[GR_LOG_ACC] = (float)e.acc;
    lg[GR_LOG_M_ACTRATE] = e.mar;
    lg[GR_LOG_M_LINSPD] = norm3(e.v);
    lg[GR_LOG_M_ANGSPD] = norm3(e.w);
    lg[GR_LOG_T_TIMEOUT] = a.buf.prev_time_out[i] ? 1.0f : 0.0f;
    reset_env(a, sl.tab, e, gid);
  }
  if (live) {
    ObsRows o;
    compute_obs(a, sl.tab, e, gid, on, lc, o);
    store_obs_direct(a, i, o, aux);
    if (a.sink_policy) store_obs_sink(a, i, o);
    if (reset_lane) {
      store_dyn(a, i, e);
      store_rst(a, i, e);
      store_istate(a, i, e);
      // new position / level: the obstacle hint is stale
      reinterpret_cast<float4*>(a.buf.state)[GR_P_OHINT * (size_t)n + i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
  }
  // (observe calls reset nothing: their rows say so, and the finalized log repeats the previous one)
  const int w = threadIdx.x >> 6;
  wave_log(a, w, lg, reset_lane, live ? (float)e.lvl : 0.0f, live ? e.nl : 0.0f);
}

// ------------------------------------------------------------- the step kernel
// One workgroup = 256 envs and 12 waves in three roles (wave-uniform):
//   physics (waves 0-3):   controller, integrator, collision, termination -> handover;
//                          then reward, state planes, step outputs, reset logs
//   policy  (waves 4-7):   observation noise while the physics runs; then the noisy
//                          policy observation, per-env gate progress, level logs
//   episode (waves 8-11):  the next episode's start state for every env (a reset
//                          depends only on the episode bookkeeping, not on this
//                          step's physics) -> handover; then gate progress, the
//                          critic observation and the episode counters
// At 65 536 envs this puts three waves on every SIMD: a single wave issues a VALU
// op at most every 4 cycles (the SIMD could take one every 2), and the waves'
// memory / LDS / transcendental latencies overlap.  Two workgroup barriers: the
// LDS track slice (1), the physics handover (2).
// (ManagerBasedDiffRLEnv.step, manager_based_diff_rl_env.py:160-267.)
// handover rows (float4 per env), physics -> others: p + aux, q, v + done, lag, last ctbr;
// episode -> others: the next episode's start state (state-plane layout)
enum { X_PA = 0, X_Q = 1, X_VD = 2, X_LAG = 3, X_LC = 4, GR_XF4 = 5, GR_XF = 4 * GR_XF4 };
enum { R_POSQ = 0, R_QV = 1, R_VW = 2, R_W = 3, R_RST0 = 4, R_RST1 = 5, GR_RF4 = 6 };
enum { GR_SF4 = 8 };  // staging rows for the coalesced observation stores (policy 4, critic 4)
// obstacle rows (obstacle tracks only): physics -> policy the post-step position and attitude,
// policy -> physics the obstacle lattice mask; then one ready flag per wave pair
enum { O_P = 0, O_Q = 1, O_MASK = 2, GR_OF4 = 3 };

// environment as the policy / episode waves see it after the handover: the post-step pose,
// or for resetting envs the next episode's start state
DEV void merge_handover(const float4* xch, int t, bool reset, Env& e) {
  // (field-wise selects: branch-dependent writes to different fields made the compiler
  // address the struct through scratch memory)
  // every row is read unconditionally and merged by value selects: a conditional read let the compiler
  // select between the LDS row and the Env field's address, which put the Env's integers in scratch and
  // read them through a flat pointer on the post-handover path
  const float4 p4 = xch[X_PA * GR_BLOCK + t], q4 = xch[X_Q * GR_BLOCK + t], v4 = xch[X_VD * GR_BLOCK + t];
  const float4* xr = xch + GR_XF4 * GR_BLOCK;
  const float4 r0 = xr[R_POSQ * GR_BLOCK + t], r1 = xr[R_QV * GR_BLOCK + t], r2 = xr[R_VW * GR_BLOCK + t];
  const float4 r3 = xr[R_W * GR_BLOCK + t], r4 = xr[R_RST0 * GR_BLOCK + t];
  e.p[0] = reset ? r0.x : p4.x; e.p[1] = reset ? r0.y : p4.y; e.p[2] = reset ? r0.z : p4.z;
  e.q[0] = reset ? r0.w : q4.x; e.q[1] = reset ? r1.x : q4.y; e.q[2] = reset ? r1.y : q4.z;
  e.q[3] = reset ? r1.z : q4.w;
  e.v[0] = reset ? r1.w : v4.x; e.v[1] = reset ? r2.x : v4.y; e.v[2] = reset ? r2.y : v4.z;
  e.lvl = reset ? __float_as_int(r3.y) : e.lvl;
  e.gate = reset ? __float_as_int(r3.z) : e.gate;
  e.nl = reset ? r4.y : e.nl;
  e.acc = reset ? 0 : e.acc;
  e.ep = reset ? 0 : e.ep + 1;
  e.epoch = reset ? e.epoch + 1 : e.epoch;
  e.azero = reset ? 1 : 0;
}

#ifdef GR_STEP_MINB  // timing variants: minimum resident workgroups per CU (caps the VGPRs)
#define GR_STEP_LB __launch_bounds__(3 * GR_BLOCK, GR_STEP_MINB)
#else
#define GR_STEP_LB __launch_bounds__(3 * GR_BLOCK)
#endif
// MAXG > 0: tracks of at most MAXG gates (checked at launch).  The 8-gate instantiation (the reference's tracks,
// BASELINE C3 / C4) runs without scratch (the generic one spills 48 B / lane in its 32-gate sphere loop).
// LEAN: a configuration compiled in (the launch checks it): 1 = BASELINE C3 / C4 (explicit integrator, no motor model,
// no rotor-constant DR), 2 = C5's (the same with rotor-constant DR); 0 = every option read at run time
template <bool USE_LDS, bool OBST, int MAXG = 0, int LEAN = 0>
__global__ GR_STEP_LB void step_kernel(KArgs a, const KConst* __restrict__ kc,
                                                             const float* __restrict__ actions) {
  a.kc = kc;
  extern __shared__ __attribute__((aligned(16))) float4 lds[];
  float4* xch = lds + a.h.lds_tab_vec;                      // [GR_XF4 + GR_RF4][GR_BLOCK] handovers
  float4* stg = xch + (GR_XF4 + GR_RF4) * GR_BLOCK;         // [GR_SF4][GR_BLOCK] store staging
  float4* obx = stg + GR_SF4 * GR_BLOCK;                    // [GR_OF4][GR_BLOCK] obstacle hand-over (OBST)
  int* oflag = reinterpret_cast<int*>(obx + GR_OF4 * GR_BLOCK);  // [GR_BLOCK / 64] mask-ready flags (OBST)
  const int role = threadIdx.x / GR_BLOCK;                  // wave-uniform: 0 physics, 1 policy, 2 episode
  const int t = threadIdx.x & (GR_BLOCK - 1);
  const int n = a.h.num_envs;
  const int i = blockIdx.x * GR_BLOCK + t;
  const bool live = i < n;
  const int ii = live ? i : n - 1;  // dead lanes mirror the last env (loads stay in bounds, no stores)
  const gr_config& c = a.kc->cfg;
  const uint32_t gid = gid_of(a, ii);
  RSTAMP(9);
  STAMP(0);
  const Slice sl = block_slice<USE_LDS>(a, lds);
  // each of the 768 threads stages up to two float4 of the table slice, loaded at entry (clamped
  // loads; extras are not stored): a two-type slice of 8-gate tracks (820 float4) needs no load later
  float4 tr = make_float4(0.0f, 0.0f, 0.0f, 0.0f), tr2 = tr;
  const bool two = sl.nvec > 3 * GR_BLOCK;
  if (USE_LDS) {
    tr = sl.src[min((int)threadIdx.x, sl.nvec - 1)];
    if (two) tr2 = sl.src[min((int)threadIdx.x + 3 * GR_BLOCK, sl.nvec - 1)];
  }
  auto commit = [&]() {
    if (USE_LDS) {
      if ((int)threadIdx.x < sl.nvec) lds[threadIdx.x] = tr;
      if (two && (int)threadIdx.x + 3 * GR_BLOCK < sl.nvec) lds[threadIdx.x + 3 * GR_BLOCK] = tr2;
      for (int idx = threadIdx.x + 6 * GR_BLOCK; idx < sl.nvec; idx += 3 * GR_BLOCK) lds[idx] = sl.src[idx];
    }
    // barrier 1: table staged; with obstacles also the physics -> policy pose hand-over and the cleared flags
    if (USE_LDS || OBST) __syncthreads();
  };

  if (role == 0) {
    // ======================= physics waves =======================
    const float4 act = ld4(reinterpret_cast<const float4*>(actions), (size_t)ii);
    Env e;
    load_env(a, ii, e);
    const float dt = c.step_dt;
    const float v_prev[3] = {e.v[0], e.v[1], e.v[2]}, w_prev[3] = {e.w[0], e.w[1], e.w[2]};
    const float mar_prev = e.mar;
    // DiffActionManager.process_action + one-step lag.  The lag plane holds the
    // *squashed* previous action tanh(a_{t-1}): the reference only ever uses
    // tanh() of the lagged / previous raw action, so each action is squashed once.
    float th_cur[4], th_prev[4], th_raw[4];
    th_cur[0] = gr_tanhf(act.x); th_cur[1] = gr_tanhf(act.y); th_cur[2] = gr_tanhf(act.z); th_cur[3] = gr_tanhf(act.w);
    for (int k = 0; k < 4; ++k) {
      th_prev[k] = e.azero ? 0.0f : e.lag[k];
      th_raw[k] = c.action_lag ? e.lag[k] : th_cur[k];
      e.lag[k] = th_cur[k];
    }
    float sc[4], of[4], cmd[4];
    action_scale(a, e.mc, sc, of);
    for (int k = 0; k < 4; ++k) cmd[k] = th_raw[k] * sc[k] + of[k];
    cmd[0] = cmd[0] * e.thr;
    float tt[4];
    if (LEAN == 2 || (LEAN == 0 && a.h.dr_rotor)) {
      const float4 rk = reinterpret_cast<const float4*>(a.buf.state)[GR_P_ROTOR * (size_t)n + ii];
      ctbr_compute<LEAN != 0>(a, cmd, e.w, e.al, e.Kp, e.Kd, e.cT, e.ct, e.T, e.tau, e.mw, tt, &rk);
    } else {
      ctbr_compute<LEAN != 0>(a, cmd, e.w, e.al, e.Kp, e.Kd, e.cT, e.ct, e.T, e.tau, e.mw, tt);
    }
    const float m = c.dr_plant ? e.mp : e.mc;
    float Jp[3];
    for (int k = 0; k < 3; ++k) Jp[k] = c.dr_plant ? e.J[k] : c.inertia[k];
    float accl[3], al[3];
    int ccount = 0;
    if (LEAN != 0 || c.integrator == GR_INTEGRATOR_DD_EXPLICIT) {
      dd_explicit(m, Jp, e.k2, e.k1, tt, dt, c.gravity, e.p, e.q, e.v, e.w, accl, al);
      STAMP(3);
      if (OBST) {  // the policy waves test the obstacles on the post-step pose while this wave tests the gates
        obx[O_P * GR_BLOCK + t] = make_float4(e.p[0], e.p[1], e.p[2], 0.0f);
        obx[O_Q * GR_BLOCK + t] = make_float4(e.q[0], e.q[1], e.q[2], e.q[3]);
        if ((t & 63) == 0) oflag[t >> 6] = 0;
      }
      commit();  // barrier 1: the table is first needed by the collision test
      STAMP(14);
      uint32_t cm = collision_mask<false, MAXG>(a, sl.tab, e.type, e.lvl, e.p, e.q, ObstGrid{});
      STAMP(15);
      if (OBST) {
        // wait for the partner policy wave's obstacle mask (same 64 envs); it is resident and never waits on us
        // (bounded: a protocol bug must not hang the GPU; a wave that gives up raises GR_STATUS_OBST_WAIT_TIMEOUT
        // in the context's status word, which gr_device_status reports)
        int spin = 0;
        while (__hip_atomic_load(oflag + (t >> 6), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 &&
               spin < (1 << 22)) {
          __builtin_amdgcn_s_sleep(1);
          ++spin;
        }
        // the loop ends on the counter or on the flag: a flag that arrived on the last poll is not a timeout, so the
        // status is raised only when one more read still finds it clear (this read runs only past the limit)
        if (__builtin_expect(spin >= (1 << 22), 0) &&
            __hip_atomic_load(oflag + (t >> 6), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 && (t & 63) == 0)
          __hip_atomic_fetch_or(a.status, GR_STATUS_OBST_WAIT_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        cm |= (uint32_t)__float_as_int(obx[O_MASK * GR_BLOCK + t].x);
      }
      ccount = __builtin_popcount(cm);
    } else {
      ObstGrid og{};
      if (OBST) og = obst_grid(a, e.type, e.lvl);
      commit();  // barrier 1: contacts are tested every substep
      float vb[3], fb[3] = {0.0f, 0.0f, tt[0]};
      quat_rotate_inverse(e.q, e.v, vb);
      for (int k = 0; k < 3; ++k) fb[k] = (fb[k] - (e.k2[k] * vb[k]) * gr_fabsf(vb[k])) - e.k1[k] * vb[k];
      for (int s = 0; s < c.decimation; ++s) {
        si_substep(m, Jp, fb, tt + 1, c.sim_dt, c.gravity, e.p, e.q, e.v, e.w, accl, al);
        int cc = __builtin_popcount(collision_mask<OBST, MAXG>(a, sl.tab, e.type, e.lvl, e.p, e.q, og));
        ccount = cc > ccount ? cc : ccount;
      }
    }
    STAMP(4);
    for (int k = 0; k < 3; ++k) e.al[k] = al[k];
    // terminations first (termination.py:24-33, IL time_out / illegal contact): the observation
    // waves need `done` for the resets; the reward is computed after the handover, in their shadow
    e.ep += 1;
    const int time_out = e.ep >= c.max_episode_length;
    const int contact = ccount > c.collision_count_threshold;
    const float* rec = sl.tab.rec(e.type, e.lvl);
    const float zw = e.p[2] + rec[1];
    const int oob = (zw < c.out_of_bound[0]) | (zw > c.out_of_bound[1]);
    const int bad = (1.0f - 2.0f * (e.q[1] * e.q[1] + e.q[2] * e.q[2])) < 0.0f;
    const int c_term = c.stage == 0 ? oob : contact;
    const int terminated = (c.term_contact && c_term) | (c.term_bad_pose && bad);
    const float* g = sl.tab.gate(e.type, e.lvl, e.gate);
    float dg[3] = {g[0] - e.p[0], g[1] - e.p[1], g[2] - e.p[2]};
    const float dist = norm3(dg);
    const int near_gate = dist < c.gate_threshold;
    int done = terminated | time_out;
    float lc[4];
    for (int k = 0; k < 4; ++k) lc[k] = th_raw[k] * sc[k] + of[k];
    lc[0] = lc[0] / e.mc;
    // hand the post-step pose over to the observation waves
    xch[X_PA * GR_BLOCK + t] = make_float4(e.p[0], e.p[1], e.p[2], near_gate ? 1.0f : 0.0f);
    xch[X_Q * GR_BLOCK + t] = make_float4(e.q[0], e.q[1], e.q[2], e.q[3]);
    xch[X_VD * GR_BLOCK + t] = make_float4(e.v[0], e.v[1], e.v[2], done ? 1.0f : 0.0f);
    xch[X_LAG * GR_BLOCK + t] = make_float4(e.lag[0], e.lag[1], e.lag[2], e.lag[3]);
    xch[X_LC * GR_BLOCK + t] = make_float4(lc[0], lc[1], lc[2], lc[3]);
    STAMP(5);
    __syncthreads();  // barrier 2: handover
    // rewards (rewards.py:154-253), IL RewardManager: f * w * dt, declaration order
    float vb[3], gb[3];
    quat_rotate_inverse(e.q, e.v, vb);
    quat_rotate_inverse(e.q, dg, gb);
    float f[7];
    f[0] = cosine_similarity(vb, gb);
    float br[3];
    for (int k = 0; k < 3; ++k) br[k] = th_cur[k + 1] * sc[k + 1];
    f[1] = norm3(br);
    float sq[4];
    for (int k = 0; k < 4; ++k) {
      float dd = (th_cur[k] * sc[k] + of[k]) - (th_prev[k] * sc[k] + of[k]);
      sq[k] = dd * dd;
    }
    f[2] = ((sq[0] + sq[1]) + sq[2]) + sq[3];
    f[3] = (float)contact;
    float nb = gr_maxf(norm3(gb), 1e-12f);
    float gh[3] = {gb[0] / nb, gb[1] / nb, gb[2] / nb}, fx[3] = {1.0f, 0.0f, 0.0f};
    f[4] = cosine_similarity(gh, fx);
    f[5] = (float)near_gate * (1.0f / (dist * dist + 1.0f));
    f[6] = (float)bad;
    float rew = 0.0f;
    for (int k = 0; k < 7; ++k) {
      const float wk = a.kc->w[k];
      if (wk == 0.0f) continue;
      float v = (f[k] * wk) * dt;
      rew = rew + v;
      e.es[k] = e.es[k] + v;
    }
    e.mar = f[2];
    // episode metrics of the resetting envs (reward / termination / command managers' reset logs)
    float lg[GR_LOG_SLOTS];
    for (int s = 0; s < GR_LOG_SLOTS; ++s) lg[s] = 0.0f;
    const bool reset_lane = done && live;
    if (reset_lane) {
      for (int k = 0; k < 7; ++k) lg[GR_LOG_EPSUM0 + k] = e.es[k];
      lg[GR_LOG_NRESET] = 1.0f;
      lg[GR_LOG_ACC] = (float)e.acc;
      lg[GR_LOG_M_ACTRATE] = mar_prev;
      lg[GR_LOG_M_LINSPD] = norm3(v_prev);
      lg[GR_LOG_M_ANGSPD] = norm3(w_prev);
      lg[GR_LOG_T_TIMEOUT] = (float)time_out;
      lg[GR_LOG_T_CONTACT] = (float)c_term;
      lg[GR_LOG_T_BADPOSE] = (float)bad;
      // the next episode's start state, from the observation waves (events.py:139-177 et al.)
      const float4* xr = xch + GR_XF4 * GR_BLOCK;
      const float4 r0 = xr[R_POSQ * GR_BLOCK + t], r1 = xr[R_QV * GR_BLOCK + t], r2 = xr[R_VW * GR_BLOCK + t];
      const float4 r3 = xr[R_W * GR_BLOCK + t], r4 = xr[R_RST0 * GR_BLOCK + t], r5 = xr[R_RST1 * GR_BLOCK + t];
      e.p[0] = r0.x; e.p[1] = r0.y; e.p[2] = r0.z; e.q[0] = r0.w;
      e.q[1] = r1.x; e.q[2] = r1.y; e.q[3] = r1.z; e.v[0] = r1.w;
      e.v[1] = r2.x; e.v[2] = r2.y; e.w[0] = r2.z; e.w[1] = r2.w;
      e.w[2] = r3.x;
      e.lvl = __float_as_int(r3.y);
      e.gate = __float_as_int(r3.z);
      e.acc = 0;
      for (int k = 0; k < 3; ++k) { e.al[k] = 0.0f; e.tau[k] = 0.0f; }
      e.T = 0.0f;
      for (int k = 0; k < 4; ++k) e.mw[k] = 0.0f;
      for (int k = 0; k < 7; ++k) e.es[k] = 0.0f;
      e.mar = 0.0f;
      e.thr = r4.x; e.nl = r4.y; e.k2[0] = r4.z; e.k2[1] = r4.w;
      e.k2[2] = r5.x; e.k1[0] = r5.y; e.k1[1] = r5.z; e.k1[2] = r5.w;
    }
    if (live) {
      st1(a.buf.reward + i, rew);
      st1(a.buf.terminated + i, (uint8_t)terminated);
      st1(a.buf.time_out + i, (uint8_t)time_out);
      st1(a.buf.dones + i, (int64_t)(terminated | time_out));
      store_dyn(a, i, e);
      if (done) store_rst(a, i, e);
    }
    STAMP(12);
    // the level slots too (post-reset level / noise level are this lane's): the policy waves, whose tail is
    // the longest of the three roles, write no log row
    wave_log(a, threadIdx.x >> 6, lg, reset_lane, live ? (float)e.lvl : 0.0f, live ? e.nl : 0.0f);
    STAMP(8);
    RSTAMP(10);
  } else if (role == 1) {
    // ======================= policy-observation waves =======================
    const uint32_t cnt = a.buf.counters[a.buf.counter_index];
    const int4 is = reinterpret_cast<const int4*>(a.buf.istate)[ii];
    const float4 r0 = reinterpret_cast<const float4*>(a.buf.state)[GR_P_RST0 * (size_t)n + ii];
    Env e;
    e.ep = is.x; e.acc = is.y; e.epoch = is.z;
    e.gate = is.w & 0xff; e.lvl = (is.w >> 8) & 0xff; e.type = (is.w >> 24) & 0xff;
    e.nl = r0.y;
    ObsNoise on;
    float4 hint = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    ObstGrid og{};
    if constexpr (OBST) {
      // Obstacles (the physics waves' registers are full, these are idle until the handover): the records
      // of the hinted cell are fetched at entry, the test runs on the post-step pose after barrier 1.
      hint = reinterpret_cast<const float4*>(a.buf.state)[GR_P_OHINT * (size_t)n + ii];
      og = obst_grid(a, e.type, e.lvl);
      const int hfirst = __float_as_int(hint.x), hcount = __float_as_int(hint.y) - 1;
      float4 psp[GR_OBST_BATCH];  // cull spheres of the hinted list's first batch
      obst_spheres(a, hfirst, 0, hcount, psp);
      STAMP(1);
      commit();  // barrier 1
      STAMP(2);
      if (c.integrator == GR_INTEGRATOR_DD_EXPLICIT) {
        const float4 p4 = obx[O_P * GR_BLOCK + t], q4 = obx[O_Q * GR_BLOCK + t];
        const float pp[3] = {p4.x, p4.y, p4.z}, qq[4] = {q4.x, q4.y, q4.z, q4.w};
        float A[3], B[3], Cz[3];
        body_axes(a, qq, A, B, Cz);
        uint32_t om = 0u;
        if (obst_hint_holds(hint, pp, a.h.obst_span)) {
          om = obst_list(a, hfirst, hcount, psp, pp, A, B, Cz);
        } else {
          om = obst_lookup(a, og, pp, A, B, Cz);
        }
        obx[O_MASK * GR_BLOCK + t] = make_float4(__int_as_float((int)om), 0.0f, 0.0f, 0.0f);
        if ((t & 63) == 0 && a.h.test_fault != GR_FAULT_OBST_NO_SIGNAL)
          __hip_atomic_store(oflag + (t >> 6), 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      STAMP(12);
      obs_noise(a, gid, cnt, on);  // off the critical path: needed after barrier 2
    } else {
      commit();  // barrier 1 (joined at once: the physics and episode waves set its time)
      STAMP(1);
      // observation noise needs only the call counter: it runs while the physics waves collide
      obs_noise(a, gid, cnt, on);
      STAMP(2);
    }
    // call counter for the observation-noise stream: double-buffered by call parity,
    // so this write never races with the reads of the current launch
    if (t == 0 && blockIdx.x == 0) a.buf.counters[a.buf.counter_index ^ 1] = cnt + 1u;
    __syncthreads();  // barrier 2: handover
    STAMP(13);
    const float4 xvd = xch[X_VD * GR_BLOCK + t], xlc = xch[X_LC * GR_BLOCK + t];
    const float aux = xch[X_PA * GR_BLOCK + t].w;
    const bool reset = xvd.w != 0.0f && live;
    merge_handover(xch, t, reset, e);
    float4 next_hint = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if constexpr (OBST) {
      // the next step's hint: the cell list of the post-step (or the next episode's start) position; its loads
      // land while the policy row is computed
      const ObstGrid ogn = reset ? obst_grid(a, e.type, e.lvl) : og;
      next_hint = obst_hint_of(a, ogn, e.p);
    }
    const float lc[4] = {xlc.x, xlc.y, xlc.z, xlc.w};
    gate_advance(a, sl.tab, e);
    STAMP(7);
    {
      float4 prow[4];
      compute_policy(a, sl.tab, e, gid, on, lc, prow);
      store_rows_staged(reinterpret_cast<float4*>(a.buf.obs_policy), blockIdx.x * GR_BLOCK + (t & ~63), n, prow,
                        stg + (t & ~63));
      if (a.sink_policy) store_rows_sink(a, a.sink_policy, blockIdx.x * GR_BLOCK + (t & ~63), n, stg + (t & ~63));
      if (live) st1(a.buf.obs_aux + i, aux);
    }
    if (OBST && live) st4s(reinterpret_cast<float4*>(a.buf.state), GR_P_OHINT * (size_t)n + i, next_hint);
    STAMP(8);
    RSTAMP(10);
  } else {
    // ======================= episode waves =======================
    const float4* S = reinterpret_cast<const float4*>(a.buf.state);
    const size_t ns = (size_t)n;
    const int4 is = reinterpret_cast<const int4*>(a.buf.istate)[ii];
    const float4 r0 = S[GR_P_RST0 * ns + ii], r1 = S[GR_P_RST1 * ns + ii], p2 = S[GR_P_PAR2 * ns + ii];
    Env e;
    e.ep = is.x; e.acc = is.y; e.epoch = is.z;
    e.gate = is.w & 0xff; e.lvl = (is.w >> 8) & 0xff; e.type = (is.w >> 24) & 0xff;
    e.thr = r0.x; e.nl = r0.y; e.k2[0] = r0.z; e.k2[1] = r0.w;
    e.k2[2] = r1.x; e.k1[0] = r1.y; e.k1[1] = r1.z; e.k1[2] = r1.w;
    e.mc = p2.w;
    // the next episode's start state, for every env (only the resetting ones use it)
    ResetDraws rd;
    reset_draws(a, gid, (uint32_t)e.epoch + 1u, e.mc, rd);
    STAMP(1);
    commit();  // barrier 1 (the start gate of the next episode's track is read from the slice)
    STAMP(2);
    {
      Env er = e;
      reset_apply(a, sl.tab, er, rd);
      float4* xr = xch + GR_XF4 * GR_BLOCK;
      xr[R_POSQ * GR_BLOCK + t] = make_float4(er.p[0], er.p[1], er.p[2], er.q[0]);
      xr[R_QV * GR_BLOCK + t] = make_float4(er.q[1], er.q[2], er.q[3], er.v[0]);
      xr[R_VW * GR_BLOCK + t] = make_float4(er.v[1], er.v[2], er.w[0], er.w[1]);
      xr[R_W * GR_BLOCK + t] = make_float4(er.w[2], __int_as_float(er.lvl), __int_as_float(er.gate), 0.0f);
      xr[R_RST0 * GR_BLOCK + t] = make_float4(er.thr, er.nl, er.k2[0], er.k2[1]);
      xr[R_RST1 * GR_BLOCK + t] = make_float4(er.k2[2], er.k1[0], er.k1[1], er.k1[2]);
    }
    STAMP(6);
    __syncthreads();  // barrier 2: handover
    STAMP(13);
    const float4 xlc = xch[X_LC * GR_BLOCK + t];
    const bool reset = xch[X_VD * GR_BLOCK + t].w != 0.0f && live;
    merge_handover(xch, t, reset, e);
    const float lc[4] = {xlc.x, xlc.y, xlc.z, xlc.w};
    gate_advance(a, sl.tab, e);
    STAMP(14);
    if (live) store_istate(a, i, e);
    {  // critic observation (noise-free) of the post-reset, post-gate-progress state
      float4 crow[4];
      compute_critic(sl.tab, e, lc, crow);
      store_rows_staged(reinterpret_cast<float4*>(a.buf.obs_critic), blockIdx.x * GR_BLOCK + (t & ~63), n, crow,
                        stg + 4 * GR_BLOCK + (t & ~63));
      if (a.sink_critic)
        store_rows_sink(a, a.sink_critic, blockIdx.x * GR_BLOCK + (t & ~63), n, stg + 4 * GR_BLOCK + (t & ~63));
    }
    STAMP(8);
    RSTAMP(10);
  }
#ifdef GR_STAMPS
  if ((threadIdx.x & 63) == 0 && blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6) < GR_STAMP_WAVES) {
    unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_ID (hwreg 4), all 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));  // XCC_ID (hwreg 20), 16 bits
    g_stamps[(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * GR_STAMP_SLOTS + 11] =
        ((unsigned long long)xcc << 32) | hw;
  }
#endif
}

// ------------------------------------------------------------- init (startup events)
__global__ __launch_bounds__(GR_BLOCK) void init_kernel(KArgs a, const KConst* __restrict__ kc) {
  a.kc = kc;
  const int i = blockIdx.x * GR_BLOCK + threadIdx.x;
  const gr_config& c = a.kc->cfg;
  if (i >= c.num_envs) return;
  const uint32_t gid = gid_of(a, i);
  Env e;
  gr_u32x4 b0 = draw(a, gid, 0, GR_TAG_STATIC, 0), b1 = draw(a, gid, 0, GR_TAG_STATIC, 1);
  gr_u32x4 b2 = draw(a, gid, 0, GR_TAG_STATIC, 2), b3 = draw(a, gid, 0, GR_TAG_STATIC, 3);
  gr_u32x4 b4 = draw(a, gid, 0, GR_TAG_STATIC, 4);
  const int dr = c.dr_startup;
  float4 rotor = make_float4(c.thrustmap[0], c.thrustmap[1], c.thrustmap[2], c.kappa);
  if (dr && c.dr_rotor) {  // config C5: thrust map and kappa x U(lo, hi) per env, for the env's lifetime
    const gr_u32x4 b5 = draw(a, gid, 0, GR_TAG_STATIC, 5);
    const float lo = c.rotor_scale_range[0], hi = c.rotor_scale_range[1];
    rotor = make_float4(c.thrustmap[0] * gr_uniform(b5.x, lo, hi), c.thrustmap[1] * gr_uniform(b5.y, lo, hi),
                        c.thrustmap[2] * gr_uniform(b5.z, lo, hi), c.kappa * gr_uniform(b5.w, lo, hi));
  }
  const float plo = c.pid_scale_range[0], phi = c.pid_scale_range[1];
  const float dlo = c.delay_scale_range[0], dhi = c.delay_scale_range[1];
  float skp[3] = {gr_uniform(b0.x, plo, phi), gr_uniform(b0.y, plo, phi), gr_uniform(b0.z, plo, phi)};
  float skd[3] = {gr_uniform(b0.w, plo, phi), gr_uniform(b1.x, plo, phi), gr_uniform(b1.y, plo, phi)};
  float sdt = gr_uniform(b1.z, dlo, dhi);
  float sdq[3] = {gr_uniform(b1.w, dlo, dhi), gr_uniform(b2.x, dlo, dhi), gr_uniform(b2.y, dlo, dhi)};
  float madd = gr_uniform(b2.z, c.mass_add_range[0], c.mass_add_range[1]);
  float sj[3] = {gr_uniform(b2.w, c.inertia_scale_range[0], c.inertia_scale_range[1]),
                 gr_uniform(b3.x, c.inertia_scale_range[0], c.inertia_scale_range[1]),
                 gr_uniform(b3.y, c.inertia_scale_range[0], c.inertia_scale_range[1])};
  for (int k = 0; k < 3; ++k) {
    e.Kp[k] = dr ? c.rate_gain_p[k] * skp[k] : c.rate_gain_p[k];
    e.Kd[k] = dr ? c.rate_gain_d[k] * skd[k] : c.rate_gain_d[k];
  }
  float tauT = dr ? c.thrust_ctrl_delay * sdt : c.thrust_ctrl_delay;
  e.cT = gr_expf(-c.step_dt / tauT);
  for (int k = 0; k < 3; ++k) {
    float tq = dr ? c.torque_ctrl_delay[k] * sdq[k] : c.torque_ctrl_delay[k];
    e.ct[k] = gr_expf(-c.step_dt / tq);
  }
  e.mc = c.mass;
  float mp = (dr && c.dr_plant) ? c.mass + madd : c.mass;
  e.mp = mp;
  for (int k = 0; k < 3; ++k) e.J[k] = (dr && c.dr_plant) ? (c.inertia[k] * (mp / c.mass)) * sj[k] : c.inertia[k];
  e.lvl = (int)gr_floorf(gr_u01(b3.z) * (float)(c.max_init_level + 1));
  float z0, z1;
  gr_box_muller(b3.w, b4.x, &z0, &z1);
  e.thr = 1.0f + z0 * 0.02f;
  e.nl = 1.0f;
  for (int k = 0; k < 3; ++k) { e.k2[k] = c.drag2[k] * c.mass; e.k1[k] = c.drag1[k] * c.mass; }
  e.k2[2] = e.k2[2] * c.z_drag;
  e.k1[2] = e.k1[2] * c.z_drag;
  for (int k = 0; k < 3; ++k) { e.p[k] = c.spawn_pos[k]; e.v[k] = 0.0f; e.w[k] = 0.0f; e.al[k] = 0.0f; e.tau[k] = 0.0f; }
  e.q[0] = 1.0f; e.q[1] = e.q[2] = e.q[3] = 0.0f;
  e.T = 0.0f;
  for (int k = 0; k < 4; ++k) { e.lag[k] = 0.0f; e.mw[k] = 0.0f; }
  for (int k = 0; k < 7; ++k) e.es[k] = 0.0f;
  e.mar = 0.0f;
  e.ep = 0; e.acc = 0; e.epoch = 0; e.gate = 0; e.azero = 1;
  int type = 0;
  for (int t = 1; t < c.num_types; ++t) type += (i >= a.kc->type_start[t]);
  e.type = type;
  store_dyn(a, i, e);
  store_rst(a, i, e);
  store_istate(a, i, e);
  {  // startup-DR parameter planes (written once)
    float4* S = reinterpret_cast<float4*>(a.buf.state);
    const size_t n = (size_t)c.num_envs;
    S[GR_P_PAR0 * n + i] = make_float4(e.Kp[0], e.Kp[1], e.Kp[2], e.cT);
    S[GR_P_PAR1 * n + i] = make_float4(e.Kd[0], e.Kd[1], e.Kd[2], e.mp);
    S[GR_P_PAR2 * n + i] = make_float4(e.ct[0], e.ct[1], e.ct[2], e.mc);
    S[GR_P_PAR3 * n + i] = make_float4(e.J[0], e.J[1], e.J[2], 0.0f);
    S[GR_P_OHINT * n + i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // no obstacle hint
    S[GR_P_ROTOR * n + i] = rotor;
  }
  // initial observation buffers: last action = ctbr(0) (DiffActions._raw_actions starts at zero)
  float sc[4], of[4];
  action_scale(a, e.mc, sc, of);
  float4* C = reinterpret_cast<float4*>(a.buf.obs_critic) + (size_t)i * 4;
  float4* P = reinterpret_cast<float4*>(a.buf.obs_policy) + (size_t)i * 4;
  const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  float4 l4 = make_float4((gr_tanhf(0.0f) * sc[0] + of[0]) / e.mc, gr_tanhf(0.0f) * sc[1] + of[1],
                          gr_tanhf(0.0f) * sc[2] + of[2], gr_tanhf(0.0f) * sc[3] + of[3]);
  C[0] = z4; C[1] = z4; C[2] = z4; C[3] = l4;
  P[0] = z4; P[1] = z4; P[2] = z4; P[3] = l4;
  a.buf.obs_aux[i] = 0.0f;
  a.buf.reward[i] = 0.0f;
  a.buf.terminated[i] = 0;
  a.buf.time_out[i] = 0;
  a.buf.dones[i] = 0;
}

// ------------------------------------------------------------- log finalize (on demand)
// Sums the per-wave rows of one call's log slab and forms the means Isaac Lab's
// managers log (RewardManager.reset: episode sum / episode_length_s; command
// metrics and curriculum: means; termination terms: counts).  No env reset in
// that call -> the previous values are kept (the reference leaves extras["log"]
// untouched).  One 256-thread workgroup, all loads issued before any reduction.
__global__ __launch_bounds__(256) void log_finalize_kernel(const float* __restrict__ rows, int nrows,
                                                           const float* __restrict__ prev, float* __restrict__ out,
                                                           float ep_len_s, float num_envs) {
  __shared__ float red[GR_LOG_SLOTS][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc[GR_LOG_SLOTS];
  for (int s = 0; s < GR_LOG_SLOTS; ++s) acc[s] = 0.0f;
  for (int r = threadIdx.x; r < nrows; r += 256) {
    const float4* row = reinterpret_cast<const float4*>(rows + (size_t)r * GR_LOG_SLOTS);
    float4 v0 = row[0], v1 = row[1], v2 = row[2], v3 = row[3], v4 = row[4];
    float v[GR_LOG_SLOTS] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w, v2.x, v2.y,
                             v2.z, v2.w, v3.x, v3.y, v3.z, v3.w, v4.x, v4.y, v4.z, v4.w};
    for (int s = 0; s < GR_LOG_SLOTS; ++s) acc[s] += v[s];
  }
  for (int s = 0; s < GR_LOG_SLOTS; ++s) {
    float v = acc[s];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) red[s][wave] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t[GR_LOG_SLOTS];
    for (int s = 0; s < GR_LOG_SLOTS; ++s) t[s] = ((red[s][0] + red[s][1]) + red[s][2]) + red[s][3];
    const float nr = t[GR_LOG_NRESET];
    if (nr == 0.0f && prev != nullptr) {
      for (int s = 0; s < GR_LOG_SLOTS; ++s) out[s] = prev[s];
      return;
    }
    for (int s = 0; s < GR_LOG_SLOTS; ++s) out[s] = t[s];
    for (int k = 0; k < 7; ++k) out[GR_LOG_EPSUM0 + k] = t[GR_LOG_EPSUM0 + k] / nr / ep_len_s;
    for (int k = GR_LOG_ACC; k <= GR_LOG_M_ANGSPD; ++k) out[k] = t[k] / nr;
    out[GR_LOG_LEVEL] = t[GR_LOG_LEVEL] / num_envs;
    out[GR_LOG_NOISE] = t[GR_LOG_NOISE] / num_envs;
  }
}

// ------------------------------------------------------------- test kernels
__global__ void test_dynamics_kernel(KArgs a, const KConst* __restrict__ kc, int n, int mode, const float* si,
                                     const float* ab, const float* cmd, const float* ci, const float* par,
                                     const float* drag, float* so, float* co, float* xo) {
  a.kc = kc;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float p[3], q[4], v[3], w[3], acc[3], al[3], tt[4], T = ci[i * 4], tau[3] = {ci[i * 4 + 1], ci[i * 4 + 2], ci[i * 4 + 3]};
  float mw[4] = {0, 0, 0, 0};
  for (int k = 0; k < 3; ++k) { p[k] = si[i * 13 + k]; v[k] = si[i * 13 + 7 + k]; w[k] = si[i * 13 + 10 + k]; }
  for (int k = 0; k < 4; ++k) q[k] = si[i * 13 + 3 + k];
  const float* pr = par + i * 16;
  float mot[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (mode == 0) {
    ctbr_compute(a, cmd + i * 4, w, ab + i * 3, pr + 0, pr + 4, pr[3], pr + 8, T, tau, mw, tt);
    for (int k = 0; k < 4; ++k) mot[k] = tt[k];
  } else if (mode == 2) {  // ThrustController.update alone: cmd = desired rotor thrusts
    for (int k = 0; k < 4; ++k) { mot[k] = cmd[i * 4 + k]; tt[k] = 0.0f; }
    MotorK mk;
    motor_consts(a, nullptr, mk);
    motor_update(a, mk, mot, mw);
  } else {
    for (int k = 0; k < 4; ++k) tt[k] = cmd[i * 4 + k];
  }
  dd_explicit(pr[7], pr + 12, drag + i * 6, drag + i * 6 + 3, tt, a.kc->cfg.step_dt, a.kc->cfg.gravity, p, q, v, w, acc, al);
  for (int k = 0; k < 3; ++k) { so[i * 13 + k] = p[k]; so[i * 13 + 7 + k] = v[k]; so[i * 13 + 10 + k] = w[k]; }
  for (int k = 0; k < 4; ++k) so[i * 13 + 3 + k] = q[k];
  co[i * 4] = T;
  for (int k = 0; k < 3; ++k) co[i * 4 + 1 + k] = tau[k];
  float ww[3];
  quat_rotate(q, w, ww);
  for (int k = 0; k < 3; ++k) { xo[i * 13 + k] = acc[k]; xo[i * 13 + 3 + k] = al[k]; xo[i * 13 + 6 + k] = ww[k]; }
  for (int k = 0; k < 4; ++k) xo[i * 13 + 9 + k] = mot[k];
}

__global__ void test_math_kernel(int fn, int n, const float* x, const float* y, float* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s, c;
  switch (fn) {
    case 0: out[i] = gr_expf(x[i]); break;
    case 1: out[i] = gr_tanhf(x[i]); break;
    case 2: out[i] = gr_logf(x[i]); break;
    case 3: gr_sincosf(x[i], &s, &c); out[i] = s; break;
    case 4: gr_sincosf(x[i], &s, &c); out[i] = c; break;
    case 5: out[i] = gr_atan2f(x[i], y[i]); break;
    case 6: out[i] = gr_sqrtf(x[i]); break;
    default: out[i] = x[i] / y[i]; break;
  }
}

__global__ void test_philox_kernel(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                   uint32_t k1, uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  gr_u32x4 r = gr_philox4x32_10(c0 + (uint32_t)i, c1, c2, c3, k0, k1);
  out[i * 4] = r.x; out[i * 4 + 1] = r.y; out[i * 4 + 2] = r.z; out[i * 4 + 3] = r.w;
}

// ------------------------------------------------------------- launchers
static int grid_of(int n) { return (n + GR_BLOCK - 1) / GR_BLOCK; }

int step_variant(const KArgs& a) {
  const bool lean = a.h.integrator == GR_INTEGRATOR_DD_EXPLICIT && !a.h.use_motor_model && !a.h.dr_rotor;
  if (a.obst_items != nullptr) return lean ? GR_STEP_OBST_LEAN : GR_STEP_OBST;
  if (a.h.lds_tab_vec <= 0) return GR_STEP_L2;
  if (a.h.max_gates <= 8) return lean ? GR_STEP_LDS8_LEAN : GR_STEP_LDS8;
  return GR_STEP_LDS;
}

template <int MODE>
static hipError_t launch_env_mode(const KArgs& a, const float* actions, const uint8_t* mask, hipStream_t s) {
  const int g = grid_of(a.h.num_envs);
  const bool lds = a.h.lds_tab_vec > 0;
  if constexpr (MODE == KMODE_STEP) {
    const int v = step_variant(a);
    if (v == GR_STEP_OBST_LEAN || v == GR_STEP_OBST) {
      // Obstacle tracks read the (L2-resident) track table directly: the workgroup barrier stays for the pose
      // hand-over, and without the slice staging a launch takes 12.3 us instead of 13.1 (65 536 envs).
      // Gate-only tracks time the same either way (9.8-9.9 us) and keep the LDS slice.
      KArgs b = a;
      b.h.lds_tab_vec = 0;
      const size_t bytes = (size_t)(GR_XF4 + GR_RF4 + GR_SF4 + GR_OF4) * GR_BLOCK * 16 + 16;
      // (the 8-gate instantiation, 28 B of scratch instead of 64, measured 0.15 us slower here: gpurun_out/o8.txt; the
      // lean one, C3's configuration compiled in, 12.14-12.17 vs 12.74-12.76 us: gpurun_out/olean.txt)
      if (v == GR_STEP_OBST_LEAN)
        hipLaunchKernelGGL((step_kernel<false, true, 0, 1>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, b, b.kc, actions);
      else
        hipLaunchKernelGGL((step_kernel<false, true>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, b, b.kc, actions);
    } else {
      const size_t bytes = (size_t)a.h.lds_tab_vec * 16 + (size_t)(GR_XF4 + GR_RF4 + GR_SF4) * GR_BLOCK * 16;
      // tracks of <= 8 gates (the reference's tracks, BASELINE C3 / C4): the sphere pass unrolled to a fixed 8, no
      // scratch (same time as the generic kernel: 9.88-9.98 vs 9.82-9.98 us, gpurun_out/g8.txt)
      if (v == GR_STEP_LDS8_LEAN)
        hipLaunchKernelGGL((step_kernel<true, false, 8, 1>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, a, a.kc, actions);
      // (C5's configuration compiled in, LEAN = 2 on 32-gate tracks with rotor DR: 11.83-11.93 vs 11.77-11.93 us,
      // gpurun_out/c5l.jsonl; not launched)
      else if (v == GR_STEP_LDS8)
        hipLaunchKernelGGL((step_kernel<true, false, 8>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, a, a.kc, actions);
      else if (v == GR_STEP_LDS)
        hipLaunchKernelGGL((step_kernel<true, false>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, a, a.kc, actions);
      else
        hipLaunchKernelGGL((step_kernel<false, false>), dim3(g), dim3(3 * GR_BLOCK), bytes, s, a, a.kc, actions);
    }
  } else {
    const size_t bytes = (size_t)a.h.lds_tab_vec * 16;
    if (lds)
      hipLaunchKernelGGL((env_kernel<MODE, true>), dim3(g), dim3(GR_BLOCK), bytes, s, a, a.kc, mask);
    else
      hipLaunchKernelGGL((env_kernel<MODE, false>), dim3(g), dim3(GR_BLOCK), 0, s, a, a.kc, mask);
  }
  return hipGetLastError();
}

hipError_t launch_env(int mode, const KArgs& a, const float* actions, const uint8_t* mask, hipStream_t s,
                      hipEvent_t t0, hipEvent_t t1) {
  hipError_t err;
  if (t0) {
    err = hipEventRecord(t0, s);
    if (err != hipSuccess) return err;
  }
  if (mode == KMODE_STEP) err = launch_env_mode<KMODE_STEP>(a, actions, mask, s);
  else if (mode == KMODE_RESET) err = launch_env_mode<KMODE_RESET>(a, actions, mask, s);
  else err = launch_env_mode<KMODE_OBSERVE>(a, actions, mask, s);
  if (err != hipSuccess) return err;
  if (t1) err = hipEventRecord(t1, s);
  return err;
}

hipError_t launch_log_finalize(const float* rows, int nrows, const float* prev, float* out, float ep_len_s,
                               float num_envs, hipStream_t s) {
  hipLaunchKernelGGL(log_finalize_kernel, dim3(1), dim3(256), 0, s, rows, nrows, prev, out, ep_len_s, num_envs);
  return hipGetLastError();
}

hipError_t launch_init(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(init_kernel, dim3(grid_of(a.h.num_envs)), dim3(GR_BLOCK), 0, s, a, a.kc);
  return hipGetLastError();
}

hipError_t launch_test_dynamics(const KArgs& a, int n, int mode, const float* si, const float* ab, const float* cmd,
                                const float* ci, const float* par, const float* drag, float* so, float* co, float* xo,
                                hipStream_t s) {
  hipLaunchKernelGGL(test_dynamics_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a, a.kc, n, mode, si, ab, cmd, ci,
                     par, drag, so, co, xo);
  return hipGetLastError();
}

hipError_t launch_test_math(int fn, int n, const float* x, const float* y, float* out, hipStream_t s) {
  hipLaunchKernelGGL(test_math_kernel, dim3((n + 255) / 256), dim3(256), 0, s, fn, n, x, y, out);
  return hipGetLastError();
}

hipError_t launch_test_philox(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                              uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(test_philox_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, c0, c1, c2, c3, k0, k1, out);
  return hipGetLastError();
}

hipError_t allow_large_lds() {
  const void* ks[] = {reinterpret_cast<const void*>(&step_kernel<true, false>),
                      reinterpret_cast<const void*>(&step_kernel<true, false, 8>),
                      reinterpret_cast<const void*>(&step_kernel<true, false, 8, 1>),
                      reinterpret_cast<const void*>(&step_kernel<false, true, 0, 1>),
                      reinterpret_cast<const void*>(&env_kernel<KMODE_RESET, true>),
                      reinterpret_cast<const void*>(&env_kernel<KMODE_OBSERVE, true>)};
  for (const void* k : ks) {
    hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, GR_LDS_MAX);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t read_stamps(unsigned long long* host, int n) {
#ifdef GR_STAMPS
  if (n > GR_STAMP_WAVES * GR_STAMP_SLOTS) n = GR_STAMP_WAVES * GR_STAMP_SLOTS;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost);
#else
  (void)host;
  (void)n;
  return hipErrorNotSupported;
#endif
}

}  // namespace gr
