/*
 * gr_rng.h — counter-based RNG (Philox4x32-10, Salmon et al. SC'11) and the
 * mapping of its words to the uniform / Gaussian draws the racing env needs.
 *
 * Every random draw of the env step is a pure function of
 *   key     = (seed_lo, seed_hi)
 *   counter = (global env id, epoch-or-step, stream tag, block index)
 * so the HIP kernel, the CPU oracle and any number of ranks reproduce the same
 * stream without storing RNG state in HBM (the reference uses torch's stateful
 * generator; its exact stream is not reproducible anyway — see DESIGN.md).
 * Shared verbatim by the kernel and the oracle; compiles as C and HIP C++.
 */
#ifndef GR_RNG_H
#define GR_RNG_H

#include "gr_math.h"

typedef struct { uint32_t x, y, z, w; } gr_u32x4;

GR_HD gr_u32x4 gr_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                uint32_t k0, uint32_t k1) {
#if defined(__HIP_DEVICE_COMPILE__)
  /* opaque key: the round-key schedule is recomputed per draw (two scalar adds per
   * round) instead of being shared across every inlined draw and kept live in SGPRs */
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
  /* fully unrolled: 262 vs 647 cycles per draw, and independent draws interleave
   * (4 draws: ~175 cycles each) — tools/mathbench.hip on gfx950 */
#pragma unroll
#endif
  for (int i = 0; i < 10; ++i) {
    uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  gr_u32x4 r = {c0, c1, c2, c3};
  return r;
}

/* Four draws that differ only in the last counter word, rounds interleaved so the
 * four dependency chains overlap (same words as four gr_philox4x32_10 calls). */
GR_HD void gr_philox4x32_10_x4(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                               gr_u32x4 out[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
#endif
  uint32_t x0[4], x1[4], x2[4], x3[4];
  for (int j = 0; j < 4; ++j) { x0[j] = c0; x1[j] = c1; x2[j] = c2; x3[j] = c3 + (uint32_t)j; }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
  for (int i = 0; i < 10; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int j = 0; j < 4; ++j) {
      uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)x0[j];
      uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)x2[j];
      uint32_t n0 = (uint32_t)(p1 >> 32) ^ x1[j] ^ k0;
      uint32_t n2 = (uint32_t)(p0 >> 32) ^ x3[j] ^ k1;
      x1[j] = (uint32_t)p1; x3[j] = (uint32_t)p0; x0[j] = n0; x2[j] = n2;
    }
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  for (int j = 0; j < 4; ++j) { out[j].x = x0[j]; out[j].y = x1[j]; out[j].z = x2[j]; out[j].w = x3[j]; }
}

/* uniform in [0, 1): 24 random bits, exact in fp32 */
GR_HD float gr_u01(uint32_t w) { return (float)(w >> 8) * 5.9604645e-08f; }
/* uniform in (0, 1]: for log() in Box-Muller */
GR_HD float gr_u01_open0(uint32_t w) { return (float)((w >> 8) + 1u) * 5.9604645e-08f; }
/* torch-style  U(lo, hi) = u * (hi - lo) + lo  (Isaac Lab sample_uniform op order) */
GR_HD float gr_uniform(uint32_t w, float lo, float hi) { return gr_u01(w) * (hi - lo) + lo; }

/* Box-Muller: two standard normals from two words */
GR_HD void gr_box_muller(uint32_t w0, uint32_t w1, float* z0, float* z1) {
  float u1 = gr_u01_open0(w0);
  float u2 = gr_u01(w1);
  float rad = gr_sqrtf(-2.0f * gr_logf(u1));
  float s, c;
  gr_sincosf(6.28318548f * u2, &s, &c);
  *z0 = rad * c;
  *z1 = rad * s;
}

/* Six 21-bit fields from one 128-bit draw (bits 0..125; 126-127 unused).  The
 * per-step streams take 21-bit uniforms so one Philox block feeds six draws
 * (a block costs ~650 cycles on gfx950, tools/mathbench.hip). */
GR_HD void gr_fields6(gr_u32x4 r, uint32_t f[6]) {
  f[0] = r.x & 0x1FFFFFu;
  f[1] = (r.x >> 21) | ((r.y & 0x3FFu) << 11);
  f[2] = (r.y >> 10) & 0x1FFFFFu;
  f[3] = (r.y >> 31) | ((r.z & 0xFFFFFu) << 1);
  f[4] = (r.z >> 20) | ((r.w & 0x1FFu) << 12);
  f[5] = (r.w >> 9) & 0x1FFFFFu;
}
/* uniform in [0, 1) / (0, 1] from a 21-bit field (exact in fp32) */
GR_HD float gr_f21(uint32_t f) { return (float)f * 4.76837158e-07f; }
GR_HD float gr_f21_open0(uint32_t f) { return (float)(f + 1u) * 4.76837158e-07f; }
/* torch-style U(lo, hi) = u * (hi - lo) + lo */
GR_HD float gr_uniform21(uint32_t f, float lo, float hi) { return gr_f21(f) * (hi - lo) + lo; }
/* Box-Muller from two 21-bit fields (radius tail truncated at 5.4 sigma) */
GR_HD void gr_box_muller21(uint32_t f1, uint32_t f2, float* z0, float* z1) {
  float u1 = gr_f21_open0(f1);
  float u2 = gr_f21(f2);
  float rad = gr_sqrtf(-2.0f * gr_logf(u1));
  float s, c;
  gr_sincosf(6.28318548f * u2, &s, &c);
  *z0 = rad * c;
  *z1 = rad * s;
}

/* A standard normal from the top 24 bits of one word, by the inverse CDF: u = (n + 0.5) / 2^24, z = Phi^-1(u), read
 * off the cubic table of gr_normal_table.h (`tab`: GR_NORMAL_TABLE_ENTRIES x 4 floats, generated and checked by
 * scripts/gen_normal_table.py: |z - Phi^-1(u)| <= 4.4e-7 over every n; |z| <= 5.42).  ~20 ALU ops, one float4 read and
 * three fmas per normal, branch-free; Box-Muller's log, sqrt and sincos cost ~3x that per normal. */
GR_HD float gr_normal24(uint32_t w, const float* tab) {
  const uint32_t n = w >> 8;
  const uint32_t up = n >> 23;                  /* u > 1/2: z > 0 */
  const uint32_t m = up ? 0xFFFFFFu - n : n;    /* the distance from the nearer end, [0, 2^23) */
  const uint32_t b = gr_f2u((float)m);          /* exact: m < 2^24 */
  const int small = m < 16u;                    /* entries 0..15: one constant per m */
  const uint32_t idx = small ? m : (b >> 19) - ((127u + 3u) << 4);  /* 16 (octave - 3) + top 4 mantissa bits */
  const float t = small ? 0.0f : (float)(b & 0x7FFFFu) * 1.9073486328125e-06f;  /* the other 19 bits / 2^19 */
  const float* c = tab + 4 * idx;
  const float g = gr_fmaf(gr_fmaf(gr_fmaf(c[3], t, c[2]), t, c[1]), t, c[0]);
  return up ? g : -g;
}

/* A standard normal from a 21-bit field (gr_fields6): the field widened to the 24 bits gr_normal24 reads, u = (f +
 * 0.5625) / 2^21 (|z| <= 5.01).  The step's observation noise: six normals from one Philox block, ~3x cheaper than
 * three gr_box_muller21 pairs and off the kernel's dependency chain sooner. */
GR_HD float gr_normal21(uint32_t f, const float* tab) { return gr_normal24((f << 11) | 0x400u, tab); }

/* stream tags (counter word 2) */
#define GR_TAG_STATIC 0x53544154u /* startup DR: gains, delays, mass, inertia, initial level */
#define GR_TAG_RESET 0x52535421u  /* per-episode reset draws, counter1 = epoch */
#define GR_TAG_GATE 0x47415445u   /* gate-pose noise, counter1 = epoch, counter3 = gates passed */
#define GR_TAG_OBS 0x4f425321u    /* observation noise, counter1 = call counter */
#define GR_TAG_IMG 0x494d4721u    /* depth-image noise, counter1 = call counter, counter3 = pixel quad */
#define GR_TAG_POLICY 0x504f4c21u /* action sampling of the fused policy inference, counter1 = call counter */

#endif /* GR_RNG_H */
