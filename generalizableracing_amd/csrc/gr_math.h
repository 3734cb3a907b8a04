/*
 * gr_math.h — portable fp32 elementary functions (exp, tanh, log, sincos,
 * atan2) built only from IEEE-754 correctly-rounded +,-,*,/ and sqrt.
 *
 * Polynomial steps use an explicit fused multiply-add (gr_fmaf), correctly rounded
 * on both sides, so they stay bit-identical with -ffp-contract=off elsewhere.
 *
 * Why this exists: the env step draws Gaussian noise (Box-Muller: log, sin,
 * cos), squashes actions (tanh) and samples reset yaw (atan2).  If the HIP
 * kernel used the device's hardware approximations (v_exp_f32, v_sin_f32 …)
 * and the CPU oracle used glibc, the two would disagree in the last ulp and
 * the parity suite could only assert tolerances.  With these functions, and
 * both sides compiled with -ffp-contract=off (and HIP's default
 * correctly-rounded fp32 divide/sqrt), kernel and oracle are bit-identical.
 *
 * Accuracy (checked in tests/test_math.py against float64): <= 4 ulp over the
 * ranges the env uses.  The header compiles as C (gcc, oracle) and HIP C++.
 */
#ifndef GR_MATH_H
#define GR_MATH_H

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define GR_HD static __host__ __device__ inline __attribute__((always_inline))
#else
#define GR_HD static inline
#endif

GR_HD uint32_t gr_f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
GR_HD float gr_u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
GR_HD float gr_fabsf(float x) { return gr_u2f(gr_f2u(x) & 0x7fffffffu); }
GR_HD float gr_copysignf(float m, float s) {
  return gr_u2f((gr_f2u(m) & 0x7fffffffu) | (gr_f2u(s) & 0x80000000u));
}
GR_HD float gr_sqrtf(float x) { return __builtin_sqrtf(x); }
/* fused multiply-add, correctly rounded on both sides (v_fma_f32 / x86 vfmadd, the
 * oracle is built with -mfma): one rounding per polynomial step, half the instructions */
GR_HD float gr_fmaf(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
GR_HD float gr_floorf(float x) { return __builtin_floorf(x); }
GR_HD float gr_minf(float a, float b) { return a < b ? a : b; }
GR_HD float gr_maxf(float a, float b) { return a > b ? a : b; }
/* torch.clamp(x, lo, hi) for non-NaN x */
GR_HD float gr_clampf(float x, float lo, float hi) { return gr_minf(gr_maxf(x, lo), hi); }

/* 2^k for k in [-126, 127] */
GR_HD float gr_exp2i(int k) { return gr_u2f((uint32_t)(k + 127) << 23); }

/* e^x, |error| <= 2 ulp on [-87, 88]; 0 below, clamps above. */
GR_HD float gr_expf(float x) {
  if (x < -87.0f) return 0.0f;
  if (x > 88.0f) x = 88.0f;
  float kf = gr_floorf(gr_fmaf(x, 1.44269502f, 0.5f));
  int k = (int)kf;
  float r = gr_fmaf(-kf, 3.19461833e-05f, gr_fmaf(-kf, 0.693115234375f, x)); /* Cody-Waite ln2 */
  float p = 1.98412698e-04f;                                                 /* 1/5040 */
  p = gr_fmaf(p, r, 1.38888889e-03f);                                        /* 1/720 */
  p = gr_fmaf(p, r, 8.33333333e-03f);                                        /* 1/120 */
  p = gr_fmaf(p, r, 4.16666667e-02f);                                        /* 1/24 */
  p = gr_fmaf(p, r, 1.66666667e-01f);                                        /* 1/6 */
  p = gr_fmaf(p, r, 0.5f);
  p = gr_fmaf(p, r, 1.0f);
  p = gr_fmaf(p, r, 1.0f);
  return p * gr_exp2i(k);
}

/* tanh(x), <= 4 ulp */
GR_HD float gr_tanhf(float x) {
  float ax = gr_fabsf(x);
  float r;
  if (ax < 0.3f) {
    float x2 = x * x;
    float p = -8.86323552e-03f;          /* -1382/155925 */
    p = gr_fmaf(p, x2, 2.18694885e-02f); /* 62/2835 */
    p = gr_fmaf(p, x2, -5.39682540e-02f); /* -17/315 */
    p = gr_fmaf(p, x2, 1.33333333e-01f); /* 2/15 */
    p = gr_fmaf(p, x2, -3.33333333e-01f); /* -1/3 */
    return gr_fmaf(x, x2 * p, x);
  }
  if (ax > 9.0f) {
    r = 1.0f;
  } else {
    float e = gr_expf(2.0f * ax);
    r = 1.0f - 2.0f / (e + 1.0f);
  }
  return gr_copysignf(r, x);
}

/* natural log for finite x > 0 (normal range), <= 2 ulp */
GR_HD float gr_logf(float x) {
  uint32_t u = gr_f2u(x);
  int e = (int)((u >> 23) & 0xffu) - 127;
  float m = gr_u2f((u & 0x007fffffu) | 0x3f800000u); /* [1,2) */
  if (m > 1.41421356f) { m = m * 0.5f; e = e + 1; }
  float f = (m - 1.0f) / (m + 1.0f);
  float f2 = f * f;
  float s = 1.53846154e-01f;             /* 2/13 */
  s = gr_fmaf(s, f2, 1.81818182e-01f);   /* 2/11 */
  s = gr_fmaf(s, f2, 2.22222222e-01f);   /* 2/9 */
  s = gr_fmaf(s, f2, 2.85714286e-01f);   /* 2/7 */
  s = gr_fmaf(s, f2, 4.00000000e-01f);   /* 2/5 */
  s = gr_fmaf(s, f2, 6.66666667e-01f);   /* 2/3 */
  float ef = (float)e;
  float lo = gr_fmaf(f, f2 * s, ef * 3.19461833e-05f);
  return gr_fmaf(ef, 0.693115234375f, 2.0f * f) + lo;
}

/* sin and cos of x for |x| < ~1e3 (Cody-Waite by pi/2), <= 2 ulp away from 0 */
GR_HD void gr_sincosf(float x, float* s_out, float* c_out) {
  float kf = gr_floorf(gr_fmaf(x, 0.636619747f, 0.5f));
  int k = (int)kf;
  float r = gr_fmaf(-kf, 7.54979013e-08f, gr_fmaf(-kf, 4.83751297e-04f, gr_fmaf(-kf, 1.5703125f, x)));
  float r2 = r * r;
  float sp = 2.75573192e-06f;            /* 1/9! */
  sp = gr_fmaf(sp, r2, -1.98412698e-04f); /* -1/7! */
  sp = gr_fmaf(sp, r2, 8.33333333e-03f); /* 1/5! */
  sp = gr_fmaf(sp, r2, -1.66666667e-01f); /* -1/3! */
  float s = gr_fmaf(r, r2 * sp, r);
  float cp = -2.75573192e-07f;           /* -1/10! */
  cp = gr_fmaf(cp, r2, 2.48015873e-05f); /* 1/8! */
  cp = gr_fmaf(cp, r2, -1.38888889e-03f); /* -1/6! */
  cp = gr_fmaf(cp, r2, 4.16666667e-02f); /* 1/4! */
  cp = gr_fmaf(cp, r2, -0.5f);
  float c = gr_fmaf(r2, cp, 1.0f);
  switch (k & 3) {
    case 0: *s_out = s; *c_out = c; break;
    case 1: *s_out = c; *c_out = -s; break;
    case 2: *s_out = -s; *c_out = -c; break;
    default: *s_out = -c; *c_out = s; break;
  }
}

/* atan(t) for 0 <= t <= 1 */
GR_HD float gr_atan_unit(float t) {
  float base = 0.0f;
  if (t > 0.414213562f) { /* atan(t) = pi/4 + atan((t-1)/(t+1)) */
    t = (t - 1.0f) / (t + 1.0f);
    base = 0.785398163f;
  }
  float t2 = t * t;
  float p = -4.76190476e-02f;            /* -1/21 */
  p = gr_fmaf(p, t2, 5.26315789e-02f);   /* 1/19 */
  p = gr_fmaf(p, t2, -5.88235294e-02f);  /* -1/17 */
  p = gr_fmaf(p, t2, 6.66666667e-02f);   /* 1/15 */
  p = gr_fmaf(p, t2, -7.69230769e-02f);  /* -1/13 */
  p = gr_fmaf(p, t2, 9.09090909e-02f);   /* 1/11 */
  p = gr_fmaf(p, t2, -1.11111111e-01f);  /* -1/9 */
  p = gr_fmaf(p, t2, 1.42857143e-01f);   /* 1/7 */
  p = gr_fmaf(p, t2, -2.00000000e-01f);  /* -1/5 */
  p = gr_fmaf(p, t2, 3.33333333e-01f);   /* 1/3 */
  return base + gr_fmaf(-t, t2 * p, t);
}

/* atan2(y, x) with C semantics for finite inputs (atan2(0,0)=0) */
GR_HD float gr_atan2f(float y, float x) {
  float ax = gr_fabsf(x), ay = gr_fabsf(y);
  float mx = gr_maxf(ax, ay), mn = gr_minf(ax, ay);
  if (mx == 0.0f) return (gr_f2u(x) & 0x80000000u) ? gr_copysignf(3.14159274f, y) : gr_copysignf(0.0f, y);
  float a = gr_atan_unit(mn / mx);
  if (ay > ax) a = 1.57079637f - a;
  if (x < 0.0f) a = 3.14159274f - a;
  return gr_copysignf(a, y);
}

/* fmod(a, b) for |a| < 2|b|, b > 0 — exact (Sterbenz) */
GR_HD float gr_fmod_small(float a, float b) {
  return gr_fabsf(a) < b ? a : a - gr_copysignf(b, a);
}
/* torch.remainder(a, b) (Python-style, result has the sign of b), b > 0, |a| < 2b */
GR_HD float gr_remainder_small(float a, float b) {
  float m = gr_fmod_small(a, b);
  if (m != 0.0f && m < 0.0f) m = m + b;
  return m;
}
/* Isaac Lab wrap_to_pi restated:  w = (a + pi) % 2pi; where(w==0 & a>0, pi, w - pi) */
GR_HD float gr_wrap_to_pi(float a) {
  const float PI = 3.14159274f, TWO_PI = 6.28318548f;
  float w = gr_remainder_small(a + PI, TWO_PI);
  return (w == 0.0f && a > 0.0f) ? PI : w - PI;
}

#endif /* GR_MATH_H */
