/*
 * gr_camera.h — the front depth camera of the racing task, as fp32 functions shared
 * verbatim by the HIP kernel (gr_camera.hip) and the CPU oracle (oracle/gr_oracle.c).
 *
 * Reference: `front_camera = RayCasterCameraCfg(...)` (extensions/diff.lab_tasks/diff/
 * lab_tasks/tasks/quadcopter_diff/racing_ctbr_env.py:77-95): a 96x72 pinhole ray caster
 * against the terrain mesh, `distance_to_image_plane`, max_distance 10 with clipping
 * behaviour "max", update_period 0.04 s (:390-391); observation term `depth_image`
 * (mdp/observation.py:65-94): x (1 + 0.02 N(0,1)) on the policy image, inf -> 0,
 * > 10 -> 10, / 10.
 *
 * Geometry.  The reference casts Warp BVH rays against the trimesh terrain: each gate
 * is `make_gate` = outer box minus inner box (trimesh/utils.py:10-33), plus the ground.
 * Here each gate is intersected analytically as a box with a through-hole prism (the
 * same solid), in the gate's own frame, from the track-table record the collision test
 * uses; the ground is the plane z = ground_z (env-local).  The track's walls / orbits /
 * ground obstacles are analytic primitives (gr_obstacles.h).  The gates and obstacles of
 * the neighbouring 40 m terrain tiles are not rendered.
 *
 * Rays.  Pixel (u, v) (row-major, v*W + u) looks along r = (1, a_u, b_v) in the camera
 * frame (x forward, y left, z up: "world" convention), a_u = (cx - (u + 0.5)) / fx,
 * b_v = (cy - (v + 0.5)) / fy (Isaac Lab's pinhole pattern, pixel centres).  Because
 * r has unit forward component, the ray parameter s of a hit IS the distance to the
 * image plane: no normalisation, no cosine.
 *
 * Every op is IEEE fp32 (+,-,*,/ correctly rounded; explicit gr_fmaf), so kernel and
 * oracle produce identical bits.  Compiles as C (gcc) and HIP C++.
 */
#ifndef GR_CAMERA_H
#define GR_CAMERA_H

#include "../../include/gr.h"
#include "gr_math.h"
#include "gr_obstacles.h"
#include "gr_rng.h"

#define GR_CAM_MAX_W 256
#define GR_CAM_MAX_H 256
#define GR_CAM_MAX_GATES 64 /* one lane per gate sets a wave's gate slots up */
#define GR_CAM_SLOT 36      /* floats per gate slot, see gr_cam_gate_setup */
#define GR_CAM_FAR 3.0e38f  /* "no hit" */

/* slot layout */
#define GR_CS_O 0     /* ray origin in the gate frame (3) */
#define GR_CS_D0 3    /* camera forward axis in the gate frame (3) */
#define GR_CS_D1 6    /* camera left axis (3) */
#define GR_CS_D2 9    /* camera up axis (3) */
#define GR_CS_HW 12   /* inner half width / height, half thickness, outer half width / height */
#define GR_CS_HH 13
#define GR_CS_HT 14
#define GR_CS_HOW 15
#define GR_CS_HOH 16
#define GR_CS_AMIN 17 /* conservative screen window in tangent space (a, b) */
#define GR_CS_AMAX 18
#define GR_CS_BMIN 19
#define GR_CS_BMAX 20
#define GR_CS_VALID 21 /* 1.0: may be hit by some pixel; 0.0: culled (behind, beyond range, or absent) */
/* a gate's inverse-depth slab constants (gr_cam_gate_hit; gr_obst_slab_prep of gr_obstacles.h): entry / exit of
 * the outer box's x, y, z slabs, of the hole's x, y slabs, and the camera-inside bits (as a float) */
#define GR_CS_UE 24   /* outer x, y, z entry (3) */
#define GR_CS_UX 27   /* outer x, y, z exit (3) */
#define GR_CS_HE 30   /* hole x, y entry (2) */
#define GR_CS_HX 32   /* hole x, y exit (2) */
#define GR_CS_UM 34   /* bits 0-2: inside outer slab x / y / z; bits 3-4: inside hole slab x / y */

/* Constants derived once from gr_camera_config (host side, identical on both sides). */
typedef struct gr_cam_const {
  int32_t width, height, npix, period_steps;
  float off_p[3];
  float R_off[9]; /* row-major, rotation of the normalised offset quaternion */
  float max_distance, obs_scale, inv_obs_scale, noise_std;
  int32_t add_noise;
  float ray_a[GR_CAM_MAX_W]; /* a_u */
  float ray_b[GR_CAM_MAX_H]; /* b_v */
} gr_cam_const;

/* rotation matrix (row-major) of a unit quaternion w,x,y,z */
GR_HD void gr_cam_quat_matrix(const float q[4], float R[9]) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1.0f - 2.0f * (y * y + z * z);
  R[1] = 2.0f * (x * y - w * z);
  R[2] = 2.0f * (x * z + w * y);
  R[3] = 2.0f * (x * y + w * z);
  R[4] = 1.0f - 2.0f * (x * x + z * z);
  R[5] = 2.0f * (y * z - w * x);
  R[6] = 2.0f * (x * z - w * y);
  R[7] = 2.0f * (y * z + w * x);
  R[8] = 1.0f - 2.0f * (x * x + y * y);
}

/* a_u / b_v of the pinhole pattern */
GR_HD float gr_cam_tan(float c, float f, int i) { return (c - ((float)i + 0.5f)) / f; }

/* camera pose in the env-local frame from the body pose (Isaac Lab combine_frame_transforms:
 * o = p + R(q) off_p, R_cam = R(q) R_off); c0/c1/c2 = camera forward / left / up axes */
GR_HD void gr_cam_pose(const gr_cam_const* cc, const float p[3], const float q[4], float o[3], float c0[3],
                       float c1[3], float c2[3]) {
  float R[9];
  gr_cam_quat_matrix(q, R);
  for (int i = 0; i < 3; ++i) {
    const float r0 = R[3 * i], r1 = R[3 * i + 1], r2 = R[3 * i + 2];
    o[i] = p[i] + gr_fmaf(r2, cc->off_p[2], gr_fmaf(r1, cc->off_p[1], r0 * cc->off_p[0]));
    c0[i] = gr_fmaf(r2, cc->R_off[6], gr_fmaf(r1, cc->R_off[3], r0 * cc->R_off[0]));
    c1[i] = gr_fmaf(r2, cc->R_off[7], gr_fmaf(r1, cc->R_off[4], r0 * cc->R_off[1]));
    c2[i] = gr_fmaf(r2, cc->R_off[8], gr_fmaf(r1, cc->R_off[5], r0 * cc->R_off[2]));
  }
}

GR_HD float gr_cam_dot3(const float* a, const float* b) { return gr_fmaf(a[2], b[2], gr_fmaf(a[1], b[1], a[0] * b[0])); }

/* A primitive with a GR_GATE_FLOATS / GR_OBST_FLOATS style record (centre 0-2, rows of R^T
 * at 4-6 / 8-10 / 12-14) and local bounding-box half extents l, seen from camera (o, c0, c1,
 * c2): fills the frame part of a slot.  Culls primitives entirely behind the camera or whose
 * nearest point is beyond max_distance (the clip makes such hits indistinguishable from
 * misses), and bounds the screen footprint by projecting the 8 box corners (convex hull of a
 * convex solid in front of the camera); the window gets a margin so that rounding never
 * culls a pixel that can hit. */
GR_HD void gr_cam_frame_setup(const float* g, const float l[3], const float o[3], const float c0[3],
                              const float c1[3], const float c2[3], float max_distance, float* s) {
  const float rel[3] = {g[0] - o[0], g[1] - o[1], g[2] - o[2]};
  const float* M[3] = {g + 4, g + 8, g + 12};
  for (int j = 0; j < 3; ++j) {
    s[GR_CS_O + j] = -gr_cam_dot3(M[j], rel);
    s[GR_CS_D0 + j] = gr_cam_dot3(M[j], c0);
    s[GR_CS_D1 + j] = gr_cam_dot3(M[j], c1);
    s[GR_CS_D2 + j] = gr_cam_dot3(M[j], c2);
  }
  const float x0 = gr_cam_dot3(c0, rel), y0 = gr_cam_dot3(c1, rel), z0 = gr_cam_dot3(c2, rel);
  float ex = 0.0f;
  for (int j = 0; j < 3; ++j) ex += gr_fabsf(l[j] * s[GR_CS_D0 + j]);
  const float xmin = x0 - ex, xmax = x0 + ex;
  s[GR_CS_VALID] = (xmax > 0.0f && xmin <= max_distance) ? 1.0f : 0.0f;
  float amin = -GR_CAM_FAR, amax = GR_CAM_FAR, bmin = -GR_CAM_FAR, bmax = GR_CAM_FAR;
  if (xmin > 1.0e-3f) {
    amin = bmin = GR_CAM_FAR;
    amax = bmax = -GR_CAM_FAR;
    for (int k = 0; k < 8; ++k) {
      const float sx = (k & 1) ? l[0] : -l[0], sy = (k & 2) ? l[1] : -l[1], sz = (k & 4) ? l[2] : -l[2];
      const float x = gr_fmaf(sz, s[GR_CS_D0 + 2], gr_fmaf(sy, s[GR_CS_D0 + 1], gr_fmaf(sx, s[GR_CS_D0], x0)));
      const float y = gr_fmaf(sz, s[GR_CS_D1 + 2], gr_fmaf(sy, s[GR_CS_D1 + 1], gr_fmaf(sx, s[GR_CS_D1], y0)));
      const float z = gr_fmaf(sz, s[GR_CS_D2 + 2], gr_fmaf(sy, s[GR_CS_D2 + 1], gr_fmaf(sx, s[GR_CS_D2], z0)));
      const float a = y / x, b = z / x;
      amin = gr_minf(amin, a);
      amax = gr_maxf(amax, a);
      bmin = gr_minf(bmin, b);
      bmax = gr_maxf(bmax, b);
    }
    const float ma = 1.0e-3f + 1.0e-4f * (gr_fabsf(amin) + gr_fabsf(amax));
    const float mb = 1.0e-3f + 1.0e-4f * (gr_fabsf(bmin) + gr_fabsf(bmax));
    amin -= ma;
    amax += ma;
    bmin -= mb;
    bmax += mb;
  }
  s[GR_CS_AMIN] = amin;
  s[GR_CS_AMAX] = amax;
  s[GR_CS_BMIN] = bmin;
  s[GR_CS_BMAX] = bmax;
  s[22] = 0.0f;
  s[23] = 0.0f;
}

/* One gate (GR_GATE_FLOATS record: centre, rows of R^T, half sizes): its outer box bounds
 * the window. */
GR_HD void gr_cam_gate_setup(const float* g, const float o[3], const float c0[3], const float c1[3],
                             const float c2[3], float max_distance, float* s) {
  const float l[3] = {g[16], g[17], g[15]};
  gr_cam_frame_setup(g, l, o, c0, c1, c2, max_distance, s);
  s[GR_CS_HW] = g[7];
  s[GR_CS_HH] = g[11];
  s[GR_CS_HT] = g[15];
  s[GR_CS_HOW] = g[16];
  s[GR_CS_HOH] = g[17];
  int m = 0, in = 0;
  gr_obst_slab_prep(s[GR_CS_O], s[GR_CS_HOW], &s[GR_CS_UE], &s[GR_CS_UX], &in);
  m |= in;
  gr_obst_slab_prep(s[GR_CS_O + 1], s[GR_CS_HOH], &s[GR_CS_UE + 1], &s[GR_CS_UX + 1], &in);
  m |= in << 1;
  gr_obst_slab_prep(s[GR_CS_O + 2], s[GR_CS_HT], &s[GR_CS_UE + 2], &s[GR_CS_UX + 2], &in);
  m |= in << 2;
  gr_obst_slab_prep(s[GR_CS_O], s[GR_CS_HW], &s[GR_CS_HE], &s[GR_CS_HX], &in);
  m |= in << 3;
  gr_obst_slab_prep(s[GR_CS_O + 1], s[GR_CS_HH], &s[GR_CS_HE + 1], &s[GR_CS_HX + 1], &in);
  m |= in << 4;
  s[GR_CS_UM] = (float)m;
  s[GR_CS_UM + 1] = 0.0f;
}

/* kernel-only tile cull of a gate slot: its outer box (gr_cam_box_outside, gr_obstacles.h) */
GR_HD int gr_cam_gate_outside(const float* s, float a_lo, float a_hi, float b_lo, float b_hi) {
  const float l[3] = {s[GR_CS_HOW], s[GR_CS_HOH], s[GR_CS_HT]};
  return gr_cam_box_outside(s, l, a_lo, a_hi, b_lo, b_hi);
}

/* One obstacle (GR_OBST_FLOATS record, gr_obstacles.h); hit by gr_cam_obst_hit. */
GR_HD void gr_cam_obst_setup(const float* r, const float o[3], const float c0[3], const float c1[3],
                             const float c2[3], float max_distance, float* s) {
  float l[3];
  gr_obst_local_box(r, l);
  gr_cam_frame_setup(r, l, o, c0, c1, c2, max_distance, s);
  s[GR_OS_E0] = r[7];
  s[GR_OS_E1] = r[11];
  s[GR_OS_E2] = r[15];
  s[GR_OS_KIND] = r[16];
  s[16] = 0.0f;
}

/* First surface crossing (s > 0) of the ray (a, b) with the gate solid
 * {|x| <= how, |y| <= hoh, |z| <= ht} minus the hole {|x| < hw, |y| < hh}; GR_CAM_FAR if none.
 * From outside the solid: the first entry; from inside a bar: the exit (a mesh ray cast
 * reports the first face it crosses either way).  In inverse depth u = 1 / s, as
 * gr_cam_obst_hit_k (gr_obstacles.h): the five slab tests are multiplies by the slot's constants,
 * and the hit costs one division. */
GR_HD float gr_cam_gate_hit(const float* s, float a, float b) {
  const float dx = gr_fmaf(b, s[GR_CS_D2], gr_fmaf(a, s[GR_CS_D1], s[GR_CS_D0]));
  const float dy = gr_fmaf(b, s[GR_CS_D2 + 1], gr_fmaf(a, s[GR_CS_D1 + 1], s[GR_CS_D0 + 1]));
  const float dz = gr_fmaf(b, s[GR_CS_D2 + 2], gr_fmaf(a, s[GR_CS_D1 + 2], s[GR_CS_D0 + 2]));
  const int m = (int)s[GR_CS_UM];
  float uin = GR_U_NONE, uout = 0.0f, hin = GR_U_NONE, hout = 0.0f;
  gr_u_slab(dx, s[GR_CS_UE], s[GR_CS_UX], m & 1, &uin, &uout);
  gr_u_slab(dy, s[GR_CS_UE + 1], s[GR_CS_UX + 1], m & 2, &uin, &uout);
  gr_u_slab(dz, s[GR_CS_UE + 2], s[GR_CS_UX + 2], m & 4, &uin, &uout);
  gr_u_slab(dx, s[GR_CS_HE], s[GR_CS_HX], m & 8, &hin, &hout);
  gr_u_slab(dy, s[GR_CS_HE + 1], s[GR_CS_HX + 1], m & 16, &hin, &hout);
  /* the hole's prism: around the camera (its entry behind), or crossed ahead (a prism interval behind the
   * camera plays no part) */
  const int prism = hin >= GR_U_NONE;
  const int ahead = !prism && hin > 0.0f && hin > hout;
  float u;
  if (uin < GR_U_NONE) {
    /* outside the solid's box: enter at its entry, unless that lies in the hole, then at the hole's exit */
    if (!(uin > 0.0f && uin >= uout)) return GR_CAM_FAR;
    const int in_hole = (prism || (ahead && hin > uin)) && uin > hout;
    u = in_hole ? (hout > uout ? hout : 0.0f) : uin;
  } else if (prism) {
    /* inside the box, in the hole: the hole's exit if it leaves through a bar */
    u = hout > uout ? hout : 0.0f;
  } else {
    /* inside a bar: leave through the hole wall or the outer box */
    u = (ahead && hin > uout) ? hin : uout;
  }
  return u > 0.0f ? 1.0f / u : GR_CAM_FAR;
}

/* ground plane z = gz seen along the ray with vertical component dz */
GR_HD float gr_cam_ground_hit(float oz, float gz, float dz) {
  const float s = (gz - oz) / dz;
  return s > 0.0f ? s : GR_CAM_FAR;
}

/* distance_to_image_plane with clipping behaviour "max" (misses and far hits -> max) */
GR_HD float gr_cam_clip(float s, float max_distance) { return s < max_distance ? s : max_distance; }

/* depth_image() (observation.py:84-92): noisy = d * (1 + z * std); inf -> 0; > scale -> scale;
 * then `images /= 10`, which torch evaluates on the GPU as a multiply by the fp32 reciprocal of
 * the Python scalar (BinaryDivTrueKernel: a * (1 / b)): inv_scale = 1.0f / scale. */
GR_HD float gr_cam_obs(float d, float z, float std, float scale, float inv_scale) {
  float x = d * (1.0f + z * std);
  x = x > scale ? scale : x;
  return x * inv_scale;
}

/* the critic image: no noise */
GR_HD float gr_cam_obs_clean(float d, float scale, float inv_scale) { return (d > scale ? scale : d) * inv_scale; }

/* the four standard normals of pixel quad `quad` (pixels 4*quad .. 4*quad+3): one Philox block, one word per pixel
 * through the inverse-CDF table (`tab` = GR_NORMAL_TABLE_INIT's floats, gr_normal24) */
GR_HD void gr_cam_noise4(uint32_t gid, uint32_t cnt, uint32_t quad, uint32_t k0, uint32_t k1, const float* tab,
                         float z[4]) {
  const gr_u32x4 r = gr_philox4x32_10(gid, cnt, GR_TAG_IMG, quad, k0, k1);
  z[0] = gr_normal24(r.x, tab);
  z[1] = gr_normal24(r.y, tab);
  z[2] = gr_normal24(r.z, tab);
  z[3] = gr_normal24(r.w, tab);
}

/* Isaac Lab sensor timing (SensorBase.update / _update_outdated_buffers): a sensor is
 * outdated once update_period has elapsed since its last render (checked every physics
 * substep, rendered lazily at the next observation), and on reset.  In env steps: a
 * render happens when `period_steps` steps have passed, or after a reset. */
GR_HD int gr_cam_period_steps(float step_dt, float update_period) {
  int k = 1;
  while ((double)k * (double)step_dt + 1e-6 < (double)update_period && k < 1000000) ++k;
  return k;
}

/* gr_camera_config -> gr_cam_const (validated by the caller) */
GR_HD void gr_cam_derive(const gr_camera_config* c, float step_dt, gr_cam_const* k) {
  k->width = c->width;
  k->height = c->height;
  k->npix = c->width * c->height;
  k->period_steps = gr_cam_period_steps(step_dt, c->update_period);
  for (int i = 0; i < 3; ++i) k->off_p[i] = c->offset_pos[i];
  const float* r = c->offset_rot;
  const float n = gr_sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2] + r[3] * r[3]);
  const float qn[4] = {r[0] / n, r[1] / n, r[2] / n, r[3] / n};
  gr_cam_quat_matrix(qn, k->R_off);
  k->max_distance = c->max_distance;
  k->obs_scale = c->obs_scale;
  k->inv_obs_scale = 1.0f / c->obs_scale;
  k->noise_std = c->noise_std;
  k->add_noise = c->add_noise;
  for (int u = 0; u < GR_CAM_MAX_W; ++u) k->ray_a[u] = u < c->width ? gr_cam_tan(c->cx, c->fx, u) : 0.0f;
  for (int v = 0; v < GR_CAM_MAX_H; ++v) k->ray_b[v] = v < c->height ? gr_cam_tan(c->cy, c->fy, v) : 0.0f;
}

#endif /* GR_CAMERA_H */
