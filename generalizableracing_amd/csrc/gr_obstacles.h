/*
 * gr_obstacles.h — the track obstacles (walls, "orbits", ground obstacles) as analytic
 * primitives: the lattice collision test and the depth-camera ray hit, as fp32 functions
 * shared verbatim by the HIP kernels (gr_kernels.hip, gr_camera.hip) and the CPU oracle
 * (oracle/gr_oracle.c).
 *
 * Reference: the sub-terrain generators add, per gate segment, `make_wall` boxes,
 * `make_orbit` boxes / cylinders / icospheres / capsules at random orientations, and
 * `make_ground_high_obs` / `make_ground_little_obj` boxes / cylinders / spheres standing
 * on the ground (extensions/diff.lab/diff/lab/terrains/trimesh/utils.py:35-131, placed by
 * trimesh/racing_terrains.py:254-319, 510-610, 750-815 when the cfg sets add_obs /
 * add_ground_obs, as RacingComplexTerrainCfg does: quadcopter_diff/terrains/
 * racing_terrains.py:137-210).  They are part of the terrain mesh, so PhysX contact
 * (base_contact termination, collision penalty) and the Warp ray caster (depth image)
 * both see them.  Here each is the exact solid the trimesh mesh approximates (trimesh's
 * 32-segment cylinders and subdivided icospheres differ from the true surface by < 0.5 %
 * of the radius; parity of that difference is unpinned: trimesh is not installed).
 *
 * Record (GR_OBST_FLOATS, env-local frame): 0-2 centre, 3 cull radius^2 (bounding radius
 * + lattice reach, with margin), 4-6 / 8-10 / 12-14 rows of R^T (world -> primitive
 * frame), 7 / 11 / 15 = e0 / e1 / e2: box half extents | cylinder r, r, half height |
 * sphere r, r, r | capsule r, r, half segment (axes along the local z), 16 kind,
 * 17 bounding radius.
 *
 * Every op is IEEE fp32 with contraction off, so kernel and oracle agree bit for bit.
 * Compiles as C (gcc) and HIP C++.
 */
#ifndef GR_OBSTACLES_H
#define GR_OBSTACLES_H

#include "../../include/gr.h"
#include "gr_math.h"

/* the drone's collision lattice (diff.lab/utils/__init__.py:19-37), in units of the
 * collider half extents */
#define GR_LATTICE_INIT                                                                                     \
  {                                                                                                         \
    {0, 0, 0}, {1, 1, 1}, {1, -1, 1}, {-1, 1, 1}, {-1, -1, 1}, {1, 1, -1}, {1, -1, -1}, {-1, 1, -1},          \
        {-1, -1, -1}, {0.5f, 0.5f, 0.5f}, {0.5f, -0.5f, 0.5f}, {-0.5f, 0.5f, 0.5f}, {-0.5f, -0.5f, 0.5f},   \
        {0.5f, 0.5f, -0.5f}, {0.5f, -0.5f, -0.5f}, {-0.5f, 0.5f, -0.5f}, { -0.5f, -0.5f, -0.5f }             \
  }

/* is the point l (primitive frame) inside the primitive?  (closed solids) */
GR_HD int gr_obst_inside(int kind, float l0, float l1, float l2, float e0, float e1, float e2) {
  const float a0 = gr_fabsf(l0), a1 = gr_fabsf(l1), a2 = gr_fabsf(l2);
  const float rr = e0 * e0, radial = l0 * l0 + l1 * l1;
  const float dz = gr_maxf(a2 - e2, 0.0f);
  const int box = (a0 <= e0) & (a1 <= e1) & (a2 <= e2);
  const int cyl = (radial <= rr) & (a2 <= e2);
  const int sph = radial + l2 * l2 <= rr;
  const int cap = radial + dz * dz <= rr;
  return kind == GR_OBST_BOX ? box : kind == GR_OBST_CYLINDER ? cyl : kind == GR_OBST_SPHERE ? sph : cap;
}

/* M v with M = rows 4-6 / 8-10 / 12-14 of a record (the gate-frame expression of the
 * collision test) */
GR_HD void gr_obst_frame(const float* r, const float v[3], float o[3]) {
  o[0] = (r[4] * v[0] + r[5] * v[1]) + r[6] * v[2];
  o[1] = (r[8] * v[0] + r[9] * v[1]) + r[10] * v[2];
  o[2] = (r[12] * v[0] + r[13] * v[1]) + r[14] * v[2];
}

/* Bit k set: lattice point k = p + (lx A + ly B) + lz C (A, B, C the rotated scaled body
 * axes; lat = GR_LATTICE_INIT) lies inside the obstacle.  Evaluated in the primitive frame
 * as d + (lx A' + ly B') + lz C' with d = M (p - c), A' = M A, ... */
GR_HD uint32_t gr_obst_lattice_mask(const float* r, const float p[3], const float A[3], const float B[3],
                                    const float C[3], const float lat[17][3]) {
  const float d[3] = {p[0] - r[0], p[1] - r[1], p[2] - r[2]};
  float dg[3], Ag[3], Bg[3], Cg[3];
  gr_obst_frame(r, d, dg);
  gr_obst_frame(r, A, Ag);
  gr_obst_frame(r, B, Bg);
  gr_obst_frame(r, C, Cg);
  const int kind = (int)r[16];
  const float e0 = r[7], e1 = r[11], e2 = r[15];
  uint32_t m = 0u;
  for (int k = 0; k < 17; ++k) {
    const float lx = lat[k][0], ly = lat[k][1], lz = lat[k][2];
    const float l0 = dg[0] + ((lx * Ag[0] + ly * Bg[0]) + lz * Cg[0]);
    const float l1 = dg[1] + ((lx * Ag[1] + ly * Bg[1]) + lz * Cg[1]);
    const float l2 = dg[2] + ((lx * Ag[2] + ly * Bg[2]) + lz * Cg[2]);
    m |= (uint32_t)gr_obst_inside(kind, l0, l1, l2, e0, e1, e2) << k;
  }
  return m;
}

/* tighter cull (kernel only; the oracle tests every obstacle): can a point within `reach` of p be
 * inside the primitive?  p in the primitive frame (the expression the lattice test uses for its
 * centre term) against the primitive grown by reach: per-axis slabs for the box and the cylinder's
 * height, radii + reach for the round parts.  Contains the Minkowski sum primitive (+) ball(reach),
 * so it never rejects a primitive a lattice point is inside. */
GR_HD int gr_obst_maybe(const float* r, const float p[3], float reach) {
  const float d[3] = {p[0] - r[0], p[1] - r[1], p[2] - r[2]};
  float l[3];
  gr_obst_frame(r, d, l);
  const int kind = (int)r[16];
  const float a0 = gr_fabsf(l[0]), a1 = gr_fabsf(l[1]), a2 = gr_fabsf(l[2]);
  const float e0 = r[7] + reach, e1 = r[11] + reach, rr = e0 * e0;
  const float radial = l[0] * l[0] + l[1] * l[1];
  const float dz = gr_maxf(a2 - r[15], 0.0f);
  const int box = (a0 <= e0) & (a1 <= e1) & (a2 <= r[15] + reach);
  const int cyl = (radial <= rr) & (a2 <= r[15] + reach);
  const int rnd = radial + (kind == GR_OBST_SPHERE ? l[2] * l[2] : dz * dz) <= rr;
  return kind == GR_OBST_BOX ? box : kind == GR_OBST_CYLINDER ? cyl : rnd;
}

/* cull: can any lattice point of a drone at p be inside?  (|p - c|^2 <= cull radius^2) */
GR_HD int gr_obst_near(const float* r, const float p[3]) {
  const float dx = p[0] - r[0], dy = p[1] - r[1], dz = p[2] - r[2];
  return (dx * dx + dy * dy) + dz * dz <= r[3];
}

/* ------------------------------------------------------------------ depth camera */
/* Camera slot of an obstacle: the gate slot layout of gr_camera.h (origin and camera axes
 * in the primitive frame, screen window, valid flag) with the primitive in 12-15. */
#define GR_OS_E0 12
#define GR_OS_E1 13
#define GR_OS_E2 14
#define GR_OS_KIND 15

/* half extents of the primitive's local bounding box (the window projects its corners) */
GR_HD void gr_obst_local_box(const float* r, float l[3]) {
  const int kind = (int)r[16];
  l[0] = r[7];
  l[1] = r[11];
  l[2] = kind == GR_OBST_CAPSULE ? r[15] + r[7] : r[15];
}

/* One side plane of a frustum of pixel rays (y = a x or z = a x in camera coordinates, x forward): is the box
 * (centre (x0, cp) in the plane's two coordinates, primitive axis j = (d0[j], dp[j]) in them, half sizes l) wholly
 * on the outer side, sgn * (y - a x) > 0?  With a margin far above the rounding of any hit test. */
GR_HD int gr_cam_box_beyond(float x0, float cp, const float* d0, const float* dp, const float l[3], float a,
                            float sgn) {
  const float v = sgn * (cp - a * x0);
  const float r = (l[0] * gr_fabsf(dp[0] - a * d0[0]) + l[1] * gr_fabsf(dp[1] - a * d0[1])) +
                  l[2] * gr_fabsf(dp[2] - a * d0[2]);
  const float m = 1.0e-3f + 1.0e-4f * ((gr_fabsf(cp) + gr_fabsf(a * x0)) + r);
  return v - r > m;
}

/* Kernel-only cull of a camera slot against a tile of pixel rays a in [a_lo, a_hi], b in [b_lo, b_hi] (the oracle
 * tests every pixel of the slot's window, so this only skips pixels that cannot hit): the solid's local bounding
 * box (half sizes l) lies wholly beyond one side plane of the tile's frustum.  A window spans the box's 8
 * projected corners, and is the whole screen when the box reaches behind the camera plane (a wall alongside the
 * drone, a gate being flown through); the planes cut both down to the tiles the box can actually cover.  Camera
 * coordinates from the slot: the centre is -(D0 . O, D1 . O, D2 . O), local axis j is (D0[j], D1[j], D2[j]). */
GR_HD int gr_cam_box_outside(const float* s, const float l[3], float a_lo, float a_hi, float b_lo, float b_hi) {
  const float* O = s;
  const float* D0 = s + 3;
  const float* D1 = s + 6;
  const float* D2 = s + 9;
  const float x0 = -((D0[0] * O[0] + D0[1] * O[1]) + D0[2] * O[2]);
  const float y0 = -((D1[0] * O[0] + D1[1] * O[1]) + D1[2] * O[2]);
  const float z0 = -((D2[0] * O[0] + D2[1] * O[1]) + D2[2] * O[2]);
  return gr_cam_box_beyond(x0, y0, D0, D1, l, a_hi, 1.0f) | gr_cam_box_beyond(x0, y0, D0, D1, l, a_lo, -1.0f) |
         gr_cam_box_beyond(x0, z0, D0, D2, l, b_hi, 1.0f) | gr_cam_box_beyond(x0, z0, D0, D2, l, b_lo, -1.0f);
}

/* an obstacle slot (gr_cam_obst_setup): the primitive's local bounding box */
GR_HD int gr_cam_obst_outside(const float* s, float a_lo, float a_hi, float b_lo, float b_hi) {
  const int kind = (int)s[GR_OS_KIND];
  const float l[3] = {s[GR_OS_E0], s[GR_OS_E1], kind == GR_OBST_CAPSULE ? s[GR_OS_E2] + s[GR_OS_E0] : s[GR_OS_E2]};
  return gr_cam_box_outside(s, l, a_lo, a_hi, b_lo, b_hi);
}

/* first crossing (s > 0) of the ray o + s d with the slab |x_j| <= h_j intersected with
 * the interval [t0, t1]; GR_CAM_FAR-style miss = 3e38 */
GR_HD float gr_obst_first(float tin, float tout) {
  if (!(tin <= tout) || !(tout > 0.0f)) return 3.0e38f;
  return tin > 0.0f ? tin : tout;
}

GR_HD float gr_obst_inv(float d) { return 1.0f / (gr_fabsf(d) < 1.0e-20f ? gr_copysignf(1.0e-20f, d) : d); }

/* entry / exit of the sphere |x - (0,0,zc)| <= rad along o + s d (tin > tout: miss) */
GR_HD void gr_obst_sphere_iv(const float o[3], const float d[3], float zc, float rad, float* tin, float* tout) {
  const float oz = o[2] - zc;
  const float A = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
  const float Bh = (o[0] * d[0] + o[1] * d[1]) + oz * d[2];
  const float Cc = ((o[0] * o[0] + o[1] * o[1]) + oz * oz) - rad * rad;
  const float disc = Bh * Bh - A * Cc;
  if (!(disc >= 0.0f)) {
    *tin = 1.0f;
    *tout = -1.0f;
    return;
  }
  const float sq = gr_sqrtf(disc);
  *tin = (-Bh - sq) / A;
  *tout = (-Bh + sq) / A;
}

/* entry / exit of the finite cylinder x^2 + y^2 <= rad^2, |z| <= hh */
GR_HD void gr_obst_cyl_iv(const float o[3], const float d[3], float rad, float hh, float* tin, float* tout) {
  const float iz = gr_obst_inv(d[2]);
  const float z0 = (-hh - o[2]) * iz, z1 = (hh - o[2]) * iz;
  float lo = gr_minf(z0, z1), hi = gr_maxf(z0, z1);
  const float A = d[0] * d[0] + d[1] * d[1];
  const float Bh = o[0] * d[0] + o[1] * d[1];
  const float Cc = (o[0] * o[0] + o[1] * o[1]) - rad * rad;
  if (A < 1.0e-12f) {
    /* parallel to the axis: inside the radius everywhere or nowhere */
    if (!(Cc <= 0.0f)) hi = lo - 1.0f;
  } else {
    const float disc = Bh * Bh - A * Cc;
    if (!(disc >= 0.0f)) {
      hi = lo - 1.0f;
    } else {
      const float sq = gr_sqrtf(disc);
      lo = gr_maxf(lo, (-Bh - sq) / A);
      hi = gr_minf(hi, (-Bh + sq) / A);
    }
  }
  *tin = lo;
  *tout = hi;
}

/* first surface crossing (s > 0) of the pixel ray (a, b) with the obstacle of slot s:
 * from outside the entry, from inside the exit (a mesh ray cast reports the first face
 * it crosses).  The capsule is the union of its cylinder and two end spheres: the
 * nearest of their crossings. */
GR_HD float gr_cam_obst_hit(const float* s, float a, float b) {
  const float d[3] = {gr_fmaf(b, s[9], gr_fmaf(a, s[6], s[3])), gr_fmaf(b, s[10], gr_fmaf(a, s[7], s[4])),
                      gr_fmaf(b, s[11], gr_fmaf(a, s[8], s[5]))};
  const float o[3] = {s[0], s[1], s[2]};
  const int kind = (int)s[GR_OS_KIND];
  const float e0 = s[GR_OS_E0], e1 = s[GR_OS_E1], e2 = s[GR_OS_E2];
  float tin, tout;
  if (kind == GR_OBST_BOX) {
    const float ix = gr_obst_inv(d[0]), iy = gr_obst_inv(d[1]), iz = gr_obst_inv(d[2]);
    const float tx0 = (-e0 - o[0]) * ix, tx1 = (e0 - o[0]) * ix;
    const float ty0 = (-e1 - o[1]) * iy, ty1 = (e1 - o[1]) * iy;
    const float tz0 = (-e2 - o[2]) * iz, tz1 = (e2 - o[2]) * iz;
    tin = gr_maxf(gr_maxf(gr_minf(tx0, tx1), gr_minf(ty0, ty1)), gr_minf(tz0, tz1));
    tout = gr_minf(gr_minf(gr_maxf(tx0, tx1), gr_maxf(ty0, ty1)), gr_maxf(tz0, tz1));
    return gr_obst_first(tin, tout);
  }
  if (kind == GR_OBST_SPHERE) {
    gr_obst_sphere_iv(o, d, 0.0f, e0, &tin, &tout);
    return gr_obst_first(tin, tout);
  }
  gr_obst_cyl_iv(o, d, e0, e2, &tin, &tout);
  float hit = gr_obst_first(tin, tout);
  if (kind == GR_OBST_CAPSULE) {
    gr_obst_sphere_iv(o, d, e2, e0, &tin, &tout);
    hit = gr_minf(hit, gr_obst_first(tin, tout));
    gr_obst_sphere_iv(o, d, -e2, e0, &tin, &tout);
    hit = gr_minf(hit, gr_obst_first(tin, tout));
  }
  return hit;
}

/* ---- slab tests in inverse depth (the camera's gate hit, gr_camera.h).  Along pixel ray (a, b) the direction in
 * the primitive frame, d, is affine in (a, b), and the depth of the crossing with a plane x_j = p is
 * s = (p - o_j) / d_j: its reciprocal u = d_j / (p - o_j) is d_j times a per-slot constant.  The slab tests
 * therefore run on u (for s > 0 the order reverses: the latest entry is the smallest u, the earliest exit the
 * largest), and a hit costs one division, 1 / u of the first crossing, instead of one per slab. */
#define GR_U_NONE 3.0e38f   /* "no entry bound" (the camera is inside that slab / sphere) */

/* slab |x| <= e seen from o: entry / exit constants (1 / (plane - o)); inside: o strictly between the planes */
GR_HD void gr_obst_slab_prep(float o, float e, float* cE, float* cX, int* inside) {
  const float lo = -e - o, hi = e - o;
  *inside = lo < 0.0f && hi > 0.0f;
  if (hi <= 0.0f) { /* beyond +e: entered through +e, left through -e */
    *cE = gr_obst_inv(hi);
    *cX = gr_obst_inv(lo);
  } else { /* below -e (entered through -e), or inside */
    *cE = gr_obst_inv(lo);
    *cX = gr_obst_inv(hi);
  }
}
/* one slab along the ray: the entry bound (outside only) and the exit */
GR_HD void gr_u_slab(float d, float cE, float cX, int inside, float* uin, float* uout) {
  const float p = d * cE, q = d * cX;
  if (inside) {
    *uout = gr_maxf(*uout, gr_maxf(p, q));
  } else {
    *uin = gr_minf(*uin, p);
    *uout = gr_maxf(*uout, q);
  }
}
#endif /* GR_OBSTACLES_H */
