/*
 * gr_oracle.c — CPU restatement of the racing-env step of
 * yufengsjtu/GeneralizableRacing (task DiffLab-Quadcopter-CTBR-Racing-v0).
 *
 * TEST INFRASTRUCTURE ONLY (see gr_oracle.h).  Plain C11, one env at a time,
 * written in the reference's operation order so that, compiled with
 * -ffp-contract=off, it is the bit-level specification the HIP kernel is
 * checked against.  Reference paths are relative to the reference repo root;
 * "IL" = Isaac Lab (external, absent here: those formulas are restated from
 * the Isaac Lab release the reference pins, omni-isaac-lab>=0.27.15, and are
 * "parity unpinned" — no reference test or fixture covers them).
 *
 * Elementary functions (exp, tanh, log, sincos, atan2) and the Philox stream
 * come from the shared headers ../generalizableracing_amd/csrc/gr_{math,rng}.h
 * on purpose: they are not part of the reference algorithm (torch supplies
 * them there), and sharing them is what makes kernel == oracle bit-exact.
 * They are pinned separately against float64 references (tests/test_math.py)
 * and the Random123 known-answer vectors (tests/test_rng.py).
 */
#include "gr_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../generalizableracing_amd/csrc/gr_math.h"
#include "../generalizableracing_amd/csrc/gr_rng.h"
#include "../generalizableracing_amd/csrc/gr_camera.h"
#include "../generalizableracing_amd/csrc/gr_normal_table.h"

static const float GRO_NORMAL_TAB[4 * GR_NORMAL_TABLE_ENTRIES] = GR_NORMAL_TABLE_INIT;

size_t gro_env_size(void) { return sizeof(gro_env); }

/* ------------------------------------------------------------------ IL math */
/* IL omni.isaac.lab.utils.math.quat_rotate: a + b + c with
 * a = v(2w^2-1), b = 2w (q_vec x v), c = 2 q_vec (q_vec . v) */
static void quat_rotate(const float q[4], const float v[3], float o[3]) {
  float s = 2.0f * (q[0] * q[0]) - 1.0f;
  float cx = q[2] * v[2] - q[3] * v[1];
  float cy = q[3] * v[0] - q[1] * v[2];
  float cz = q[1] * v[1] - q[2] * v[0];
  float d = (q[1] * v[0] + q[2] * v[1]) + q[3] * v[2];
  o[0] = (v[0] * s + (cx * q[0]) * 2.0f) + (q[1] * d) * 2.0f;
  o[1] = (v[1] * s + (cy * q[0]) * 2.0f) + (q[2] * d) * 2.0f;
  o[2] = (v[2] * s + (cz * q[0]) * 2.0f) + (q[3] * d) * 2.0f;
}
/* IL quat_rotate_inverse: a - b + c */
static void quat_rotate_inverse(const float q[4], const float v[3], float o[3]) {
  float s = 2.0f * (q[0] * q[0]) - 1.0f;
  float cx = q[2] * v[2] - q[3] * v[1];
  float cy = q[3] * v[0] - q[1] * v[2];
  float cz = q[1] * v[1] - q[2] * v[0];
  float d = (q[1] * v[0] + q[2] * v[1]) + q[3] * v[2];
  o[0] = (v[0] * s - (cx * q[0]) * 2.0f) + (q[1] * d) * 2.0f;
  o[1] = (v[1] * s - (cy * q[0]) * 2.0f) + (q[2] * d) * 2.0f;
  o[2] = (v[2] * s - (cz * q[0]) * 2.0f) + (q[3] * d) * 2.0f;
}
/* IL quat_mul (w,x,y,z), the 8-multiply form */
static void quat_mul(const float a[4], const float b[4], float o[4]) {
  float w1 = a[0], x1 = a[1], y1 = a[2], z1 = a[3];
  float w2 = b[0], x2 = b[1], y2 = b[2], z2 = b[3];
  float ww = (z1 + x1) * (x2 + y2);
  float yy = (w1 - y1) * (w2 + z2);
  float zz = (w1 + y1) * (w2 - z2);
  float xx = (ww + yy) + zz;
  float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  o[0] = (qq - ww) + (z1 - y1) * (y2 - z2);
  o[1] = (qq - xx) + (x1 + w1) * (x2 + w2);
  o[2] = (qq - yy) + (w1 - x1) * (y2 + z2);
  o[3] = (qq - zz) + (z1 + y1) * (w2 - x2);
}
/* IL quat_from_euler_xyz (ZYX composition) */
static void quat_from_euler_xyz(float roll, float pitch, float yaw, float o[4]) {
  float sy, cy, sr, cr, sp, cp;
  gr_sincosf(yaw * 0.5f, &sy, &cy);
  gr_sincosf(roll * 0.5f, &sr, &cr);
  gr_sincosf(pitch * 0.5f, &sp, &cp);
  o[0] = (cy * cr) * cp + (sy * sr) * sp;
  o[1] = (cy * sr) * cp - (sy * cr) * sp;
  o[2] = (cy * cr) * sp + (sy * sr) * cp;
  o[3] = (sy * cr) * cp - (cy * sr) * sp;
}
/* IL matrix_from_quat, third row only (observation.py:31-32 uses [:, 2, :]) */
static void matrix_row2(const float q[4], float o[3]) {
  float r = q[0], i = q[1], j = q[2], k = q[3];
  float two_s = 2.0f / (((r * r + i * i) + j * j) + k * k);
  o[0] = two_s * (i * k - j * r);
  o[1] = two_s * (j * k + i * r);
  o[2] = 1.0f - two_s * (i * i + j * j);
}
static void cross3(const float a[3], const float b[3], float o[3]) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
static float norm3(const float a[3]) { return gr_sqrtf((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]); }
/* torch.nn.functional.cosine_similarity (eps=1e-8): sum((x1/|x1|_eps) * (x2/|x2|_eps)) */
static float cosine_similarity(const float a[3], const float b[3]) {
  float na = gr_maxf(norm3(a), 1e-8f), nb = gr_maxf(norm3(b), 1e-8f);
  return ((a[0] / na) * (b[0] / nb) + (a[1] / na) * (b[1] / nb)) + (a[2] / na) * (b[2] / nb);
}

/* ------------------------------------------------------------- constants */
static float thrust_of_omega(const gr_config* c, double w) {
  return (float)(c->thrustmap[0] * w * w + c->thrustmap[1] * w + c->thrustmap[2]);
}
/* controller_diff.py:96-99  gross thrust bounds (python double, cast at clamp), for the rotor constants
 * k = (k2, k1, k0) of the env (the config's thrust map unless dr_rotor) */
static void thrust_bounds(const gr_config* c, const float k[3], float* lo, float* hi) {
  double tmin = (double)k[0] * c->motor_omega[0] * c->motor_omega[0] + (double)k[1] * c->motor_omega[0] + (double)k[2];
  double tmax = (double)k[0] * c->motor_omega[1] * c->motor_omega[1] + (double)k[1] * c->motor_omega[1] + (double)k[2];
  *lo = (float)(tmin * 4.0);
  *hi = (float)(tmax * 4.0);
  (void)thrust_of_omega;
}
/* diff_action.py:257-262  "medium" action scale/offset */
static void action_scale(const gr_config* c, float m_ctrl, float scale[4], float offset[4]) {
  float weight = m_ctrl * c->gravity;
  float s0 = (weight * c->max_thrust_weight_ratio) / 2.0f;
  scale[0] = s0; offset[0] = s0;
  for (int i = 1; i < 4; ++i) { scale[i] = c->body_rate_bound; offset[i] = 0.0f; }
}

static uint32_t gid_of(const gr_config* c, int i) { return (uint32_t)(c->env_id_offset + i); }
static gr_u32x4 draw(const gr_config* c, uint32_t gid, uint32_t c1, uint32_t tag, uint32_t c3) {
  return gr_philox4x32_10(gid, c1, tag, c3, c->seed_lo, c->seed_hi);
}

/* ----------------------------------------------------------- track table */
static int track_index(const gr_config* c, int type, int level) { return type * c->num_levels + level; }
static const float* gate_rec(const gr_config* c, const gro_tracks* tr, int track, int g) {
  return tr->gates + ((size_t)track * c->max_gates + g) * GR_GATE_FLOATS;
}
static const float* track_rec(const gro_tracks* tr, int track) { return tr->tracks + (size_t)track * GR_TRACK_FLOATS; }
static int track_num_gates(const gro_tracks* tr, int track) { return (int)track_rec(tr, track)[3]; }
static int track_start(const gro_tracks* tr, int track) { return (int)track_rec(tr, track)[2]; }

/* Collision predicate (replaces PhysX contact, racing_ctbr_env.py:65,253-256,
 * and the Warp lattice ray test, diff.lab/utils/mesh_tools.py:128-233):
 * count the 17 lattice points (utils/__init__.py:19-37) of the drone box that
 * lie inside a gate frame (outer box minus the through-hole, trimesh/utils.py:10-33)
 * or below the ground plane. */
static const float LATTICE[17][3] = GR_LATTICE_INIT;

static const float* obst_rec(const gro_tracks* tr, int track, int j) {
  return tr->obst + ((size_t)track * tr->max_obst + j) * GR_OBST_FLOATS;
}
static int track_num_obst(const gro_tracks* tr, int track) { return tr->obst ? tr->obst_count[track] : 0; }

/* Lattice point k = p + (lx*A + ly*B) + lz*C with A, B, C = quat_rotate(q, scaled body
 * axes) — quat_rotate is linear, so this is the reference's center + quat_rotate(q, vec)
 * (mesh_tools.py:187-189) evaluated as a fixed sum.  Inside a gate frame M (rows of
 * R_gate^T) the point is d_g + (lx*A_g + ly*B_g) + lz*C_g, d_g = M(p - c), A_g = M A, ... */
static void gate_frame(const float* g, const float v[3], float o[3]) {
  o[0] = (g[4] * v[0] + g[5] * v[1]) + g[6] * v[2];
  o[1] = (g[8] * v[0] + g[9] * v[1]) + g[10] * v[2];
  o[2] = (g[12] * v[0] + g[13] * v[1]) + g[14] * v[2];
}

int gro_collision_count(const gr_config* c, const gro_tracks* tr, int track, const float p[3], const float q[4]) {
  const float ground = track_rec(tr, track)[0];
  int ng = track_num_gates(tr, track);
  const float ex[3] = {c->collider_half[0], 0.0f, 0.0f}, ey[3] = {0.0f, c->collider_half[1], 0.0f},
              ez[3] = {0.0f, 0.0f, c->collider_half[2]};
  float A[3], B[3], Cz[3];
  quat_rotate(q, ex, A);
  quat_rotate(q, ey, B);
  quat_rotate(q, ez, Cz);
  /* obstacles (walls / orbits / ground obstacles, trimesh/racing_terrains.py:87-150 et al.):
   * every obstacle of the track, no culling */
  uint32_t obst_mask = 0u;
  const int no = track_num_obst(tr, track);
  for (int j = 0; j < no; ++j) obst_mask |= gr_obst_lattice_mask(obst_rec(tr, track, j), p, A, B, Cz, LATTICE);
  int count = 0;
  for (int k = 0; k < 17; ++k) {
    const float lx = LATTICE[k][0], ly = LATTICE[k][1], lz = LATTICE[k][2];
    float oz = (lx * A[2] + ly * B[2]) + lz * Cz[2];
    int inside = p[2] + oz < ground; /* below the ground plane (ground box top) */
    for (int g = 0; g < ng && !inside; ++g) {
      const float* gr = gate_rec(c, tr, track, g);
      float d[3] = {p[0] - gr[0], p[1] - gr[1], p[2] - gr[2]}, dg[3], Ag[3], Bg[3], Cg[3];
      gate_frame(gr, d, dg);
      gate_frame(gr, A, Ag);
      gate_frame(gr, B, Bg);
      gate_frame(gr, Cz, Cg);
      float l0 = dg[0] + ((lx * Ag[0] + ly * Bg[0]) + lz * Cg[0]);
      float l1 = dg[1] + ((lx * Ag[1] + ly * Bg[1]) + lz * Cg[1]);
      float l2 = dg[2] + ((lx * Ag[2] + ly * Bg[2]) + lz * Cg[2]);
      float a0 = gr_fabsf(l0), a1 = gr_fabsf(l1), a2 = gr_fabsf(l2);
      int in_outer = (a0 <= gr[16]) & (a1 <= gr[17]) & (a2 <= gr[15]);
      int in_hole = (a0 < gr[7]) & (a1 < gr[11]);
      inside = in_outer & !in_hole; /* frame = outer box minus the through-hole */
    }
    count += inside | (int)((obst_mask >> k) & 1u);
  }
  return count;
}

/* allocation matrix and its inverse (controller_diff.py:56-69; fp32 as torch builds it) for torque ratio k */
static void motor_allocation(const gr_config* c, float k, float B[4][4], float Bi[4][4]) {
  float l = c->arm_length * 0.707106769f;
  static const float sx[4] = {1, -1, -1, 1}, sy[4] = {-1, -1, 1, 1}, sz[4] = {1, -1, 1, -1};
  for (int j = 0; j < 4; ++j) {
    B[0][j] = 1.0f; B[1][j] = l * sx[j]; B[2][j] = l * sy[j]; B[3][j] = k * sz[j];
    Bi[j][0] = 0.25f; Bi[j][1] = sx[j] / (4.0f * l); Bi[j][2] = sy[j] / (4.0f * l); Bi[j][3] = sz[j] / (4.0f * k);
  }
}

/* --------------------------------------------------------- controller */
/* ThrustController.update, thrust_controller_diff.py:182-186, in place: desired rotor thrusts ->
 * Thrust2Omega (:167-176) -> w <- c w + (1 - c) w_des, c = exp(-(1/tau) dt) (:117-118) ->
 * Omega2Thrust (:178-179) */
static void motor_update(const gr_config* c, const float rk[3], float f[4], float motor_w[4]) {
  double k2 = rk[0], k1 = rk[1], k0 = rk[2];
  float cc = gr_expf(-(float)(1.0 / (double)c->motor_tau) * c->step_dt);
  for (int i = 0; i < 4; ++i) {
    float t3 = (float)(k1 * k1) - (float)(4.0 * k2) * ((float)k0 - f[i]);
    float wdes = (float)(1.0 / (2.0 * k2)) * ((float)(-k1) + gr_sqrtf(t3));
    motor_w[i] = cc * motor_w[i] + (1.0f - cc) * wdes;
    f[i] = ((float)k2 * motor_w[i] * motor_w[i] + (float)k1 * motor_w[i]) + (float)k0;
  }
}

/* CTBRController.compute, controller_diff.py:120-144 (use_motor_model=False
 * returns (T, tau) at :137-138); motor model :140-144 + thrust_controller_diff.py:83-102 */
/* rk: the env's rotor constants k2 k1 k0 kappa (config C5's dr_rotor; else the config's) */
static void ctbr_compute(const gr_config* c, const float cmd[4], const float wb[3], const float ab[3], const float Kp[3],
                         const float Kd[3], float cT, const float ctau[3], float* T, float tau[3], float motor_w[4],
                         const float rk[4], float out_tt[4]) {
  float tlo, thi;
  thrust_bounds(c, rk, &tlo, &thi);
  float T_des = gr_clampf(cmd[0], tlo, thi);
  *T = (1.0f - cT) * T_des + cT * (*T);
  const float* J = c->inertia; /* controller inertia: nominal, diff_action.py:59 */
  float err[3], Jw[3], cr[3];
  for (int i = 0; i < 3; ++i) err[i] = gr_clampf(cmd[i + 1], -c->body_rate_bound, c->body_rate_bound) - wb[i];
  for (int i = 0; i < 3; ++i) Jw[i] = J[i] * wb[i];
  cross3(wb, Jw, cr);
  for (int i = 0; i < 3; ++i) {
    float tdes = (J[i] * (Kp[i] * err[i]) + cr[i]) - Kd[i] * ab[i];
    tau[i] = (1.0f - ctau[i]) * tdes + ctau[i] * tau[i];
  }
  out_tt[0] = *T; out_tt[1] = tau[0]; out_tt[2] = tau[1]; out_tt[3] = tau[2];
  if (!c->use_motor_model) return;
  /* allocation B (controller_diff.py:56-69): rows [1 1 1 1], l/sqrt2 [1 -1 -1 1],
   * l/sqrt2 [-1 -1 1 1], kappa [1 -1 1 -1]; B^-1 entries 1/4, +-1/(4l), +-1/(4 kappa) */
  float B[4][4], Bi[4][4];
  motor_allocation(c, rk[3], B, Bi);
  float f[4];
  for (int r = 0; r < 4; ++r)
    f[r] = ((out_tt[0] * Bi[r][0] + out_tt[1] * Bi[r][1]) + out_tt[2] * Bi[r][2]) + out_tt[3] * Bi[r][3];
  double w1 = c->motor_omega[1];
  float fmax = (float)((double)rk[0] * w1 * w1 + (double)rk[1] * w1 + (double)rk[2]);
  for (int i = 0; i < 4; ++i) f[i] = gr_clampf(f[i], 0.0f, fmax); /* controller_diff.py:142 */
  motor_update(c, rk, f, motor_w);
  for (int r = 0; r < 4; ++r) out_tt[r] = ((f[0] * B[r][0] + f[1] * B[r][1]) + f[2] * B[r][2]) + f[3] * B[r][3];
}

/* ------------------------------------------------------------ integrator */
/* DroneDynamics.step, droneDynamics.py:119-135 (explicit Euler, one step of dt) */
static void dd_explicit(float m, const float J[3], const float k2[3], const float k1[3], const float tt[4], float dt,
                        float gz, float p[3], float q[4], float v[3], float w[3], float a_out[3], float al_out[3]) {
  float vb[3];
  quat_rotate_inverse(q, v, vb);
  float thr[3] = {0.0f, 0.0f, tt[0]};
  for (int i = 0; i < 3; ++i) thr[i] = (thr[i] - (k2[i] * vb[i]) * gr_fabsf(vb[i])) - k1[i] * vb[i];
  float tw[3];
  quat_rotate(q, thr, tw);
  float a[3] = {0.0f + tw[0] / m, 0.0f + tw[1] / m, -gz + tw[2] / m};
  float Jw[3] = {J[0] * w[0], J[1] * w[1], J[2] * w[2]}, cr[3];
  cross3(w, Jw, cr);
  float al[3];
  for (int i = 0; i < 3; ++i) {
    float ji = 1.0f / J[i];
    al[i] = ji * tt[i + 1] - ji * cr[i];
  }
  for (int i = 0; i < 3; ++i) p[i] = (p[i] + v[i] * dt) + ((0.5f * a[i]) * dt) * dt;
  float wq[4] = {0.0f, w[0], w[1], w[2]}, qd[4];
  quat_mul(q, wq, qd);
  for (int i = 0; i < 4; ++i) q[i] = q[i] + (0.5f * qd[i]) * dt;
  float n = gr_sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / n;
  for (int i = 0; i < 3; ++i) v[i] = v[i] + a[i] * dt;
  for (int i = 0; i < 3; ++i) w[i] = w[i] + al[i] * dt;
  for (int i = 0; i < 3; ++i) { a_out[i] = a[i]; al_out[i] = al[i]; }
}

/* Semi-implicit Euler substep (PhysX-like role; no in-repo reference formula):
 * body wrench held over the substep (diff_action.py:209-210 applies the same
 * force each of the `decimation` substeps), drag from the pre-step body velocity. */
static void si_substep(float m, const float J[3], const float fb[3], const float tb[3], float h, float gz, float p[3],
                       float q[4], float v[3], float w[3], float a_out[3], float al_out[3]) {
  float tw[3];
  quat_rotate(q, fb, tw);
  float a[3] = {0.0f + tw[0] / m, 0.0f + tw[1] / m, -gz + tw[2] / m};
  float Jw[3] = {J[0] * w[0], J[1] * w[1], J[2] * w[2]}, cr[3];
  cross3(w, Jw, cr);
  float al[3];
  for (int i = 0; i < 3; ++i) al[i] = (tb[i] - cr[i]) / J[i];
  for (int i = 0; i < 3; ++i) v[i] = v[i] + a[i] * h;
  for (int i = 0; i < 3; ++i) w[i] = w[i] + al[i] * h;
  for (int i = 0; i < 3; ++i) p[i] = p[i] + v[i] * h;
  float wq[4] = {0.0f, w[0], w[1], w[2]}, qd[4];
  quat_mul(q, wq, qd);
  for (int i = 0; i < 4; ++i) q[i] = q[i] + (0.5f * qd[i]) * h;
  float n = gr_sqrtf(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  for (int i = 0; i < 4; ++i) q[i] = q[i] / n;
  for (int i = 0; i < 3; ++i) { a_out[i] = a[i]; al_out[i] = al[i]; }
}

/* ------------------------------------------------------------------ init */
void gro_type_starts(const gr_config* c, int32_t* ts) {
  /* IL TerrainImporter: terrain_types = floor(arange(N) / (N / num_cols)), fp32 divisor */
  float s = (float)((double)c->num_envs / (double)c->num_types);
  for (int t = 0; t <= c->num_types; ++t) {
    double lim = (double)t * (double)s; /* exact: 24-bit mantissa times t < 2^8 */
    int i = (int)ceil(lim);
    if (i > c->num_envs) i = c->num_envs;
    ts[t] = i;
  }
}

static void write_last_ctbr0(const gr_config* c, const gro_env* e, float* row) {
  float sc[4], of[4];
  action_scale(c, e->m_ctrl, sc, of);
  float ctbr0 = gr_tanhf(0.0f) * sc[0] + of[0];
  row[12] = ctbr0 / e->m_ctrl;
  for (int i = 1; i < 4; ++i) row[12 + i] = gr_tanhf(0.0f) * sc[i] + of[i];
}

void gro_init(const gr_config* c, gro_env* envs, int n, gro_out* out) {
  int32_t ts[260];
  gro_type_starts(c, ts);
  for (int i = 0; i < n; ++i) {
    gro_env* e = &envs[i];
    memset(e, 0, sizeof(*e));
    uint32_t gid = gid_of(c, i);
    gr_u32x4 b0 = draw(c, gid, 0, GR_TAG_STATIC, 0), b1 = draw(c, gid, 0, GR_TAG_STATIC, 1);
    gr_u32x4 b2 = draw(c, gid, 0, GR_TAG_STATIC, 2), b3 = draw(c, gid, 0, GR_TAG_STATIC, 3);
    gr_u32x4 b4 = draw(c, gid, 0, GR_TAG_STATIC, 4);
    int dr = c->dr_startup;
    /* config C5 (not in the reference): thrust map and kappa x U(lo, hi) per env, for the env's lifetime */
    e->rotor[0] = c->thrustmap[0]; e->rotor[1] = c->thrustmap[1]; e->rotor[2] = c->thrustmap[2];
    e->rotor[3] = c->kappa;
    if (dr && c->dr_rotor) {
      gr_u32x4 b5 = draw(c, gid, 0, GR_TAG_STATIC, 5);
      float lo = c->rotor_scale_range[0], hi = c->rotor_scale_range[1];
      e->rotor[0] = c->thrustmap[0] * gr_uniform(b5.x, lo, hi);
      e->rotor[1] = c->thrustmap[1] * gr_uniform(b5.y, lo, hi);
      e->rotor[2] = c->thrustmap[2] * gr_uniform(b5.z, lo, hi);
      e->rotor[3] = c->kappa * gr_uniform(b5.w, lo, hi);
    }
    float plo = c->pid_scale_range[0], phi = c->pid_scale_range[1];
    float dlo = c->delay_scale_range[0], dhi = c->delay_scale_range[1];
    /* events.py:105-137 randomize_rate_controller_gain_and_thrust_delay */
    float skp[3] = {gr_uniform(b0.x, plo, phi), gr_uniform(b0.y, plo, phi), gr_uniform(b0.z, plo, phi)};
    float skd[3] = {gr_uniform(b0.w, plo, phi), gr_uniform(b1.x, plo, phi), gr_uniform(b1.y, plo, phi)};
    float sdt = gr_uniform(b1.z, dlo, dhi);
    float sdq[3] = {gr_uniform(b1.w, dlo, dhi), gr_uniform(b2.x, dlo, dhi), gr_uniform(b2.y, dlo, dhi)};
    /* events.py:30-103 randomize_articulation_mass_and_inertia (add / scale) */
    float madd = gr_uniform(b2.z, c->mass_add_range[0], c->mass_add_range[1]);
    float sj[3] = {gr_uniform(b2.w, c->inertia_scale_range[0], c->inertia_scale_range[1]),
                   gr_uniform(b3.x, c->inertia_scale_range[0], c->inertia_scale_range[1]),
                   gr_uniform(b3.y, c->inertia_scale_range[0], c->inertia_scale_range[1])};
    for (int k = 0; k < 3; ++k) {
      e->Kp[k] = dr ? c->rate_gain_p[k] * skp[k] : c->rate_gain_p[k];
      e->Kd[k] = dr ? c->rate_gain_d[k] * skd[k] : c->rate_gain_d[k];
    }
    float tauT = dr ? c->thrust_ctrl_delay * sdt : c->thrust_ctrl_delay;
    e->cT = gr_expf(-c->step_dt / tauT);
    for (int k = 0; k < 3; ++k) {
      float tq = dr ? c->torque_ctrl_delay[k] * sdq[k] : c->torque_ctrl_delay[k];
      e->ctau[k] = gr_expf(-c->step_dt / tq);
    }
    e->m_ctrl = c->mass; /* diff_action.py:55 reads the mass before the startup event runs */
    float mp = (dr && c->dr_plant) ? c->mass + madd : c->mass;
    e->m_plant = mp;
    for (int k = 0; k < 3; ++k)
      e->J[k] = (dr && c->dr_plant) ? (c->inertia[k] * (mp / c->mass)) * sj[k] : c->inertia[k];
    /* initial level: IL _compute_env_origins_curriculum randint(0, max_init+1) */
    e->level = (int)gr_floorf(gr_u01(b3.z) * (float)(c->max_init_level + 1));
    /* diff_action.py:86 thr_est_error = 1 + randn * 0.02 */
    float z0, z1;
    gr_box_muller(b3.w, b4.x, &z0, &z1);
    e->thr_err = 1.0f + z0 * 0.02f;
    e->noise_level = 1.0f;
    /* droneDynamics.py:25-36 (no randomness at construction) */
    for (int k = 0; k < 3; ++k) {
      e->k2[k] = c->drag2[k] * c->mass;
      e->k1[k] = c->drag1[k] * c->mass;
    }
    e->k2[2] = e->k2[2] * c->z_drag;
    e->k1[2] = e->k1[2] * c->z_drag;
    for (int k = 0; k < 3; ++k) e->p[k] = c->spawn_pos[k];
    e->q[0] = 1.0f;
    e->azero = 1;
    int type = 0;
    for (int t = 1; t < c->num_types; ++t) type += (i >= ts[t]);
    e->type = type;
    /* initial observation buffers: last action = ctbr(0) (DiffActions._raw_actions starts at zero) */
    float* pol = out->obs_policy + (size_t)i * 16;
    float* cri = out->obs_critic + (size_t)i * 16;
    for (int k = 0; k < 16; ++k) { pol[k] = 0.0f; cri[k] = 0.0f; }
    write_last_ctbr0(c, e, cri);
    write_last_ctbr0(c, e, pol);
    out->obs_aux[i] = 0.0f;
    out->reward[i] = 0.0f;
    out->terminated[i] = 0;
    out->time_out[i] = 0;
    out->dones[i] = 0;
  }
}

/* ------------------------------------------------------------------ reset */
typedef struct logacc { double s[GR_LOG_SLOTS]; } logacc;

/* noise of the current (out[0..2]) and next (out[3..5]) gate pose: one draw per
 * (episode, gates passed); U(-r, r) * noise_level per axis, commands.py:287-289,329-350 */
static void gate_noise(const gr_config* c, const gro_env* e, uint32_t gid, float out[6]) {
  if (!c->add_gate_noise) { for (int k = 0; k < 6; ++k) out[k] = 0.0f; return; }
  uint32_t f[6];
  gr_fields6(draw(c, gid, (uint32_t)e->epoch, GR_TAG_GATE, (uint32_t)e->acc), f);
  for (int k = 0; k < 6; ++k) {
    float lo = (-c->gate_noise_pos[k % 3]) * e->noise_level, hi = c->gate_noise_pos[k % 3] * e->noise_level;
    out[k] = lo + gr_f21(f[k]) * (hi - lo);
  }
}

/* ManagerBasedDiffRLEnv._reset_idx, manager_based_diff_rl_env.py:362-410, for one env */
static void reset_env(const gr_config* c, gro_env* e, uint32_t gid, const gro_tracks* tr) {
  /* curriculum first (:369): curriculums.py:25-38 + IL update_env_origins */
  int up = e->acc >= c->level_up_threshold, down = e->acc < c->level_down_threshold;
  int lvl = e->level + up - down;
  uint32_t ep = (uint32_t)e->epoch + 1u;
  /* 24 x 21-bit fields: pos 0-2, att 3-5, vel 6-11, z-drag 12, k2 13-15, k1 16-18, level 19, thr 20-21 */
  uint32_t f[24];
  gr_fields6(draw(c, gid, ep, GR_TAG_RESET, 0), f);
  gr_fields6(draw(c, gid, ep, GR_TAG_RESET, 1), f + 6);
  gr_fields6(draw(c, gid, ep, GR_TAG_RESET, 2), f + 12);
  gr_fields6(draw(c, gid, ep, GR_TAG_RESET, 3), f + 18);
  if (lvl >= c->num_levels) lvl = (int)gr_floorf(gr_f21(f[19]) * (float)c->num_levels);
  else if (lvl < 0) lvl = 0;
  if (c->noise_curriculum) { /* curriculums.py:40-54 + commands.py:385-402 */
    float upf = e->acc >= c->noise_enhance_threshold ? 1.0f + c->noise_enhance : 1.0f;
    float dnf = e->acc < c->noise_decay_threshold ? 1.0f - c->noise_decay : 1.0f;
    e->noise_level = e->noise_level * upf;
    e->noise_level = e->noise_level * dnf;
  }
  e->level = lvl;
  int track = track_index(c, e->type, lvl);
  /* reset_root_state_racing, events.py:139-177 (env-local frame: world - env_origin) */
  float rp[6], rv[6];
  for (int k = 0; k < 3; ++k) {
    rp[k] = gr_uniform21(f[k], -c->reset_pos_half[k], c->reset_pos_half[k]);
    rp[3 + k] = gr_uniform21(f[3 + k], -c->reset_att_half[k], c->reset_att_half[k]);
  }
  for (int k = 0; k < 6; ++k) rv[k] = gr_uniform21(f[6 + k], -c->reset_vel_half[k], c->reset_vel_half[k]);
  for (int k = 0; k < 3; ++k) e->p[k] = c->spawn_pos[k] + rp[k];
  int start = track_start(tr, track);
  const float* g0 = gate_rec(c, tr, track, start);
  float tx = g0[0] - e->p[0], ty = g0[1] - e->p[1];
  float yaw = gr_wrap_to_pi(gr_atan2f(ty, tx)) + rp[5];
  float qd[4], qid[4] = {1.0f, 0.0f, 0.0f, 0.0f};
  quat_from_euler_xyz(rp[3], rp[4], yaw, qd);
  quat_mul(qid, qd, e->q);
  for (int k = 0; k < 3; ++k) e->v[k] = 0.0f + rv[k];
  float ww[3] = {0.0f + rv[3], 0.0f + rv[4], 0.0f + rv[5]};
  quat_rotate_inverse(e->q, ww, e->w); /* droneDynamics.py:119 reset_state: ang_vel_b */
  /* action manager: IL ActionManager.reset zeroes _action/_prev_action; DiffActions.reset_idx
   * (diff_action.py:223-233): controller filters, drag DR, thrust-estimate error */
  e->azero = 1;
  e->T = 0.0f;
  for (int k = 0; k < 3; ++k) { e->tau[k] = 0.0f; e->alpha[k] = 0.0f; }
  for (int k = 0; k < 4; ++k) e->motor_w[k] = 0.0f;
  if (c->random_drag) { /* droneDynamics.py:50-57 */
    float z = c->z_drag + gr_f21(f[12]) * c->z_drag_rand;
    float u2[3] = {gr_f21(f[13]), gr_f21(f[14]), gr_f21(f[15])};
    float u1[3] = {gr_f21(f[16]), gr_f21(f[17]), gr_f21(f[18])};
    for (int k = 0; k < 3; ++k) {
      e->k2[k] = c->drag2[k] * e->m_ctrl + u2[k] * c->drag2_rand;
      e->k1[k] = c->drag1[k] * e->m_ctrl + u1[k] * c->drag1_rand;
    }
    e->k2[2] = e->k2[2] * z;
    e->k1[2] = e->k1[2] * z;
  }
  float z0, z1;
  gr_box_muller21(f[20], f[21], &z0, &z1);
  e->thr_err = 1.0f + z0 * 0.01f;
  /* reward manager: episode sums; command manager: metrics + _resample_command (commands.py:262-306) */
  for (int k = 0; k < 7; ++k) e->ep_sum[k] = 0.0f;
  e->m_actrate = 0.0f;
  e->acc = 0;
  e->gate_id = start;
  e->ep_len = 0;
  e->epoch = (int32_t)ep;
}

/* ------------------------------------------------------------ observations */
static void compute_obs(const gr_config* c, gro_env* e, uint32_t gid, uint32_t cnt, const gro_tracks* tr,
                        const float last_ctbr[4], float aux, float* pol, float* cri, float* auxo) {
  int track = track_index(c, e->type, e->level);
  int ng = track_num_gates(tr, track);
  const float* g = gate_rec(c, tr, track, e->gate_id);
  const float* gn = gate_rec(c, tr, track, (e->gate_id + 1) % ng);
  float vb[3], r2[3];
  quat_rotate_inverse(e->q, e->v, vb);
  matrix_row2(e->q, r2);
  float d[3] = {g[0] - e->p[0], g[1] - e->p[1], g[2] - e->p[2]};
  float dn[3] = {gn[0] - g[0], gn[1] - g[1], gn[2] - g[2]};
  float cg[3], cn[3];
  quat_rotate_inverse(e->q, d, cg);
  quat_rotate_inverse(e->q, dn, cn);
  for (int k = 0; k < 3; ++k) { cri[k] = vb[k]; cri[3 + k] = r2[k]; cri[6 + k] = cg[k]; cri[9 + k] = cn[k]; }
  for (int k = 0; k < 4; ++k) cri[12 + k] = last_ctbr[k];
  /* policy: observation.py:47-53 (lin vel noise), :22-32 (attitude noise), commands.py:208-221 (noisy gates) */
  float nz[6] = {0};
  if (c->obs_noise) { /* randn(N,3) for the velocity and for the attitude noise */
    uint32_t f[6];
    gr_fields6(draw(c, gid, cnt, GR_TAG_OBS, 0), f);
    for (int k = 0; k < 6; ++k) nz[k] = gr_normal21(f[k], GRO_NORMAL_TAB);
  }
  float qn[4], qq[4], r2n[3];
  quat_from_euler_xyz(nz[3] * c->obs_att_noise, nz[4] * c->obs_att_noise, nz[5] * c->obs_att_noise, qn);
  quat_mul(e->q, qn, qq);
  matrix_row2(qq, r2n);
  float gnz[6];
  gate_noise(c, e, gid, gnz);
  float gw[3] = {g[0] + gnz[0], g[1] + gnz[1], g[2] + gnz[2]};
  float gnw[3] = {gn[0] + gnz[3], gn[1] + gnz[4], gn[2] + gnz[5]};
  float dp[3] = {gw[0] - e->p[0], gw[1] - e->p[1], gw[2] - e->p[2]};
  float dnp[3] = {gnw[0] - gw[0], gnw[1] - gw[1], gnw[2] - gw[2]};
  float pg[3], pn[3];
  quat_rotate_inverse(e->q, dp, pg);
  quat_rotate_inverse(e->q, dnp, pn);
  for (int k = 0; k < 3; ++k) {
    pol[k] = vb[k] * (1.0f + nz[k] * c->obs_lin_vel_noise);
    pol[3 + k] = r2n[k];
    pol[6 + k] = pg[k];
    pol[9 + k] = pn[k];
  }
  for (int k = 0; k < 4; ++k) pol[12 + k] = last_ctbr[k];
  *auxo = aux;
}

static void finalize_log(const gr_config* c, const logacc* L, float* out) {
  double nr = L->s[GR_LOG_NRESET];
  /* no env reset this call: the reference leaves extras["log"] (set only in _reset_idx,
   * manager_based_diff_rl_env.py:380) untouched, i.e. the previous step's values */
  if (nr == 0.0) return;
  for (int k = 0; k < GR_LOG_SLOTS; ++k) out[k] = 0.0f;
  out[GR_LOG_NRESET] = (float)nr;
  for (int k = 0; k < 7; ++k) out[GR_LOG_EPSUM0 + k] = (float)(L->s[GR_LOG_EPSUM0 + k] / nr / c->episode_length_s);
  for (int k = GR_LOG_ACC; k <= GR_LOG_M_ANGSPD; ++k) out[k] = (float)(L->s[k] / nr);
  for (int k = GR_LOG_T_TIMEOUT; k <= GR_LOG_T_BADPOSE; ++k) out[k] = (float)L->s[k];
  out[GR_LOG_LEVEL] = (float)(L->s[GR_LOG_LEVEL] / c->num_envs);
  out[GR_LOG_NOISE] = (float)(L->s[GR_LOG_NOISE] / c->num_envs);
}

void gro_reset(const gr_config* c, gro_env* envs, int n, const uint8_t* mask, const gro_tracks* tr, uint32_t* counter,
               gro_out* out) {
  logacc L;
  memset(&L, 0, sizeof(L));
  uint32_t cnt = *counter;
  for (int i = 0; i < n; ++i) {
    gro_env* e = &envs[i];
    uint32_t gid = gid_of(c, i);
    if (!mask || mask[i]) {
      L.s[GR_LOG_NRESET] += 1;
      for (int k = 0; k < 7; ++k) L.s[GR_LOG_EPSUM0 + k] += e->ep_sum[k];
      L.s[GR_LOG_ACC] += e->acc;
      L.s[GR_LOG_M_ACTRATE] += e->m_actrate;
      L.s[GR_LOG_M_LINSPD] += norm3(e->v);
      L.s[GR_LOG_M_ANGSPD] += norm3(e->w);
      L.s[GR_LOG_T_TIMEOUT] += out->time_out[i] ? 1 : 0;
      reset_env(c, e, gid, tr);
    }
    L.s[GR_LOG_LEVEL] += e->level;
    L.s[GR_LOG_NOISE] += e->noise_level;
    float lc[4];
    for (int k = 0; k < 4; ++k) lc[k] = out->obs_critic[(size_t)i * 16 + 12 + k];
    compute_obs(c, e, gid, cnt, tr, lc, out->obs_aux[i], out->obs_policy + (size_t)i * 16,
                out->obs_critic + (size_t)i * 16, &out->obs_aux[i]);
  }
  finalize_log(c, &L, out->log_out);
  *counter = cnt + 1u;
}

void gro_observe(const gr_config* c, gro_env* envs, int n, const gro_tracks* tr, uint32_t* counter, gro_out* out) {
  uint32_t cnt = *counter;
  for (int i = 0; i < n; ++i) {
    float lc[4];
    for (int k = 0; k < 4; ++k) lc[k] = out->obs_critic[(size_t)i * 16 + 12 + k];
    compute_obs(c, &envs[i], gid_of(c, i), cnt, tr, lc, out->obs_aux[i], out->obs_policy + (size_t)i * 16,
                out->obs_critic + (size_t)i * 16, &out->obs_aux[i]);
  }
  *counter = cnt + 1u;
}

/* -------------------------------------------------------------------- step */
void gro_step(const gr_config* c, gro_env* envs, int n, const float* actions, const gro_tracks* tr, uint32_t* counter,
              gro_out* out) {
  logacc Lsum;
  memset(&Lsum, 0, sizeof(Lsum));
  uint32_t cnt = *counter;
  const float dt = c->step_dt;
  const float w[7] = {c->w_progress, c->w_body_rate, c->w_action_rate, c->w_collision,
                      c->w_perception, c->w_success, c->w_bad_pose};
  /* envs are independent: one OpenMP team over them (OMP_NUM_THREADS; per-env results do not
   * depend on the thread count, only the summation order of the log means does) */
#pragma omp parallel
  {
  logacc L;
  memset(&L, 0, sizeof(L));
#pragma omp for schedule(static)
  for (int i = 0; i < n; ++i) {
    gro_env* e = &envs[i];
    uint32_t gid = gid_of(c, i);
    const float* a = actions + (size_t)i * 4;
    float lin_prev = norm3(e->v), ang_prev = norm3(e->w), mar_prev = e->m_actrate;
    /* 1. DiffActionManager.process_action (action_manager.py:44-45): prev <- action <- a.
     * 2. DiffActions.process_actions: one-step lag (diff_action.py:160-163).
     * Every use of the lagged / previous raw action goes through tanh() (:174,
     * rewards.py:194,201-202, observation.py:61), so the lag record stores
     * tanh(a) and each action is squashed once (bit-identical values). */
    float th_cur[4], th_prev[4], th_raw[4];
    for (int k = 0; k < 4; ++k) th_cur[k] = gr_tanhf(a[k]);
    for (int k = 0; k < 4; ++k) {
      th_prev[k] = e->azero ? 0.0f : e->lag[k]; /* IL ActionManager.reset zeroes _action (tanh(0) = 0) */
      th_raw[k] = c->action_lag ? e->lag[k] : th_cur[k];
      e->lag[k] = th_cur[k];
    }
    e->azero = 0;
    /* tanh -> scale/offset -> thrust-estimate error (:174-176) */
    float sc[4], of[4], cmd[4];
    action_scale(c, e->m_ctrl, sc, of);
    for (int k = 0; k < 4; ++k) cmd[k] = th_raw[k] * sc[k] + of[k];
    cmd[0] = cmd[0] * e->thr_err;
    /* 3. controller (:182) with the state "read from sim" (:126-154) */
    float tt[4];
    const float nominal[4] = {c->thrustmap[0], c->thrustmap[1], c->thrustmap[2], c->kappa};
    ctbr_compute(c, cmd, e->w, e->alpha, e->Kp, e->Kd, e->cT, e->ctau, &e->T, e->tau, e->motor_w,
                 c->dr_rotor ? e->rotor : nominal, tt);
    /* 4. physics (:189-203): wrench held over the substeps */
    int track = track_index(c, e->type, e->level);
    float m = c->dr_plant ? e->m_plant : e->m_ctrl;
    const float* J = c->dr_plant ? e->J : c->inertia;
    float acc_l[3], al[3];
    int contact_count = 0;
    if (c->integrator == GR_INTEGRATOR_DD_EXPLICIT) {
      dd_explicit(m, J, e->k2, e->k1, tt, dt, c->gravity, e->p, e->q, e->v, e->w, acc_l, al);
      contact_count = gro_collision_count(c, tr, track, e->p, e->q);
    } else {
      float vb[3], fb[3] = {0.0f, 0.0f, tt[0]};
      quat_rotate_inverse(e->q, e->v, vb);
      for (int k = 0; k < 3; ++k) fb[k] = (fb[k] - (e->k2[k] * vb[k]) * gr_fabsf(vb[k])) - e->k1[k] * vb[k];
      float h = c->sim_dt;
      for (int s = 0; s < c->decimation; ++s) {
        si_substep(m, J, fb, tt + 1, h, c->gravity, e->p, e->q, e->v, e->w, acc_l, al);
        int cc = gro_collision_count(c, tr, track, e->p, e->q);
        if (cc > contact_count) contact_count = cc; /* contact history: max over substeps */
      }
    }
    for (int k = 0; k < 3; ++k) e->alpha[k] = al[k];
    /* 5. counters (:215) */
    e->ep_len += 1;
    /* 6. terminations (:218-220), racing_ctbr_env.py:248-260 */
    int time_out = e->ep_len >= c->max_episode_length;
    int contact = contact_count > c->collision_count_threshold;
    float origin_z = track_rec(tr, track)[1];
    float zw = e->p[2] + origin_z;
    int oob = (zw < c->out_of_bound[0]) | (zw > c->out_of_bound[1]); /* termination.py:15-22 */
    int bad = (1.0f - 2.0f * (e->q[1] * e->q[1] + e->q[2] * e->q[2])) < 0.0f; /* termination.py:24-33, see DESIGN.md */
    int c_term = c->stage == 0 ? oob : contact;
    int terminated = (c->term_contact && c_term) | (c->term_bad_pose && bad);
    /* 7. rewards (:222), rewards.py:154-253, weights racing_ctbr_env.py:281-328, IL RewardManager: f*w*dt */
    const float* g = gate_rec(c, tr, track, e->gate_id);
    float vb[3], dg[3] = {g[0] - e->p[0], g[1] - e->p[1], g[2] - e->p[2]}, gb[3];
    quat_rotate_inverse(e->q, e->v, vb);
    quat_rotate_inverse(e->q, dg, gb);
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
    float dist = norm3(dg);
    int near_gate = dist < c->gate_threshold;
    f[5] = (float)near_gate * (1.0f / (dist * dist + 1.0f));
    f[6] = (float)bad;
    float rew = 0.0f;
    for (int k = 0; k < 7; ++k) {
      if (w[k] == 0.0f) continue;
      float v = (f[k] * w[k]) * dt;
      rew = rew + v;
      e->ep_sum[k] = e->ep_sum[k] + v;
    }
    out->reward[i] = rew;
    float aux = near_gate ? 1.0f : 0.0f;
    e->m_actrate = f[2];
    /* 8. reset (:232-240) */
    int done = terminated | time_out;
    out->terminated[i] = (uint8_t)terminated;
    out->time_out[i] = (uint8_t)time_out;
    out->dones[i] = done;
    if (done) {
      L.s[GR_LOG_NRESET] += 1;
      for (int k = 0; k < 7; ++k) L.s[GR_LOG_EPSUM0 + k] += e->ep_sum[k];
      L.s[GR_LOG_ACC] += e->acc;
      L.s[GR_LOG_M_ACTRATE] += mar_prev;
      L.s[GR_LOG_M_LINSPD] += lin_prev;
      L.s[GR_LOG_M_ANGSPD] += ang_prev;
      L.s[GR_LOG_T_TIMEOUT] += time_out;
      L.s[GR_LOG_T_CONTACT] += c_term;
      L.s[GR_LOG_T_BADPOSE] += bad;
      reset_env(c, e, gid, tr);
    }
    L.s[GR_LOG_LEVEL] += e->level;
    L.s[GR_LOG_NOISE] += e->noise_level;
    /* 9. command compute (:249): _update_metrics then _update_command (commands.py:247-260, 308-350) */
    {
      int tk = track_index(c, e->type, e->level);
      const float* gg = gate_rec(c, tr, tk, e->gate_id);
      float dd[3] = {gg[0] - e->p[0], gg[1] - e->p[1], gg[2] - e->p[2]};
      if (norm3(dd) < c->gate_threshold) {
        e->acc += 1;
        e->gate_id = (e->gate_id + 1) % track_num_gates(tr, tk);
      }
    }
    /* 10. observations (:264) */
    float lc[4];
    for (int k = 0; k < 4; ++k) lc[k] = th_raw[k] * sc[k] + of[k];
    lc[0] = lc[0] / e->m_ctrl; /* observation.py:55-63 */
    compute_obs(c, e, gid, cnt, tr, lc, aux, out->obs_policy + (size_t)i * 16, out->obs_critic + (size_t)i * 16,
                &out->obs_aux[i]);
  }
#pragma omp critical
  for (int k = 0; k < GR_LOG_SLOTS; ++k) Lsum.s[k] += L.s[k];
  }
  finalize_log(c, &Lsum, out->log_out);
  *counter = cnt + 1u;
}

int gro_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------ test hooks */
void gro_test_dynamics(const gr_config* c, int n, int mode, const float* si, const float* ab, const float* cmd,
                       const float* ci, const float* par, const float* drag, float* so, float* co, float* xo) {
  const float nominal[4] = {c->thrustmap[0], c->thrustmap[1], c->thrustmap[2], c->kappa};
  for (int i = 0; i < n; ++i) {
    float p[3], q[4], v[3], w[3], a[3], al[3], tt[4], T = ci[i * 4], tau[3] = {ci[i * 4 + 1], ci[i * 4 + 2], ci[i * 4 + 3]};
    float mw[4] = {0, 0, 0, 0};
    for (int k = 0; k < 3; ++k) { p[k] = si[i * 13 + k]; v[k] = si[i * 13 + 7 + k]; w[k] = si[i * 13 + 10 + k]; }
    for (int k = 0; k < 4; ++k) q[k] = si[i * 13 + 3 + k];
    const float* pr = par + i * 16;
    float mot[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (mode == 0) {
      ctbr_compute(c, cmd + i * 4, w, ab + i * 3, pr + 0, pr + 4, pr[3], pr + 8, &T, tau, mw, nominal, tt);
      for (int k = 0; k < 4; ++k) mot[k] = tt[k];
    } else if (mode == 2) { /* ThrustController.update alone: cmd = desired rotor thrusts */
      for (int k = 0; k < 4; ++k) { mot[k] = cmd[i * 4 + k]; tt[k] = 0.0f; }
      motor_update(c, nominal, mot, mw);
    } else {
      for (int k = 0; k < 4; ++k) tt[k] = cmd[i * 4 + k];
    }
    dd_explicit(pr[7], pr + 12, drag + i * 6, drag + i * 6 + 3, tt, c->step_dt, c->gravity, p, q, v, w, a, al);
    for (int k = 0; k < 3; ++k) { so[i * 13 + k] = p[k]; so[i * 13 + 7 + k] = v[k]; so[i * 13 + 10 + k] = w[k]; }
    for (int k = 0; k < 4; ++k) so[i * 13 + 3 + k] = q[k];
    co[i * 4] = T;
    for (int k = 0; k < 3; ++k) co[i * 4 + 1 + k] = tau[k];
    float ww[3];
    quat_rotate(q, w, ww);
    for (int k = 0; k < 3; ++k) { xo[i * 13 + k] = a[k]; xo[i * 13 + 3 + k] = al[k]; xo[i * 13 + 6 + k] = ww[k]; }
    for (int k = 0; k < 4; ++k) xo[i * 13 + 9 + k] = mot[k];
  }
}

void gro_test_math(int fn, int n, const float* x, const float* y, float* out) {
  for (int i = 0; i < n; ++i) {
    float s, cc;
    switch (fn) {
      case 0: out[i] = gr_expf(x[i]); break;
      case 1: out[i] = gr_tanhf(x[i]); break;
      case 2: out[i] = gr_logf(x[i]); break;
      case 3: gr_sincosf(x[i], &s, &cc); out[i] = s; break;
      case 4: gr_sincosf(x[i], &s, &cc); out[i] = cc; break;
      case 5: out[i] = gr_atan2f(x[i], y[i]); break;
      case 6: out[i] = gr_sqrtf(x[i]); break;
      default: out[i] = x[i] / y[i]; break;
    }
  }
}

void gro_test_philox(int n, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                     uint32_t* out4) {
  for (int i = 0; i < n; ++i) {
    gr_u32x4 r = gr_philox4x32_10(c0 + (uint32_t)i, c1, c2, c3, k0, k1);
    out4[i * 4] = r.x; out4[i * 4 + 1] = r.y; out4[i * 4 + 2] = r.z; out4[i * 4 + 3] = r.w;
  }
}

/* The random values env i's step / reset / observation consume (tests/golden/make_golden_noise.py feeds them to the
 * reference's own functions in place of torch's draws, so the arithmetic that APPLIES them is pinned):
 *   kind 0: observation noise of call counter c1 (compute_obs): out[0..5] = the six N(0,1), velocity 0-2 then the
 *           attitude euler angles 3-5 (before x obs_att_noise)
 *   kind 1: gate-pose noise of (epoch c1, gates passed c3) (gate_noise): out[0..5] = the six U(0,1), gate x y z
 *           then next gate x y z
 *   kind 2: reset draws of epoch c1 (reset_env: the epoch AFTER the reset): out[0..23] = the 24 fields as U(0,1),
 *           out[24] = the thrust-error N(0,1)
 *   kind 3: startup draws (gro_init): out[0..13] = U(0,1) of Kp 0-2, Kd 3-5, thrust delay 6, torque delays 7-9,
 *           mass add 10, inertia 11-13; out[14] = the initial-level U(0,1); out[15] = the thrust-error N(0,1) */
void gro_draws(const gr_config* c, int i, int kind, uint32_t c1, uint32_t c3, float* out) {
  const uint32_t gid = gid_of(c, i);
  uint32_t f[24];
  if (kind == 0) {
    gr_fields6(draw(c, gid, c1, GR_TAG_OBS, 0), f);
    for (int k = 0; k < 6; ++k) out[k] = gr_normal21(f[k], GRO_NORMAL_TAB);
  } else if (kind == 1) {
    gr_fields6(draw(c, gid, c1, GR_TAG_GATE, c3), f);
    for (int k = 0; k < 6; ++k) out[k] = gr_f21(f[k]);
  } else if (kind == 2) {
    for (int b = 0; b < 4; ++b) gr_fields6(draw(c, gid, c1, GR_TAG_RESET, (uint32_t)b), f + 6 * b);
    for (int k = 0; k < 24; ++k) out[k] = gr_f21(f[k]);
    float z1;
    gr_box_muller21(f[20], f[21], &out[24], &z1);
  } else {
    gr_u32x4 b0 = draw(c, gid, 0, GR_TAG_STATIC, 0), b1 = draw(c, gid, 0, GR_TAG_STATIC, 1);
    gr_u32x4 b2 = draw(c, gid, 0, GR_TAG_STATIC, 2), b3 = draw(c, gid, 0, GR_TAG_STATIC, 3);
    gr_u32x4 b4 = draw(c, gid, 0, GR_TAG_STATIC, 4);
    const uint32_t w[15] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w, b2.x, b2.y, b2.z, b2.w, b3.x, b3.y, b3.z};
    for (int k = 0; k < 15; ++k) out[k] = gr_u01(w[k]);
    float z1;
    gr_box_muller(b3.w, b4.x, &out[15], &z1);
  }
}

/* gr_normal24 of n words (the camera noise's inverse-CDF table) */
void gro_test_normal24(int n, const uint32_t* w, float* z) {
  for (int i = 0; i < n; ++i) z[i] = gr_normal24(w[i], GRO_NORMAL_TAB);
}

/* the camera noise of env id gid, call counter cnt, pixel quads q0 .. q0 + nq - 1 (gr_cam_noise4): z[4 nq] */
void gro_test_cam_noise(uint32_t gid, uint32_t cnt, uint32_t q0, int nq, uint32_t k0, uint32_t k1, float* z) {
  for (int q = 0; q < nq; ++q) gr_cam_noise4(gid, cnt, q0 + (uint32_t)q, k0, k1, GRO_NORMAL_TAB, z + 4 * q);
}

void gro_test_fields6(int n, const uint32_t* in4, uint32_t* out6) {
  for (int i = 0; i < n; ++i) {
    gr_u32x4 r = {in4[i * 4], in4[i * 4 + 1], in4[i * 4 + 2], in4[i * 4 + 3]};
    gr_fields6(r, out6 + i * 6);
  }
}

/* ------------------------------------------------------------ depth camera */
/* The front camera + depth_image observation (racing_ctbr_env.py:77-95,141-160,390-391;
 * mdp/observation.py:65-94), pixel by pixel with the shared gr_camera.h functions: one
 * env at a time, rays in row-major order, gates in index order. */
void gro_camera(const gr_config* c, const gr_camera_config* kcfg, const gro_env* envs, int n, const gro_tracks* tr,
                int mode, const uint8_t* mask, const uint8_t* terminated, const uint8_t* time_out, uint32_t cnt,
                float* depth, int32_t* age, const float* obs_p16, const float* obs_c16, float* out_p, float* out_c) {
  gr_cam_const K;
  gr_cam_derive(kcfg, c->step_dt, &K);
  const int W = K.width, npix = K.npix;
  const size_t row = (size_t)(16 + npix);
#pragma omp parallel for schedule(static)
  for (int i = 0; i < n; ++i) {
    /* SensorBase: outdated after update_period (in whole env steps) or on reset */
    int outdated = age[i] < 0, aged = age[i] < 0 ? 0 : age[i];
    if (mode == GR_CAM_STEP) {
      aged += 1;
      outdated = outdated || terminated[i] || time_out[i] || aged >= K.period_steps;
    } else if (mode == GR_CAM_RESET) {
      outdated = outdated || mask == NULL || mask[i];
    }
    age[i] = outdated ? 0 : aged;
    float* dep = depth + (size_t)i * npix;
    if (outdated) {
      const gro_env* e = &envs[i];
      float o[3], c0[3], c1[3], c2[3];
      gr_cam_pose(&K, e->p, e->q, o, c0, c1, c2);
      const int track = track_index(c, e->type, e->level);
      const float gz = track_rec(tr, track)[0];
      const int ng = track_num_gates(tr, track);
      float slot[GR_CAM_MAX_GATES][GR_CAM_SLOT];
      for (int g = 0; g < ng; ++g) gr_cam_gate_setup(gate_rec(c, tr, track, g), o, c0, c1, c2, K.max_distance, slot[g]);
      const int no = track_num_obst(tr, track);
      float* oslot = (float*)malloc(sizeof(float) * GR_CAM_SLOT * (size_t)(no > 0 ? no : 1));
      for (int j = 0; j < no; ++j)
        gr_cam_obst_setup(obst_rec(tr, track, j), o, c0, c1, c2, K.max_distance, oslot + (size_t)j * GR_CAM_SLOT);
      for (int k = 0; k < npix; ++k) {
        const int v = k / W, u = k % W;
        const float a = K.ray_a[u], b = K.ray_b[v];
        const float dz = gr_fmaf(b, c2[2], gr_fmaf(a, c1[2], c0[2]));
        float d = gr_cam_ground_hit(o[2], gz, dz);
        for (int g = 0; g < ng; ++g) {
          const float* sl = slot[g];
          if (sl[GR_CS_VALID] == 0.0f) continue;
          if (b >= sl[GR_CS_BMIN] && b <= sl[GR_CS_BMAX] && a >= sl[GR_CS_AMIN] && a <= sl[GR_CS_AMAX])
            d = gr_minf(d, gr_cam_gate_hit(sl, a, b));
        }
        for (int j = 0; j < no; ++j) {
          const float* sl = oslot + (size_t)j * GR_CAM_SLOT;
          if (sl[GR_CS_VALID] == 0.0f) continue;
          if (b >= sl[GR_CS_BMIN] && b <= sl[GR_CS_BMAX] && a >= sl[GR_CS_AMIN] && a <= sl[GR_CS_AMAX])
            d = gr_minf(d, gr_cam_obst_hit(sl, a, b));
        }
        dep[k] = gr_cam_clip(d, K.max_distance);
      }
      free(oslot);
    }
    float* rp = out_p + (size_t)i * row;
    float* rc = out_c + (size_t)i * row;
    for (int k = 0; k < 16; ++k) {
      rp[k] = obs_p16[(size_t)i * 16 + k];
      rc[k] = obs_c16[(size_t)i * 16 + k];
    }
    const uint32_t gid = gid_of(c, i);
    for (int q = 0; q < npix / 4; ++q) {
      float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (K.add_noise) gr_cam_noise4(gid, cnt, (uint32_t)q, c->seed_lo, c->seed_hi, GRO_NORMAL_TAB, z);
      for (int j = 0; j < 4; ++j) {
        const float d = dep[4 * q + j];
        rp[16 + 4 * q + j] = gr_cam_obs(d, z[j], K.noise_std, K.obs_scale, K.inv_obs_scale);
        rc[16 + 4 * q + j] = gr_cam_obs_clean(d, K.obs_scale, K.inv_obs_scale);
      }
    }
  }
}

/* the shared pinhole / pose / gate-slot / hit functions, one ray at a time (known-answer tests) */
float gro_camera_ray(const gr_config* c, const gr_camera_config* kcfg, const gro_tracks* tr, int track,
                     const float p[3], const float q[4], int u, int v) {
  gr_cam_const K;
  gr_cam_derive(kcfg, c->step_dt, &K);
  float o[3], c0[3], c1[3], c2[3];
  gr_cam_pose(&K, p, q, o, c0, c1, c2);
  const float a = K.ray_a[u], b = K.ray_b[v];
  const float dz = gr_fmaf(b, c2[2], gr_fmaf(a, c1[2], c0[2]));
  float d = gr_cam_ground_hit(o[2], track_rec(tr, track)[0], dz);
  const int ng = track_num_gates(tr, track);
  for (int g = 0; g < ng; ++g) {
    float sl[GR_CAM_SLOT];
    gr_cam_gate_setup(gate_rec(c, tr, track, g), o, c0, c1, c2, K.max_distance, sl);
    if (sl[GR_CS_VALID] == 0.0f) continue;
    if (b >= sl[GR_CS_BMIN] && b <= sl[GR_CS_BMAX] && a >= sl[GR_CS_AMIN] && a <= sl[GR_CS_AMAX])
      d = gr_minf(d, gr_cam_gate_hit(sl, a, b));
  }
  const int no = track_num_obst(tr, track);
  for (int j = 0; j < no; ++j) {
    float sl[GR_CAM_SLOT];
    gr_cam_obst_setup(obst_rec(tr, track, j), o, c0, c1, c2, K.max_distance, sl);
    if (sl[GR_CS_VALID] == 0.0f) continue;
    if (b >= sl[GR_CS_BMIN] && b <= sl[GR_CS_BMAX] && a >= sl[GR_CS_AMIN] && a <= sl[GR_CS_AMAX])
      d = gr_minf(d, gr_cam_obst_hit(sl, a, b));
  }
  return gr_cam_clip(d, K.max_distance);
}

/* Check of the camera kernel's per-tile cull (gr_cam_gate_outside / gr_cam_obst_outside, kernel-only): for the
 * pose (p, q) on `track`, over every (8 x 32 tile, gate or obstacle in view) pair whose window meets the tile,
 * out[0] = pairs, out[1] = pairs the cull removes, out[2] = removed pairs with some pixel of the window that the
 * oracle's per-pixel test hits (must be 0), out[3] = window pixels of the removed pairs; gates in out[0..3],
 * obstacles in out[4..7]. */
void gro_camera_cull_check(const gr_config* c, const gr_camera_config* kcfg, const gro_tracks* tr, int track,
                           const float p[3], const float q[4], int64_t out[8]) {
  gr_cam_const K;
  gr_cam_derive(kcfg, c->step_dt, &K);
  float o[3], c0[3], c1[3], c2[3];
  gr_cam_pose(&K, p, q, o, c0, c1, c2);
  const int W = K.width, H = K.height;
  const int ng = track_num_gates(tr, track), no = track_num_obst(tr, track);
  for (int j = 0; j < 8; ++j) out[j] = 0;
  for (int j = 0; j < ng + no; ++j) {
    const int gate = j < ng;
    int64_t* ot = out + (gate ? 0 : 4);
    float sl[GR_CAM_SLOT];
    if (gate)
      gr_cam_gate_setup(gate_rec(c, tr, track, j), o, c0, c1, c2, K.max_distance, sl);
    else
      gr_cam_obst_setup(obst_rec(tr, track, j - ng), o, c0, c1, c2, K.max_distance, sl);
    if (sl[GR_CS_VALID] == 0.0f) continue;
    for (int v0 = 0; v0 < H; v0 += 8) {
      for (int u0 = 0; u0 < W; u0 += 32) {
        const int v1 = v0 + 7 < H ? v0 + 7 : H - 1, u1 = u0 + 31 < W ? u0 + 31 : W - 1;
        const float a_hi = K.ray_a[u0], a_lo = K.ray_a[u1], b_hi = K.ray_b[v0], b_lo = K.ray_b[v1];
        if (sl[GR_CS_AMAX] < a_lo || sl[GR_CS_AMIN] > a_hi || sl[GR_CS_BMAX] < b_lo || sl[GR_CS_BMIN] > b_hi) continue;
        ot[0] += 1;
        if (!(gate ? gr_cam_gate_outside(sl, a_lo, a_hi, b_lo, b_hi) : gr_cam_obst_outside(sl, a_lo, a_hi, b_lo, b_hi)))
          continue;
        ot[1] += 1;
        int hit = 0;
        for (int v = v0; v <= v1; ++v)
          for (int u = u0; u <= u1; ++u) {
            const float a = K.ray_a[u], b = K.ray_b[v];
            if (b >= sl[GR_CS_BMIN] && b <= sl[GR_CS_BMAX] && a >= sl[GR_CS_AMIN] && a <= sl[GR_CS_AMAX]) {
              ot[3] += 1;
              hit |= (gate ? gr_cam_gate_hit(sl, a, b) : gr_cam_obst_hit(sl, a, b)) < 3.0e38f;
            }
          }
        ot[2] += hit;
      }
    }
  }
}

/* camera pose + per-pixel ray constants, for the independent float64 mesh check */
void gro_camera_frame(const gr_config* c, const gr_camera_config* kcfg, const float p[3], const float q[4],
                      float* out /* o3 c0 c1 c2 (12), ray_a[W], ray_b[H] */) {
  gr_cam_const K;
  gr_cam_derive(kcfg, c->step_dt, &K);
  gr_cam_pose(&K, p, q, out, out + 3, out + 6, out + 9);
  for (int u = 0; u < K.width; ++u) out[12 + u] = K.ray_a[u];
  for (int v = 0; v < K.height; ++v) out[12 + K.width + v] = K.ray_b[v];
}
