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

namespace gr {

#define CAM_WAVES 4
#define CAM_SLOT4 (GR_CAM_SLOT / 4)

__global__ __launch_bounds__(CAM_WAVES * 64) void camera_kernel(CamArgs a) {
  __shared__ __attribute__((aligned(16))) float s_ray_a[GR_CAM_MAX_W];
  __shared__ float s_ray_b[GR_CAM_MAX_H];
  __shared__ float4 s_slot[CAM_WAVES][GR_CAM_MAX_GATES][CAM_SLOT4];

  const gr_cam_const* __restrict__ cc = a.cc;
  const int W = cc->width, npix = cc->npix;
  for (int k = threadIdx.x; k < W; k += CAM_WAVES * 64) s_ray_a[k] = cc->ray_a[k];
  for (int k = threadIdx.x; k < cc->height; k += CAM_WAVES * 64) s_ray_b[k] = cc->ray_b[k];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = blockIdx.x * CAM_WAVES + w;
  const bool active = i < a.num_envs;
  const int N = a.num_envs;

  // ---- is the sensor outdated? (SensorBase.update / reset; wave-uniform)
  int render = 0, age_new = 0;
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
    age_new = render ? 0 : aged;
    if (lane == 0) a.age[i] = age_new;
  }

  // ---- camera pose and the gate slots of this env's track
  float o[3] = {0.0f, 0.0f, 0.0f}, c0[3] = {1.0f, 0.0f, 0.0f}, c1[3] = {0.0f, 1.0f, 0.0f},
        c2[3] = {0.0f, 0.0f, 1.0f};
  float gz = 0.0f;
  uint64_t valid_mask = 0;
  if (render) {
    const float4 posq = reinterpret_cast<const float4*>(a.state)[(size_t)GR_P_POSQ * N + i];
    const float4 qv = reinterpret_cast<const float4*>(a.state)[(size_t)GR_P_QV * N + i];
    const float p[3] = {posq.x, posq.y, posq.z}, q[4] = {posq.w, qv.x, qv.y, qv.z};
    gr_cam_pose(cc, p, q, o, c0, c1, c2);
    const int packed = a.istate[4 * i + GR_I_PACKED];
    const int track = ((packed >> 24) & 0xff) * a.num_levels + ((packed >> 8) & 0xff);
    const float* tb = a.table + (size_t)track * a.track_stride;
    const float* rec = tb + a.max_gates * GR_GATE_FLOATS;
    gz = rec[0];
    const int ng = (int)rec[3];
    float s[GR_CAM_SLOT];
    int valid = 0;
    if (lane < ng) {
      gr_cam_gate_setup(tb + lane * GR_GATE_FLOATS, o, c0, c1, c2, cc->max_distance, s);
      valid = s[GR_CS_VALID] != 0.0f;
#pragma unroll
      for (int k = 0; k < CAM_SLOT4; ++k)
        s_slot[w][lane][k] = make_float4(s[4 * k], s[4 * k + 1], s[4 * k + 2], s[4 * k + 3]);
    }
    valid_mask = __ballot(valid);
  }
  __syncthreads();

  // ---- pixels
  const uint32_t gid = (uint32_t)(a.env_id_offset + i);
  const uint32_t cnt = a.counters[a.counter_index];
  const size_t row = (size_t)(16 + npix);
  if (active) {
    if (lane < 4) {
      const float4 sp = reinterpret_cast<const float4*>(a.obs_p16)[4 * i + lane];
      const float4 sc = reinterpret_cast<const float4*>(a.obs_c16)[4 * i + lane];
      reinterpret_cast<float4*>(a.out_p + i * row)[lane] = sp;
      reinterpret_cast<float4*>(a.out_c + i * row)[lane] = sc;
    }
    const float maxd = cc->max_distance, scale = cc->obs_scale, inv_scale = cc->inv_obs_scale;
    const float nstd = cc->noise_std;
    const int noise = cc->add_noise, H = cc->height;
    // 8-row x 32-column tiles: a lane owns one pixel quad (row lane/8, columns 4*(lane%8)..+3), so a
    // gate's screen window culls whole tiles and each store writes 8 full 128-byte row segments
    const int tiles_x = (W + 31) >> 5, ntiles = tiles_x * ((H + 7) >> 3);
    for (int t = 0; t < ntiles; ++t) {
      const int ty = t / tiles_x, tx = t - ty * tiles_x;
      const int v = ty * 8 + (lane >> 3), u0 = tx * 32 + 4 * (lane & 7);
      if (v >= H || u0 >= W) continue;
      const int k0 = v * W + u0;
      float d[4];
      if (render) {
        const float b = s_ray_b[v];
        const float4 a4 = *reinterpret_cast<const float4*>(&s_ray_a[u0]);
        const float av[4] = {a4.x, a4.y, a4.z, a4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float dz = gr_fmaf(b, c2[2], gr_fmaf(av[j], c1[2], c0[2]));
          d[j] = gr_cam_ground_hit(o[2], gz, dz);
        }
        uint64_t m = valid_mask;
        while (m) {
          const int g = __builtin_ctzll(m);
          m &= m - 1;
          float s[GR_CAM_SLOT];
#pragma unroll
          for (int k = 0; k < CAM_SLOT4; ++k) {
            const float4 q4 = s_slot[w][g][k];
            s[4 * k] = q4.x; s[4 * k + 1] = q4.y; s[4 * k + 2] = q4.z; s[4 * k + 3] = q4.w;
          }
          if (b >= s[GR_CS_BMIN] && b <= s[GR_CS_BMAX] && av[3] <= s[GR_CS_AMAX] && av[0] >= s[GR_CS_AMIN]) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (av[j] >= s[GR_CS_AMIN] && av[j] <= s[GR_CS_AMAX]) d[j] = gr_minf(d[j], gr_cam_gate_hit(s, av[j], b));
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = gr_cam_clip(d[j], maxd);
        reinterpret_cast<float4*>(a.depth + (size_t)i * npix)[k0 >> 2] = make_float4(d[0], d[1], d[2], d[3]);
      } else {
        const float4 q4 = reinterpret_cast<const float4*>(a.depth + (size_t)i * npix)[k0 >> 2];
        d[0] = q4.x; d[1] = q4.y; d[2] = q4.z; d[3] = q4.w;
      }
      float z[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (noise) gr_cam_noise4(gid, cnt, (uint32_t)(k0 >> 2), a.seed_lo, a.seed_hi, z);
      float4 op, oc;
      op.x = gr_cam_obs(d[0], z[0], nstd, scale, inv_scale); oc.x = gr_cam_obs_clean(d[0], scale, inv_scale);
      op.y = gr_cam_obs(d[1], z[1], nstd, scale, inv_scale); oc.y = gr_cam_obs_clean(d[1], scale, inv_scale);
      op.z = gr_cam_obs(d[2], z[2], nstd, scale, inv_scale); oc.z = gr_cam_obs_clean(d[2], scale, inv_scale);
      op.w = gr_cam_obs(d[3], z[3], nstd, scale, inv_scale); oc.w = gr_cam_obs_clean(d[3], scale, inv_scale);
      reinterpret_cast<float4*>(a.out_p + i * row + 16)[k0 >> 2] = op;
      reinterpret_cast<float4*>(a.out_c + i * row + 16)[k0 >> 2] = oc;
    }
  }
}

hipError_t launch_camera(const CamArgs& a, hipStream_t s) {
  const int blocks = (a.num_envs + CAM_WAVES - 1) / CAM_WAVES;
  hipLaunchKernelGGL(camera_kernel, dim3(blocks), dim3(CAM_WAVES * 64), 0, s, a);
  return hipGetLastError();
}

}  // namespace gr
