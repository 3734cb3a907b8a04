// gr_rollout.hip — the rollout loop's per-step bookkeeping as one launch each (rsl_rl/rollout_ops.py).
//
// At 4 096 envs a training iteration's rollout is host-bound: per env step the runner launched ~40 small torch
// ops besides the env step and the policy (the time-out bootstrap and the transition copies of
// PPO.process_env_step, the episode-statistics updates of the runner) and the GAE of compute_returns another ~200
// per rollout, each a few microseconds of host time for microseconds of GPU work.  Each group is one launch here,
// with the torch ops' arithmetic in their order (fp32, no contraction: the Makefile's -ffp-contract=off), so the
// stored rollout is bit-identical.
#include "gr_kernels.h"

namespace gr {

__device__ __forceinline__ bool flag_at(const void* p, int bytes, long long i) {
  if (bytes == 8) return static_cast<const long long*>(p)[i] != 0;
  if (bytes == 4) return static_cast<const int*>(p)[i] != 0;
  return static_cast<const uint8_t*>(p)[i] != 0;
}

// PPO.process_env_step + RolloutStorage.add_transitions (ppo.py:83-95, rollout_storage.py:74-98): the reward with
// the time-out bootstrap r + gamma * (v * time_out) (torch: rewards += gamma * squeeze(values * time_outs)), the
// done flag as a byte, and the action / value / log prob / mean / std rows into the storage's slot
__global__ __launch_bounds__(256) void store_transition(gr_transition_args a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  float r = a.reward[i];
  const float v = a.value[i * a.ld_value];
  if (a.time_out) {
    const float to = a.time_out[i] ? 1.0f : 0.0f;
    r = r + a.gamma * (v * to);
  }
  a.out_reward[i] = r;
  a.out_dones[i] = flag_at(a.dones, a.dones_bytes, i) ? 1 : 0;
  a.out_value[i] = v;
  a.out_logp[i] = a.logp[i * a.ld_logp];
  for (int j = 0; j < a.k; ++j) {
    a.out_action[i * a.k + j] = a.action[i * a.ld_action + j];
    a.out_mu[i * a.k + j] = a.mu[i * a.ld_mu + j];
    a.out_sigma[i * a.k + j] = a.sigma[i * a.ld_sigma + j];
  }
}

// the runner's episode sums (on_policy_runner.py:167-173): cur += reward, len += 1; the finished episodes' sums set
// aside for the deques (fin_*, fin_done), the sums of done envs zeroed
__global__ __launch_bounds__(256) void episode_accumulate(long long n, const float* __restrict__ reward,
                                                          const void* __restrict__ dones, int dones_bytes,
                                                          float* __restrict__ cur_rew, float* __restrict__ cur_len,
                                                          float* __restrict__ fin_rew, float* __restrict__ fin_len,
                                                          uint8_t* __restrict__ fin_done) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float c = cur_rew[i] + reward[i];
  const float l = cur_len[i] + 1.0f;
  const bool d = flag_at(dones, dones_bytes, i);
  fin_rew[i] = c;
  fin_len[i] = l;
  fin_done[i] = d ? 1 : 0;
  cur_rew[i] = d ? 0.0f : c;
  cur_len[i] = d ? 0.0f : l;
}

// RolloutStorage.compute_returns (rollout_storage.py:113-127) per env, backwards over the T steps:
//   delta = r_t + (nnt * gamma) * v_next - v_t;  adv = delta + ((nnt * gamma) * lam) * adv;  ret_t = adv + v_t
// with nnt = 1 - done_t; then advantages = returns - values (the normalisation stays in torch: global statistics)
__global__ __launch_bounds__(256) void gae(long long n, int t_steps, float gamma, float lam,
                                           const float* __restrict__ rewards, const uint8_t* __restrict__ dones,
                                           const float* __restrict__ values, const float* __restrict__ last_values,
                                           long long ld_last, float* __restrict__ returns,
                                           float* __restrict__ advantages) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float adv = 0.0f;
  float next = last_values[i * ld_last];
  for (int t = t_steps - 1; t >= 0; --t) {
    const long long o = (long long)t * n + i;
    const float nnt = 1.0f - (dones[o] ? 1.0f : 0.0f);
    const float v = values[o];
    const float ng = nnt * gamma;
    const float delta = (rewards[o] + ng * next) - v;
    adv = t == t_steps - 1 ? delta + (ng * lam) * 0.0f : delta + (ng * lam) * adv;
    const float ret = adv + v;
    returns[o] = ret;
    advantages[o] = ret - v;
    next = v;
  }
}

hipError_t launch_store_transition(const gr_transition_args& a, hipStream_t s) {
  hipLaunchKernelGGL(store_transition, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_episode_accumulate(long long n, const float* reward, const void* dones, int dones_bytes,
                                     float* cur_rew, float* cur_len, float* fin_rew, float* fin_len,
                                     uint8_t* fin_done, hipStream_t s) {
  hipLaunchKernelGGL(episode_accumulate, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, reward, dones,
                     dones_bytes, cur_rew, cur_len, fin_rew, fin_len, fin_done);
  return hipGetLastError();
}

hipError_t launch_gae(long long n, int t_steps, float gamma, float lam, const float* rewards, const uint8_t* dones,
                      const float* values, const float* last_values, long long ld_last, float* returns,
                      float* advantages, hipStream_t s) {
  hipLaunchKernelGGL(gae, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, n, t_steps, gamma, lam, rewards, dones,
                     values, last_values, ld_last, returns, advantages);
  return hipGetLastError();
}

// PPOL2C2's mixed observations (ppo_l2c2.py:179-180): out = o + w * (n - o) with w one scalar per row, in the torch
// expression's three roundings (sub, mul, add; no contraction): one pass (read o, n, write out) instead of three
// elementwise kernels over [rows, cols] matrices of ~680 MB at 4 096 envs.  With row indices the pair is read
// straight from the rollout storage (row ra[r] of o, rb[r] of n, ld floats apart) instead of from gathered copies.
__global__ __launch_bounds__(256) void l2c2_mix(const float* __restrict__ o, const float* __restrict__ nx, long long ld4,
                                                 const long long* __restrict__ ra, const long long* __restrict__ rb,
                                                 const float* __restrict__ w, long long rows, int cols4,
                                                 float* __restrict__ out) {
  const long long n4 = rows * cols4;
  for (long long q = (long long)blockIdx.x * 256 + threadIdx.x; q < n4; q += (long long)gridDim.x * 256) {
    const long long r = q / cols4, c = q - r * cols4;
    const float wr = w[r];
    const long long ia = (ra ? ra[r] : r) * ld4 + c, ib = (rb ? rb[r] : r) * ld4 + c;
    const float4 a = reinterpret_cast<const float4*>(o)[ia], b = reinterpret_cast<const float4*>(nx)[ib];
    float4 v;
    v.x = a.x + wr * (b.x - a.x);
    v.y = a.y + wr * (b.y - a.y);
    v.z = a.z + wr * (b.z - a.z);
    v.w = a.w + wr * (b.w - a.w);
    reinterpret_cast<float4*>(out)[q] = v;
  }
}

hipError_t launch_l2c2_mix(const float* o, const float* nx, long long ld, const long long* ra, const long long* rb,
                           const float* w, long long rows, int cols, float* out, hipStream_t s) {
  const long long n4 = rows * (cols / 4);
  long long blocks = (n4 + 256 * 8 - 1) / (256 * 8);
  blocks = blocks < 1 ? 1 : (blocks > 8192 ? 8192 : blocks);
  hipLaunchKernelGGL(l2c2_mix, dim3((unsigned)blocks), dim3(256), 0, s, o, nx, ld / 4, ra, rb, w, rows, cols / 4, out);
  return hipGetLastError();
}

}  // namespace gr
