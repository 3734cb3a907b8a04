"""Host side of rsl_rl/rollout_ops.py: EpisodeStats against the reference's deques (standalone/rsl_rl/ext/runners/
on_policy_runner.py:128-173: deque(maxlen=100).extend(cur_reward_sum[new_ids]) per step), and the ctypes layout
of gr_transition_args.  The device ops are pinned bit-exact in tests/test_gpu_rollout_ops.py."""
import ctypes as C
from collections import deque

import numpy as np
import torch

from generalizableracing_amd.rsl_rl.rollout_ops import EpisodeStats, GrTransitionArgs


def _reference_deques(rews, dones, maxlen=100):
    n = rews.shape[1]
    cur_r, cur_l = torch.zeros(n), torch.zeros(n)
    rb, lb = deque(maxlen=maxlen), deque(maxlen=maxlen)
    for r, d in zip(rews, dones):
        cur_r += r
        cur_l += 1
        new_ids = (d > 0).nonzero(as_tuple=False)
        rb.extend(cur_r[new_ids][:, 0].numpy().tolist())
        lb.extend(cur_l[new_ids][:, 0].numpy().tolist())
        cur_r[new_ids] = 0
        cur_l[new_ids] = 0
    return list(rb), list(lb), cur_r, cur_l


def test_episode_stats_match_reference_deques():
    g = torch.Generator().manual_seed(0)
    n, steps = 300, 70
    rews = torch.randn(steps, n, generator=g)
    dones = (torch.rand(steps, n, generator=g) < 0.05).long()
    dones[40] = 1  # one step with more finished episodes than the deque holds
    st = EpisodeStats(n, "cpu", steps=24)
    for r, d in zip(rews, dones):
        st.update(r, d)
    rb, lb, cur_r, cur_l = _reference_deques(rews, dones)
    mr, ml = st.means()
    assert st.buf_rew.numpy().tolist() == rb and st.buf_len.numpy().tolist() == lb
    assert torch.equal(st.cur_rew, cur_r) and torch.equal(st.cur_len, cur_l)
    assert abs(mr - float(np.mean(rb))) < 1e-5 and abs(ml - float(np.mean(lb))) < 1e-4


def test_episode_stats_empty():
    st = EpisodeStats(4, "cpu", steps=3)
    for _ in range(5):
        st.update(torch.ones(4), torch.zeros(4, dtype=torch.bool))
    assert st.means() is None
    assert torch.equal(st.cur_len, torch.full((4,), 5.0))


def test_transition_args_layout():
    # int64 n, int32 k, int32 dones_bytes, float gamma, int32 pad, 8 pointers, 5 int64 strides, 7 pointers
    assert C.sizeof(GrTransitionArgs) == 8 + 4 + 4 + 4 + 4 + 8 * 8 + 5 * 8 + 7 * 8
