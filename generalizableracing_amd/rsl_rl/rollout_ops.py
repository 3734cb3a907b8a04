"""The rollout loop's per-step bookkeeping as one HIP launch each (gr_store_transition, gr_episode_accumulate,
gr_gae in csrc/gr_rollout.hip).

At config C2's 4 096 envs a training iteration's rollout is host-bound: besides the env step (one launch) and the
policy, every env step cost ~40 small torch ops — PPO.process_env_step's time-out bootstrap and the transition
copies of RolloutStorage.add_transitions (standalone/rsl_rl/ext/algorithms/ppo.py:83-95, rsl_rl
rollout_storage.py:74-98), the runner's episode-statistics updates (standalone/rsl_rl/ext/runners/
on_policy_runner.py:167-173) — and compute_returns' GAE (rollout_storage.py:113-127) ~200 more per rollout, each a
few microseconds of host time for microseconds of GPU work (scripts/prof_rollout.py).  Here each group is one
launch with the torch ops' arithmetic in their order, so the stored rollout is bit-identical
(tests/test_gpu_rollout_ops.py); CPU tensors, other dtypes and other storages keep the torch ops.
"""
from __future__ import annotations

import ctypes as C

import torch


class GrTransitionArgs(C.Structure):
    """Mirror of gr_transition_args (include/gr.h)."""
    _fields_ = [("n", C.c_int64), ("k", C.c_int32), ("dones_bytes", C.c_int32), ("gamma", C.c_float),
                ("pad", C.c_int32)] + [
        (f, C.c_void_p) for f in ("reward", "dones", "time_out", "value", "action", "logp", "mu", "sigma")] + [
        (f, C.c_int64) for f in ("ld_value", "ld_action", "ld_logp", "ld_mu", "ld_sigma")] + [
        (f, C.c_void_p) for f in ("out_reward", "out_dones", "out_action", "out_value", "out_logp", "out_mu",
                                  "out_sigma")]


_FLAG_BYTES = {torch.bool: 1, torch.uint8: 1, torch.int32: 4, torch.int64: 8}


def _call(name, *args):
    from .. import _abi

    rc = getattr(_abi.load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (status {rc})")


def _stream(t):
    from .. import _abi

    return _abi.raw_stream(t.device)


def _flags_ok(t, n) -> bool:
    return t is not None and t.is_cuda and t.dtype in _FLAG_BYTES and t.numel() == n and t.is_contiguous()


def _rows_ok(t, n, k) -> bool:
    """fp32 CUDA rows [n, k] (or [n] for k = 1) with unit column stride (the row stride may be 0: a broadcast)."""
    if t is None or not t.is_cuda or t.dtype != torch.float32:
        return False
    if t.dim() == 1:
        return k == 1 and t.shape[0] == n and (t.stride(0) == 1 or n == 1)
    return t.dim() == 2 and tuple(t.shape) == (n, k) and (t.stride(1) == 1 or k == 1)


def _ld(t) -> int:
    return int(t.stride(0))


def store_ok(storage, tr, rewards, dones, time_outs) -> bool:
    """gr_store_transition applies: the plain RolloutStorage (rl) on CUDA and fp32 transition rows."""
    from .rollout_storage import RolloutStorage

    if type(storage) is not RolloutStorage or storage.training_type != "rl" or not storage.rewards.is_cuda:
        return False
    n, k = storage.num_envs, storage.actions.shape[-1]
    if k > 8 or storage.actions.dim() != 3:
        return False
    if not (rewards.is_cuda and rewards.dtype == torch.float32 and rewards.numel() == n and rewards.is_contiguous()):
        return False
    if not _flags_ok(dones, n) or (time_outs is not None and not (_flags_ok(time_outs, n)
                                                                  and time_outs.dtype in (torch.bool, torch.uint8))):
        return False
    return (_rows_ok(tr.actions, n, k) and _rows_ok(tr.values, n, 1) and _rows_ok(tr.actions_log_prob, n, 1)
            and _rows_ok(tr.action_mean, n, k) and _rows_ok(tr.action_sigma, n, k))


def store_transition(storage, tr, rewards, dones, time_outs, gamma):
    """PPO.process_env_step's bootstrap + RolloutStorage.add_transitions in one launch (the observations: the
    env's sink rows, or two copies)."""
    st = storage
    if st.step >= st.num_transitions_per_env:
        raise AssertionError("Rollout buffer overflow")
    t = st.step
    if st.prefilled[t]:  # written by the env's kernel (observation sink)
        st.prefilled[t] = False
    else:
        st.observations[t].copy_(tr.observations)
        if st.privileged_observations is not None:
            st.privileged_observations[t].copy_(tr.privileged_observations)
    n, k = st.num_envs, st.actions.shape[-1]
    a = GrTransitionArgs()
    a.n, a.k, a.dones_bytes, a.gamma = n, k, _FLAG_BYTES[dones.dtype], float(gamma)
    a.reward, a.dones = rewards.data_ptr(), dones.data_ptr()
    a.time_out = time_outs.data_ptr() if time_outs is not None else None
    for name, src in (("value", tr.values), ("action", tr.actions), ("logp", tr.actions_log_prob),
                      ("mu", tr.action_mean), ("sigma", tr.action_sigma)):
        setattr(a, name, src.data_ptr())
        setattr(a, "ld_" + name, _ld(src))
    for name, dst in (("out_reward", st.rewards), ("out_dones", st.dones), ("out_action", st.actions),
                      ("out_value", st.values), ("out_logp", st.actions_log_prob), ("out_mu", st.mu),
                      ("out_sigma", st.sigma)):
        setattr(a, name, dst[t].data_ptr())
    _call("gr_store_transition", C.addressof(a), _stream(rewards))
    st.step += 1


def gae_ok(storage, last_values) -> bool:
    st = storage
    n = st.num_envs
    return (st.rewards.is_cuda and st.rewards.dtype == torch.float32 and st.values.dtype == torch.float32
            and st.dones.dtype == torch.uint8 and all(x.is_contiguous() for x in (st.rewards, st.values, st.dones,
                                                                                    st.returns, st.advantages))
            and _rows_ok(last_values, n, 1))


def gae(storage, last_values, gamma, lam):
    """compute_returns' backward loop + advantages = returns - values, one launch."""
    st = storage
    _call("gr_gae", st.num_envs, st.num_transitions_per_env, C.c_float(gamma), C.c_float(lam),
          st.rewards.data_ptr(), st.dones.data_ptr(), st.values.data_ptr(), last_values.data_ptr(),
          _ld(last_values), st.returns.data_ptr(), st.advantages.data_ptr(), _stream(st.rewards))


class EpisodeStats:
    """The runner's rewbuffer / lenbuffer deques (maxlen 100) and episode sums (on_policy_runner.py:128-173) on the
    device.  Per env step one launch on CUDA (gr_episode_accumulate; the same ops in torch elsewhere): the sums,
    and the sums of the episodes that finished set aside per step.  The deques are brought up to date from those
    in (step, env) order — the order of the reference's deque.extend calls — when read (means) or when the
    step buffer is full: one host synchronisation per rollout instead of the reference's one per step."""

    def __init__(self, num_envs, device, maxlen=100, steps=32):
        self.n, self.maxlen, self.steps = num_envs, maxlen, steps
        self.device = torch.device(device)
        self.cur_rew = torch.zeros(num_envs, device=device)
        self.cur_len = torch.zeros(num_envs, device=device)
        self.fin_rew = torch.zeros(steps, num_envs, device=device)
        self.fin_len = torch.zeros(steps, num_envs, device=device)
        self.fin_done = torch.zeros(steps, num_envs, dtype=torch.uint8, device=device)
        self.t = 0
        self.buf_rew = torch.zeros(0, device=device)
        self.buf_len = torch.zeros(0, device=device)

    def update(self, rewards, dones):
        if self.t == self.steps:
            self.flush()
        t = self.t
        r = rewards.reshape(-1)
        if (self.cur_rew.is_cuda and r.dtype == torch.float32 and r.is_contiguous() and r.numel() == self.n
                and _flags_ok(dones, self.n)):
            _call("gr_episode_accumulate", self.n, r.data_ptr(), dones.data_ptr(), _FLAG_BYTES[dones.dtype],
                  self.cur_rew.data_ptr(), self.cur_len.data_ptr(), self.fin_rew[t].data_ptr(),
                  self.fin_len[t].data_ptr(), self.fin_done[t].data_ptr(), _stream(self.cur_rew))
        else:
            d = dones.reshape(-1) > 0
            self.cur_rew += r
            self.cur_len += 1
            self.fin_rew[t].copy_(self.cur_rew)
            self.fin_len[t].copy_(self.cur_len)
            self.fin_done[t].copy_(d)
            self.cur_rew.masked_fill_(d, 0.0)
            self.cur_len.masked_fill_(d, 0.0)
        self.t += 1

    def flush(self):
        if self.t == 0:
            return
        t = self.t
        idx = self.fin_done[:t].reshape(-1).nonzero()[:, 0]  # (step, env) order: the deque.extend order
        if idx.numel():
            self.buf_rew = torch.cat([self.buf_rew, self.fin_rew[:t].reshape(-1)[idx]])[-self.maxlen:]
            self.buf_len = torch.cat([self.buf_len, self.fin_len[:t].reshape(-1)[idx]])[-self.maxlen:]
        self.t = 0

    def means(self):
        self.flush()
        if self.buf_rew.numel() == 0:
            return None
        return float(self.buf_rew.mean()), float(self.buf_len.mean())
