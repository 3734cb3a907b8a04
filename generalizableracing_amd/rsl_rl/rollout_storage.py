"""RolloutStorage (standalone/rsl_rl/ext/storage/rollout_storage.py:12-191).

(T, N, .) device buffers, GAE, advantage normalisation and the shuffled
mini-batch generator.  Multi-GPU: advantages are normalised with the GLOBAL
mean / std over all ranks (two all-reduces), so a k-rank run normalises
exactly like one rank holding all k shards.
"""
from __future__ import annotations

import torch

from . import distributed as gdist


class RolloutStorage:
    class Transition:
        def __init__(self):
            self.observations = None
            self.privileged_observations = None
            self.actions = None
            self.privileged_actions = None
            self.rewards = None
            self.dones = None
            self.values = None
            self.actions_log_prob = None
            self.action_mean = None
            self.action_sigma = None
            self.hidden_states = None

        def clear(self):
            self.__init__()

    def __init__(self, training_type, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape,
                 actions_shape, device="cpu", obs_dtype=torch.float32):
        self.device = device
        self.training_type = training_type
        self.obs_shape = obs_shape
        self.privileged_obs_shape = privileged_obs_shape
        self.actions_shape = actions_shape
        T, N = num_transitions_per_env, num_envs
        self.observations = torch.zeros(T, N, *obs_shape, device=device, dtype=obs_dtype)
        if privileged_obs_shape[0] is not None:
            self.privileged_observations = torch.zeros(T, N, *privileged_obs_shape, device=device, dtype=obs_dtype)
        else:
            self.privileged_observations = None
        self.rewards = torch.zeros(T, N, 1, device=device)
        self.actions = torch.zeros(T, N, *actions_shape, device=device)
        self.dones = torch.zeros(T, N, 1, device=device).byte()
        if training_type == "distillation":
            self.privileged_actions = torch.zeros(T, N, *actions_shape, device=device)
        if training_type == "rl":
            self.actions_log_prob = torch.zeros(T, N, 1, device=device)
            self.values = torch.zeros(T, N, 1, device=device)
            self.returns = torch.zeros(T, N, 1, device=device)
            self.advantages = torch.zeros(T, N, 1, device=device)
            self.mu = torch.zeros(T, N, *actions_shape, device=device)
            self.sigma = torch.zeros(T, N, *actions_shape, device=device)
        self.num_transitions_per_env = T
        self.num_envs = N
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0
        # observation sink (enable_obs_sink): the env's kernel writes the observations of transition t into
        # slot t itself; slot T holds the rollout's last observations (transition 0 of the next rollout)
        self.sink = False
        self.prefilled = [False] * (T + 1)

    def enable_obs_sink(self):
        """Observation buffers with one more slot, written by the env (RacingEnv.set_obs_sink) instead of copied
        by add_transitions.  The mini-batch generators and the GAE read the first T slots only."""
        if self.sink:
            return
        T = self.num_transitions_per_env
        self.observations = torch.cat([self.observations, torch.zeros_like(self.observations[:1])])
        if self.privileged_observations is not None:
            self.privileged_observations = torch.cat([self.privileged_observations,
                                                      torch.zeros_like(self.privileged_observations[:1])])
        self.sink = True
        self.prefilled = [False] * (T + 1)

    def sink_slot(self, t: int):
        """(policy, critic) observation rows of slot t, marked as filled by the env."""
        self.prefilled[t] = True
        priv = self.privileged_observations if self.privileged_observations is not None else self.observations
        return self.observations[t], priv[t]

    def sink_skipped(self):
        """A transition was not stored (PPOL2C2's zero-observation skip): the rows the env wrote for its successor
        (slot step + 1) belong to the transition stored next, at slot step."""
        t = self.step
        if self.prefilled[t + 1]:
            self.observations[t].copy_(self.observations[t + 1])
            if self.privileged_observations is not None:
                self.privileged_observations[t].copy_(self.privileged_observations[t + 1])
            self.prefilled[t], self.prefilled[t + 1] = True, False
        else:
            self.prefilled[t] = False

    def discard_sink(self):
        """Slots marked filled by the env are stale (the runner observed afresh): copy on the next adds."""
        self.prefilled = [False] * (self.num_transitions_per_env + 1)

    def add_transitions(self, transition: "RolloutStorage.Transition"):
        if self.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        if self.prefilled[self.step]:  # written by the env's kernel (observation sink)
            self.prefilled[self.step] = False
        else:
            self.observations[self.step].copy_(transition.observations)
            if self.privileged_observations is not None:
                self.privileged_observations[self.step].copy_(transition.privileged_observations)
        self.actions[self.step].copy_(transition.actions)
        self.rewards[self.step].copy_(transition.rewards.view(-1, 1))
        self.dones[self.step].copy_(transition.dones.view(-1, 1))
        if self.training_type == "distillation":
            self.privileged_actions[self.step].copy_(transition.privileged_actions)
        if self.training_type == "rl":
            self.values[self.step].copy_(transition.values)
            self.actions_log_prob[self.step].copy_(transition.actions_log_prob.view(-1, 1))
            self.mu[self.step].copy_(transition.action_mean)
            self.sigma[self.step].copy_(transition.action_sigma)
        self.step += 1

    def clear(self):
        self.step = 0
        T = self.num_transitions_per_env
        if self.sink and self.prefilled[T]:  # the rollout's last observations open the next rollout
            self.observations[0].copy_(self.observations[T])
            if self.privileged_observations is not None:
                self.privileged_observations[0].copy_(self.privileged_observations[T])
            self.prefilled = [False] * (T + 1)
            self.prefilled[0] = True

    def compute_returns(self, last_values, gamma, lam, normalize_advantage: bool = True):
        """GAE, rollout_storage.py:113-127 (CUDA fp32: one launch, rollout_ops.gae, the same bits)."""
        from . import rollout_ops

        if rollout_ops.gae_ok(self, last_values):
            rollout_ops.gae(self, last_values, gamma, lam)
            if normalize_advantage:
                mean, std = gdist.global_mean_std(self.advantages)
                self.advantages.sub_(mean).div_(std + 1e-8)
            return
        advantage = 0
        for step in reversed(range(self.num_transitions_per_env)):
            next_values = last_values if step == self.num_transitions_per_env - 1 else self.values[step + 1]
            next_is_not_terminal = 1.0 - self.dones[step].float()
            delta = self.rewards[step] + next_is_not_terminal * gamma * next_values - self.values[step]
            advantage = delta + next_is_not_terminal * gamma * lam * advantage
            self.returns[step] = advantage + self.values[step]
        # in place: the graph-captured update (ppo.py _GraphedStep) gathers from this allocation, so
        # rebinding the attribute would leave its replays reading the first iteration's freed buffer
        torch.sub(self.returns, self.values, out=self.advantages)
        if normalize_advantage:
            mean, std = gdist.global_mean_std(self.advantages)
            self.advantages.sub_(mean).div_(std + 1e-8)

    def get_statistics(self):
        done = self.dones.clone()
        done[-1] = 1
        flat_dones = done.permute(1, 0, 2).reshape(-1, 1)
        done_indices = torch.cat((flat_dones.new_tensor([-1], dtype=torch.int64),
                                  flat_dones.nonzero(as_tuple=False)[:, 0]))
        trajectory_lengths = done_indices[1:] - done_indices[:-1]
        return trajectory_lengths.float().mean(), self.rewards.mean()

    PACK_MAX_COLS = 128  # sample rows up to this many floats are gathered as one packed row

    def sample_sources(self):
        """The per-sample fields the PPO mini-batches read, each [T * N, width]: observations, critic observations,
        actions, values, advantages, returns, old log prob, old mean, old std."""
        T = self.num_transitions_per_env
        obs = self.observations[:T].flatten(0, 1)
        priv = self.privileged_observations[:T].flatten(0, 1) if self.privileged_observations is not None else obs
        return (obs, priv, self.actions.flatten(0, 1), self.values.flatten(0, 1), self.advantages.flatten(0, 1),
                self.returns.flatten(0, 1), self.actions_log_prob.flatten(0, 1), self.mu.flatten(0, 1),
                self.sigma.flatten(0, 1))

    def sample_columns(self):
        """Column ranges of the fields in a packed sample row (pack_samples), or None when the rows are too wide
        to pack (the camera task's image rows: the fields are then gathered one by one)."""
        widths = [x.shape[1] for x in self.sample_sources()]
        if sum(widths) > self.PACK_MAX_COLS:
            return None
        cols, c = [], 0
        for w in widths:
            cols.append((c, c + w))
            c += w
        return cols

    def pack_samples(self, out=None):
        """[T * N, sum of widths] fp32: every field of a sample in one row, so a mini-batch is ONE row gather
        (the fields one by one were nine gathers of 4-64-byte rows per mini-batch, each latency-bound:
        profiles/round03_update65536_graphed_kernel_stats.csv).  Pure data movement: the mini-batches are
        the same values."""
        src = [x.detach().float() for x in self.sample_sources()]
        with torch.no_grad():
            if out is None:
                return torch.cat(src, dim=1)
            return torch.cat(src, dim=1, out=out)

    def packed_buffer(self):
        """The persistent [T * N, packed width] fp32 buffer pack_samples fills (allocated on first use)."""
        cols = self.sample_columns()
        shape = (self.num_transitions_per_env * self.num_envs, cols[-1][1])
        buf = getattr(self, "_packed", None)
        if buf is None or tuple(buf.shape) != shape:
            buf = self._packed = torch.empty(shape, dtype=torch.float32, device=self.device)
        return buf

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        """rollout_storage.py:152-191: one randperm, `num_epochs` passes of `num_mini_batches` chunks."""
        if self.training_type != "rl":
            raise ValueError("This function is only available for reinforcement learning training.")
        batch_size = self.num_envs * self.num_transitions_per_env
        mini_batch_size = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mini_batch_size, requires_grad=False, device=self.device)
        cols = self.sample_columns()
        if cols is not None and self.observations.dtype == torch.float32:
            # one persistent packed buffer (fp32 storage only: packing bf16 observations would upcast the whole
            # rollout and undo what the bf16 storage saves; those are gathered field by field below)
            pack = self.pack_samples(out=self.packed_buffer())
            for _ in range(num_epochs):
                for i in range(num_mini_batches):
                    g = pack.index_select(0, indices[i * mini_batch_size:(i + 1) * mini_batch_size])
                    yield tuple(g[:, a:b] for a, b in cols) + ((None, None), None)
            return
        observations = self.observations.flatten(0, 1)
        privileged = self.privileged_observations.flatten(0, 1) if self.privileged_observations is not None else observations
        actions = self.actions.flatten(0, 1)
        values = self.values.flatten(0, 1)
        returns = self.returns.flatten(0, 1)
        old_logp = self.actions_log_prob.flatten(0, 1)
        advantages = self.advantages.flatten(0, 1)
        old_mu = self.mu.flatten(0, 1)
        old_sigma = self.sigma.flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mini_batch_size:(i + 1) * mini_batch_size]
                yield (observations[idx].float(), privileged[idx].float(), actions[idx], values[idx], advantages[idx],
                       returns[idx], old_logp[idx], old_mu[idx], old_sigma[idx], (None, None), None)
