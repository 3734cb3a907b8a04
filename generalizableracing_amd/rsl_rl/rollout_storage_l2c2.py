"""RolloutStorageL2C2 (standalone/rsl_rl/ext/storage/rollout_storage_l2c2.py:6-167).

The PPO rollout buffer plus what the L2C2 smoothness loss needs: each sample
of the first T-1 steps is paired with the observation of the NEXT step of the
same env and a continuation flag (1 - done).  The last step of the rollout has
no successor inside the buffer, so the batch is (T-1)*N samples
(rollout_storage_l2c2.py:131-132).  Advantages are always normalised
(:117-118), with the global mean / std over all ranks as in RolloutStorage.
"""
from __future__ import annotations

import torch

from .rollout_storage import RolloutStorage


class RolloutStorageL2C2(RolloutStorage):
    Transition = RolloutStorage.Transition

    def compute_returns(self, last_values, gamma, lam, normalize_advantage: bool = True):
        super().compute_returns(last_values, gamma, lam, True)

    def mini_batch_generator(self, num_mini_batches, num_epochs=8):
        """rollout_storage_l2c2.py:131-167: one randperm over (T-1)*N samples; yields
        (obs, critic_obs, next_obs, cont, actions, values, advantages, returns, old_logp,
        old_mu, old_sigma, (None, None), None)."""
        if self.training_type != "rl":
            raise ValueError("This function is only available for reinforcement learning training.")
        T = self.num_transitions_per_env
        if T < 2:
            raise ValueError("L2C2 needs at least 2 transitions per env (pairs obs[t] with obs[t+1])")
        batch_size = self.num_envs * (T - 1)
        mini_batch_size = batch_size // num_mini_batches
        indices = torch.randperm(num_mini_batches * mini_batch_size, requires_grad=False, device=self.device)
        observations = self.observations[:T - 1].flatten(0, 1)
        critic = (self.privileged_observations[:T - 1].flatten(0, 1)
                  if self.privileged_observations is not None else observations)
        next_observations = self.observations[1:T].flatten(0, 1)
        actions = self.actions[:T - 1].flatten(0, 1)
        values = self.values[:T - 1].flatten(0, 1)
        returns = self.returns[:T - 1].flatten(0, 1)
        old_logp = self.actions_log_prob[:T - 1].flatten(0, 1)
        advantages = self.advantages[:T - 1].flatten(0, 1)
        old_mu = self.mu[:T - 1].flatten(0, 1)
        old_sigma = self.sigma[:T - 1].flatten(0, 1)
        not_dones = 1 - self.dones[:T - 1].float().flatten(0, 1)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                idx = indices[i * mini_batch_size:(i + 1) * mini_batch_size]
                yield (observations[idx].float(), critic[idx].float(), next_observations[idx].float(),
                       not_dones[idx], actions[idx], values[idx], advantages[idx], returns[idx], old_logp[idx],
                       old_mu[idx], old_sigma[idx], (None, None), None)
