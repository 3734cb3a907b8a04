"""PPOL2C2 — PPO with the L2C2 smoothness regulariser
(standalone/rsl_rl/ext/algorithms/ppo_l2c2.py:8-212), the algorithm the vision racing
recipe registers (quadcopter_diff/agents/rsl_rl_ppo_cfg.py:87-101, class_name="PPOL2C2").

Same act / process_env_step / compute_returns / PPO losses as PPO, plus, per
minibatch (ppo_l2c2.py:176-190):
    eps   = lb / (ub - lb);   c_pi = ub * eps;   c_v = value_smoothness_coef * c_pi
    w     = cont * U(-1, 1)                           (one scalar per sample; 0 across a reset)
    o_mix = o + w * (o_next - o)
    L_s   = c_pi * mean(|mu(o) - mu(o_mix)|^2) + c_v * mean(|V(o) - V(o_mix)|^2)
added to the PPO loss.  Multi-GPU as in PPO: KL mean averaged across ranks
before the learning-rate decision, gradients averaged in one flat all-reduce.

Deviations (documented):
  * `act_inference` of the reference's VisionActorCritic returns (mean, feat) and
    ppo_l2c2.py:184,189 take `[0]`; on a plain ActorCritic `[0]` would pick the first
    ROW of the mean and broadcast it.  Here `_mean_of` takes [0] only of a tuple.
  * the transition is stored unless the whole observation batch is ~0
    (ppo_l2c2.py:98), as in the reference; that test costs one host sync per step.  With the
    observation sink (the camera kernel writes the rows into the storage slot) the test runs in act(),
    on the same rows, and a skipped transition's successor rows move down into its slot
    (RolloutStorage.sink_skipped).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from . import distributed as gdist
from . import flat_adam as _fadam
from . import fused_loss as _floss
from .ppo import PPO, _GraphedStep
from .rollout_storage_l2c2 import RolloutStorageL2C2


def _mean_of(out):
    return out[0] if isinstance(out, (tuple, list)) else out


def _mix(obs, next_obs, w):
    """obs + w * (next_obs - obs) (ppo_l2c2.py:179-180), w [rows, 1]: on the GPU one pass of gr_l2c2_mix (the same
    three fp32 roundings as the torch expression), else the expression."""
    fused = (obs.is_cuda and obs.dim() == 2 and obs.dtype == torch.float32 and next_obs.dtype == torch.float32
             and obs.shape == next_obs.shape and obs.shape[1] % 4 == 0 and w.numel() == obs.shape[0]
             and obs.is_contiguous() and next_obs.is_contiguous()
             and not (obs.requires_grad or next_obs.requires_grad or w.requires_grad))
    if fused:
        from .. import _abi

        w = w.reshape(-1).float().contiguous()
        out = torch.empty_like(obs)
        rc = _abi.load().gr_l2c2_mix(obs.data_ptr(), next_obs.data_ptr(), w.data_ptr(), obs.shape[0], obs.shape[1],
                                     out.data_ptr(), _abi.raw_stream(obs.device))
        if rc != 0:
            raise RuntimeError(f"gr_l2c2_mix failed (status {rc})")
        return out
    return obs + w * (next_obs - obs)


def _mix_rows(src, rows_obs, rows_next, w):
    """_mix(src[rows_obs], src[rows_next], w) in one pass over the storage rows (gr_l2c2_mix_rows): no gathered copies
    of the pair."""
    from .. import _abi

    w = w.reshape(-1).float().contiguous()
    out = torch.empty(rows_obs.numel(), src.shape[1], device=src.device, dtype=torch.float32)
    rc = _abi.load().gr_l2c2_mix_rows(src.data_ptr(), src.data_ptr(), src.stride(0), rows_obs.data_ptr(),
                                      rows_next.data_ptr(), w.data_ptr(), out.shape[0], out.shape[1], out.data_ptr(),
                                      _abi.raw_stream(src.device))
    if rc != 0:
        raise RuntimeError(f"gr_l2c2_mix_rows failed (status {rc})")
    return out


class PPOL2C2(PPO):
    def __init__(self, policy, env=None, value_smoothness_coef=0.1, smoothness_upper_bound=1.0,
                 smoothness_lower_bound=0.1, share_mix_features=True, rows_update=True, **kwargs):
        kwargs.pop("normalize_advantage", None)
        # one stem evaluation of the mixed batch for the actor and the critic (policies with shared_features)
        self.share_mix_features = bool(share_mix_features)
        # the graphed update reads the mini-batch's image rows through its permutation (no gathered copies)
        self.rows_update = bool(rows_update)
        super().__init__(policy, env=env, normalize_advantage=True, **kwargs)
        self.transition = RolloutStorageL2C2.Transition()
        self._mix_uniform = torch.rand_like  # the smoothness loss's uniform draw (tests substitute a fixed one)
        self.value_smoothness_coef = value_smoothness_coef
        self.smoothness_upper_bound = smoothness_upper_bound
        self.smoothness_lower_bound = smoothness_lower_bound

    def init_storage(self, training_type, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                     action_shape):
        self.storage = RolloutStorageL2C2(training_type, num_envs, num_transitions_per_env, actor_obs_shape,
                                          critic_obs_shape, action_shape, self.device,
                                          obs_dtype=self.storage_obs_dtype)
        self._init_fused(num_envs)

    def smooth_coefs(self):
        """ppo_l2c2.py:176-178."""
        eps = self.smoothness_lower_bound / (self.smoothness_upper_bound - self.smoothness_lower_bound)
        policy_coef = self.smoothness_upper_bound * eps
        return policy_coef, self.value_smoothness_coef * policy_coef

    def _store_test(self, obs):
        """ppo_l2c2.py:98's zero-observation test on these rows, issued before the policy forward and the env step
        (stream order: the step cannot have touched them yet).  On the GPU its result is copied to pinned host
        memory behind an event and read in process_env_step: the host never waits for the policy forward or the env
        step, only for this reduction, long finished by then (the same decision, no per-step drain of the queue)."""
        flag = torch.norm(obs).mean() > 1e-4
        if not flag.is_cuda:
            self._store_flag = bool(flag)
            return
        if getattr(self, "_flag_host", None) is None:
            with torch.inference_mode(False):
                self._flag_host = torch.zeros((), dtype=torch.bool, pin_memory=True)
            self._flag_event = torch.cuda.Event()
        self._flag_host.copy_(flag, non_blocking=True)
        self._flag_event.record()
        self._store_flag = None

    def _stored(self) -> bool:
        if not hasattr(self, "_store_flag"):  # (a transition stored without act: test its rows now)
            self._store_test(self.transition.observations)
        if self._store_flag is None:
            self._flag_event.synchronize()
            self._store_flag = bool(self._flag_host)
        return self._store_flag

    def act(self, obs, critic_obs):
        # (with the observation sink the rows of a skipped transition are moved down a slot and the env's next step
        # writes the slot `obs` views: the test is on these rows as they are now)
        self._store_test(obs)
        return super().act(obs, critic_obs)

    def process_env_step(self, rewards, dones, infos):
        self.transition.rewards = rewards.clone()
        self.transition.dones = dones
        if "time_outs" in infos:  # ppo_l2c2.py:91-95
            self.transition.rewards += self.gamma * torch.squeeze(
                self.transition.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        sink = getattr(self.storage, "sink", False)
        store = self._stored()  # ppo_l2c2.py:98
        del self._store_flag
        if store:
            self.storage.add_transitions(self.transition)
        elif sink:
            self.storage.sink_skipped()
        self.transition.clear()
        self.policy.reset(dones)

    def smooth_loss(self, obs_batch, next_obs_batch, cont_batch, mu_batch, value_batch, rows=None,
                    want_smoothness=True):
        """ppo_l2c2.py:176-188; returns (smooth_loss, action_smoothness).  rows (src, idx, next_idx): the pair is
        src[idx], src[next_idx] (the rollout storage's rows, read through the indices; obs_batch / next_obs_batch
        unused).  want_smoothness False (the update, which never reads it, ppo_l2c2.py:188-191): action_smoothness is
        None and the successor forward runs only for its side effects, the BatchNorm statistics of a training-mode
        forward (policies with record_batch_statistics; none for the others)."""
        policy_coef, value_coef = self.smooth_coefs()
        mix_weights = cont_batch * (self._mix_uniform(cont_batch) - 0.5) * 2.0
        if rows is not None:
            mix_obs_batch = _mix_rows(rows[0], rows[1], rows[2], mix_weights)
        else:
            mix_obs_batch = _mix(obs_batch, next_obs_batch, mix_weights)
        shared = getattr(self.policy, "shared_features", None)
        if shared is not None and self.share_mix_features:
            # the actor's and the critic's forward of the mixed batch share one stem evaluation (VisionActorCritic:
            # the same features, BatchNorm running statistics updated as by the reference's two forwards)
            feat = shared(mix_obs_batch, 2)
            mix_mean, mix_value = self.policy.actor(feat), self.policy.critic(feat)
        else:
            mix_mean = _mean_of(self.policy.act_inference(mix_obs_batch))
            mix_value = self.policy.evaluate(mix_obs_batch)
        policy_smooth = torch.square(torch.norm(mu_batch - mix_mean, dim=-1)).mean()
        value_smooth = torch.square(torch.norm(value_batch - mix_value, dim=-1)).mean()
        loss = policy_coef * policy_smooth + value_coef * value_smooth
        with torch.inference_mode():
            if not want_smoothness:
                record = getattr(self.policy, "record_batch_statistics", None)
                if record is not None:
                    record(*((rows[0], rows[2]) if rows is not None else (next_obs_batch,)))
                return loss, None
            if rows is not None:
                next_mean = self.policy.actor(self.policy.features_rows(rows[0], rows[2]))
            else:
                next_mean = _mean_of(self.policy.act_inference(next_obs_batch))
            action_smoothness = torch.norm(mu_batch - next_mean, dim=-1).mean()
        return loss, action_smoothness

    def update(self):
        if self.graph_update and self.storage is not None and str(self.device).startswith("cuda"):
            if self._graphed is None:
                self._graphed = _GraphedStepL2C2(self)
            out = self._graphed.update()
            if self.fused is not None:  # graph replays write the parameters without bumping their versions
                self.fused.refresh()
            return out
        mean_value_loss = torch.zeros((), device=self.device)
        mean_surrogate_loss = torch.zeros((), device=self.device)
        mean_smooth_loss = torch.zeros((), device=self.device)
        generator = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        params = list(self.policy.parameters())
        flat = self.flat_grads()
        flat.bind()
        for (obs_batch, critic_obs_batch, next_obs_batch, cont_batch, actions_batch, target_values_batch,
             advantages_batch, returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch,
             hid_states_batch, masks_batch) in generator:
            self.policy.act(obs_batch)
            actions_log_prob_batch = self.policy.get_actions_log_prob(actions_batch)
            value_batch = self.policy.evaluate(critic_obs_batch)
            mu_batch = self.policy.action_mean
            sigma_batch = self.policy.action_std
            entropy_batch = self.policy.entropy
            self._adapt_learning_rate(mu_batch, sigma_batch, old_mu_batch, old_sigma_batch)
            surrogate_loss, value_loss = self._ppo_losses(actions_log_prob_batch, old_actions_log_prob_batch,
                                                          advantages_batch, value_batch, target_values_batch,
                                                          returns_batch)
            loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_batch.mean()
            smooth_loss, _ = self.smooth_loss(obs_batch, next_obs_batch, cont_batch, mu_batch, value_batch,
                                              want_smoothness=False)
            loss = loss + smooth_loss
            self.optimizer.zero_grad(set_to_none=False)
            if not self._grads_checked:
                flat = self._check_all_grads(loss, params)
                flat.bind()
            loss.backward()
            gdist.allreduce_grads(params, flat)
            _fadam.clip_grad_norm_(self.optimizer, params, self.max_grad_norm)
            self.optimizer.step()
            mean_value_loss += value_loss.detach()
            mean_surrogate_loss += surrogate_loss.detach()
            mean_smooth_loss += smooth_loss.detach()
        num_updates = self.num_learning_epochs * self.num_mini_batches
        self.storage.clear()
        return {
            "value_function": float(mean_value_loss) / num_updates,
            "surrogate": float(mean_surrogate_loss) / num_updates,
            "smooth_loss": float(mean_smooth_loss) / num_updates,
        }


class _GraphedStepL2C2(_GraphedStep):
    """PPOL2C2.update's mini-batch step as hipGraph replays (ppo.py _GraphedStep: one graph per epoch on one rank,
    two segments around the eager all-reduce on several): the vision recipe's update is ~590 launches per
    mini-batch, most of them small, and the eager loop reads the KL back to the host once per mini-batch.

    Segment A is ppo_l2c2.py:127-191 on the mini-batch gathered by a static index buffer from the (T-1) N samples
    (rollout_storage_l2c2.py:131-167; the continuation flags in a persistent buffer refreshed per update): the
    distribution and values, the KL mean into the flat buffer's extra slot, the PPO losses, the smoothness loss
    (its own uniform draw per replay: torch's graph-safe generator), and the backward into the flat gradient
    views.  Segment B is the base class's: the rate rule on the device, the clip and Adam.  As in _GraphedStep the
    learning rate is an fp32 device tensor and the eager loop's unused action draw is not made; the BatchNorm
    running statistics of the warm-up and captured steps are restored after the capture."""

    _PACK = False  # (the pairs are gathered field by field, _gather: no packed copy of the samples)

    def __init__(self, alg: "PPOL2C2"):
        super().__init__(alg)
        st, dev = alg.storage, alg.device
        if self.T < 2:
            raise ValueError("L2C2 needs at least 2 transitions per env (pairs obs[t] with obs[t+1])")
        self.mb = (self.T - 1) * self.N // self.nmb
        self.perm = torch.zeros(self.nmb * self.mb, dtype=torch.long, device=dev)
        self.idx = self.perm[:self.mb]
        self.acc = torch.zeros(3, device=dev)  # the update's sums of the surrogate, value and smoothness means
        self.cont = torch.zeros((self.T - 1) * self.N, 1, device=dev)

    def _refresh_sources(self):
        st = self.alg.storage
        with torch.no_grad():
            torch.sub(1.0, st.dones[:self.T - 1].float().flatten(0, 1), out=self.cont)

    def _sources(self):
        st, T = self.alg.storage, self.T
        obs = st.observations[:T - 1].flatten(0, 1)
        crit = st.privileged_observations[:T - 1].flatten(0, 1) if st.privileged_observations is not None else obs
        return (obs, crit, st.observations[1:T].flatten(0, 1), self.cont) + tuple(
            x[:T - 1].flatten(0, 1) for x in (st.actions, st.values, st.advantages, st.returns, st.actions_log_prob,
                                               st.mu, st.sigma))

    def _gather(self, idx):
        return tuple(x.index_select(0, idx) for x in self._sources())

    def _fused_losses_ok(self, obs) -> bool:
        """The PPO losses as one device op each way (fused_loss._PPOLossCombinedFn, as PPO's graphed step uses them):
        a policy with actor / critic heads and a state-independent std over <= 8 actions, fp32 outside autocast."""
        pol = self.alg.policy
        return (self.alg.fused_losses and obs.is_cuda and obs.dtype == torch.float32 and hasattr(pol, "features")
                and isinstance(pol.actor, nn.Sequential) and pol.actor[-1].out_features <= 8
                and getattr(pol, "noise_std_type", None) in ("scalar", "log")
                and not torch.is_autocast_enabled("cuda"))

    def _rows_ok(self) -> bool:
        """The mini-batch's image rows read through the permutation (VisionActorCritic.features_rows, the fused
        first block's row indices, gr_l2c2_mix_rows) instead of gathered: fp32 storage rows, a policy with
        features_rows, the fused losses."""
        st, pol = self.alg.storage, self.alg.policy
        srcs = [st.observations] + ([st.privileged_observations] if st.privileged_observations is not None else [])
        return (self.alg.rows_update and hasattr(pol, "features_rows") and st.observations.is_cuda
                and all(x.dtype == torch.float32 and x.is_contiguous() for x in srcs)
                and st.observations.shape[-1] % 4 == 0 and self._fused_losses_ok(st.observations[0]))

    def _seg_a_rows(self, idx):
        """Segment A with the image rows read through `idx` (the same values as the gathered form)."""
        alg, pol, st = self.alg, self.alg.policy, self.alg.storage
        src = st.observations.flatten(0, 1)  # row j + N is the successor of row j
        csrc = st.privileged_observations.flatten(0, 1) if st.privileged_observations is not None else src
        nidx = idx + self.N
        cont, act, val, adv, ret, logp, mu, sig = (x.index_select(0, idx) for x in self._sources()[3:])
        mu_b = pol.actor(pol.features_rows(src, idx))
        value_b = pol.critic(pol.features_rows(csrc, idx))
        std = _floss._policy_std(pol)
        loss, _ = _floss._PPOLossCombinedFn.apply(
            mu_b, std, value_b, act, logp, adv, val, ret, mu, sig, float(alg.clip_param),
            bool(alg.use_clipped_value_loss), float(alg.value_loss_coef), self.acc[:2],
            self.flat.extra[:1] if self._adaptive() else None, None)
        if alg.entropy_coef != 0.0:
            loss = loss - alg.entropy_coef * (0.5 + 0.5 * math.log(2.0 * math.pi) + torch.log(std)).sum()
        smooth_loss, _ = alg.smooth_loss(None, None, cont, mu_b, value_b, rows=(src, idx, nidx),
                                         want_smoothness=False)
        self.acc[2:].add_(smooth_loss.detach())
        self._backward(loss + smooth_loss)

    def _seg_a(self, idx=None):
        alg, pol = self.alg, self.alg.policy
        idx = self.idx if idx is None else idx
        if self._rows_ok():
            self._seg_a_rows(idx)
            return
        obs, crit, nxt, cont, act, val, adv, ret, logp, mu, sig = self._gather(idx)
        obs, crit, nxt = obs.float(), crit.float(), nxt.float()
        if self._fused_losses_ok(obs):
            # ppo_l2c2.py:127-175 with the log prob, KL, surrogate and value losses in one launch each way; the KL
            # mean lands in the flat buffer's extra slot, the surrogate and value means accumulate in acc[:2]
            mu_b = pol.actor(pol.features(obs))
            value_b = pol.critic(pol.features(crit))
            std = _floss._policy_std(pol)
            loss, _ = _floss._PPOLossCombinedFn.apply(
                mu_b, std, value_b, act, logp, adv, val, ret, mu, sig, float(alg.clip_param),
                bool(alg.use_clipped_value_loss), float(alg.value_loss_coef), self.acc[:2],
                self.flat.extra[:1] if self._adaptive() else None, None)
            if alg.entropy_coef != 0.0:  # Normal.entropy summed over the actions: the same for every sample
                loss = loss - alg.entropy_coef * (0.5 + 0.5 * math.log(2.0 * math.pi) + torch.log(std)).sum()
            smooth_loss, _ = alg.smooth_loss(obs, nxt, cont, mu_b, value_b, want_smoothness=False)
            self.acc[2:].add_(smooth_loss.detach())
            self._backward(loss + smooth_loss)
            return
        pol.update_distribution(obs)
        logp_b = pol.get_actions_log_prob(act)
        value_b = pol.evaluate(crit)
        mu_b, sigma_b, entropy_b = pol.action_mean, pol.action_std, pol.entropy
        if self._adaptive():
            with torch.no_grad():
                kl = torch.sum(torch.log(sigma_b / sig + 1.0e-5)
                               + (torch.square(sig) + torch.square(mu - mu_b)) / (2.0 * torch.square(sigma_b)) - 0.5,
                               axis=-1)
                self.flat.extra[0].copy_(torch.mean(kl))
        surrogate_loss, value_loss = alg._ppo_losses(logp_b, logp, adv, value_b, val, ret)
        loss = surrogate_loss + alg.value_loss_coef * value_loss - alg.entropy_coef * entropy_b.mean()
        smooth_loss, _ = alg.smooth_loss(obs, nxt, cont, mu_b, value_b, want_smoothness=False)
        loss = loss + smooth_loss
        self.acc.add_(torch.stack([surrogate_loss.detach(), value_loss.detach(), smooth_loss.detach()]))
        self._backward(loss)

    def _stats(self, num_updates):
        sl, vl, ml = self.acc.tolist()
        return {"value_function": vl / num_updates, "surrogate": sl / num_updates, "smooth_loss": ml / num_updates}
