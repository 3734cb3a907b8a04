"""PPO (standalone/rsl_rl/ext/algorithms/ppo.py:14-190) + data parallelism.

Same act / process_env_step (time-out bootstrap) / compute_returns / update
as the reference: clipped surrogate, clipped value loss, adaptive-KL learning
rate, grad-norm clipping, Adam.  Added for the multi-GPU path:
the KL mean is averaged across ranks before the learning-rate decision and
gradients are averaged in one flat all-reduce before clipping, so every rank
applies the identical update.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn
import torch.optim as optim
import torch.distributed as dist

from . import distributed as gdist
from . import flat_adam as _fadam
from . import fused_loss as _floss
from . import linear as _lin
from . import rollout_ops as _rops
from .rollout_storage import RolloutStorage


class PPO:
    def __init__(self, policy, env=None, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998,
                 lam=0.95, value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu",
                 normalize_advantage=True, storage_obs_dtype=torch.float32, fused_rollout_inference=False,
                 fused_rollout_precision="bf16", graph_update=False, update_autocast_bf16=False,
                 graph_update_segmented=False, fused_losses=True, fused_adam=True, fused_mlp=True,
                 graph_update_per_step=False, **kwargs):
        self.env = env
        self.device = device
        self.desired_kl = desired_kl
        self.schedule = schedule
        self.learning_rate = learning_rate
        self.policy = policy
        self.policy.to(self.device)
        gdist.broadcast_params(self.policy)
        self.storage: RolloutStorage | None = None
        # Adam (ppo.py:39) and the grad-norm clip as four device launches over the parameter table on CUDA
        # (flat_adam.py); torch.optim.Adam + nn.utils.clip_grad_norm_ on CPU or with fused_adam=False
        self.optimizer = _fadam.make_adam(self.policy.parameters(), learning_rate, fused=fused_adam)
        self.transition = RolloutStorage.Transition()
        self.clip_param = clip_param
        self.num_learning_epochs = num_learning_epochs
        self.num_mini_batches = num_mini_batches
        self.value_loss_coef = value_loss_coef
        self.entropy_coef = entropy_coef
        self.gamma = gamma
        self.lam = lam
        self.max_grad_norm = max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.normalize_advantage = normalize_advantage
        # "float32" / "bfloat16" from a cfg dict, or a torch dtype (BASELINE C5: bf16 rollout obs buffers)
        self.storage_obs_dtype = getattr(torch, storage_obs_dtype) if isinstance(storage_obs_dtype, str) \
            else storage_obs_dtype
        # rollout inference on MFMA (rsl_rl/fused_inference.py, BASELINE config C5): bf16 operands, fp32
        # accumulation, one launch for actor + sampling + log prob + critic; the update stays fp32 PyTorch
        self.fused_rollout_inference = bool(fused_rollout_inference)
        self.fused_rollout_precision = str(fused_rollout_precision)
        self.fused = None
        # the update's mini-batch step (gather, forward, adaptive learning rate, losses, backward, clip,
        # Adam) captured once in a hipGraph and replayed per mini-batch (single rank, GPU): see _GraphedStep
        self.graph_update = bool(graph_update)
        # two graph segments with the collectives run eagerly between them: always at world size > 1; this
        # switch forces it on one rank (tests: the segmented step must equal the single graph)
        self.graph_update_segmented = bool(graph_update_segmented)
        # one graph per mini-batch step instead of one per epoch (the state between steps can be inspected: tests)
        self.graph_update_per_step = bool(graph_update_per_step)
        self._graphed = None
        self._grads_checked = False  # which parameters the loss reaches (see _check_all_grads)
        self._unused: set = set()
        # not in the reference (fp32 update): forward/backward of the update under torch.autocast(bf16);
        # the losses' exp / log / sums stay fp32 (autocast's fp32 list), parameters and Adam stay fp32
        self.update_autocast_bf16 = bool(update_autocast_bf16)
        self._flat = None  # gdist.FlatGrads: the parameters' gradients as views of one buffer
        # the mini-batch losses (log prob, KL, surrogate, value loss) as one device op each way on CUDA
        # (fused_loss.py); False: the torch ops
        self.fused_losses = bool(fused_losses)
        # with the fused losses: the actor and critic MLPs as whole-network fp32-MFMA kernels (linear.fused_mlps)
        self.fused_mlp = bool(fused_mlp)

    def flat_grads(self) -> gdist.FlatGrads:
        """The flat gradient buffer over the parameters the loss reaches (all of them until the first mini-batch
        has been checked, see _check_all_grads)."""
        used = [p for p in self.policy.parameters() if id(p) not in self._unused]
        if self._flat is None or len(self._flat.params) != len(used) or \
                any(a is not b for a, b in zip(self._flat.params, used)):
            self._flat = gdist.FlatGrads(used)
        return self._flat

    def init_storage(self, training_type, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                     action_shape):
        self.storage = RolloutStorage(training_type, num_envs, num_transitions_per_env, actor_obs_shape,
                                      critic_obs_shape, action_shape, self.device, obs_dtype=self.storage_obs_dtype)
        self._init_fused(num_envs)

    def _init_fused(self, num_envs):
        if not self.fused_rollout_inference:
            return
        from .fused_inference import FusedPolicyInference

        ucfg = getattr(getattr(self.env, "unwrapped", None), "cfg", None)
        seed = getattr(ucfg, "seed", None)
        self.fused = FusedPolicyInference(self.policy, num_envs, self.device, seed=42 if seed is None else int(seed),
                                          env_id_offset=int(getattr(ucfg, "env_id_offset", 0) or 0),
                                          precision=self.fused_rollout_precision)

    def test_mode(self):
        self.policy.eval()

    def train_mode(self):
        self.policy.train()

    def act(self, obs, critic_obs):
        if self.fused is not None:
            a, v, lp, mu, sd = self.fused.act(obs, critic_obs)
            self.transition.actions, self.transition.values, self.transition.actions_log_prob = a, v, lp
            self.transition.action_mean, self.transition.action_sigma = mu, sd
            self.transition.observations = obs
            self.transition.privileged_observations = critic_obs
            return a
        self.transition.actions = self.policy.act(obs).detach()
        self.transition.values = self.policy.evaluate(critic_obs).detach()
        self.transition.actions_log_prob = self.policy.get_actions_log_prob(self.transition.actions).detach()
        self.transition.action_mean = self.policy.action_mean.detach()
        self.transition.action_sigma = self.policy.action_std.detach()
        self.transition.observations = obs
        self.transition.privileged_observations = critic_obs
        return self.transition.actions

    def process_env_step(self, rewards, dones, infos):
        tos = infos.get("time_outs")
        tos = tos.to(self.device) if tos is not None else None
        if _rops.store_ok(self.storage, self.transition, rewards, dones, tos):
            # the bootstrap below and add_transitions as one launch (rollout_ops.py), the same bits
            _rops.store_transition(self.storage, self.transition, rewards, dones, tos, self.gamma)
            self.transition.clear()
            self.policy.reset(dones)
            return
        self.transition.rewards = rewards.clone()
        self.transition.dones = dones
        if "time_outs" in infos:  # bootstrapping on time outs (ppo.py:88-92)
            self.transition.rewards += self.gamma * torch.squeeze(
                self.transition.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(self.transition)
        self.transition.clear()
        self.policy.reset(dones)

    def compute_returns(self, last_critic_obs):
        last_values = self.policy.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam, self.normalize_advantage)

    def _adapt_learning_rate(self, mu_batch, sigma_batch, old_mu_batch, old_sigma_batch):
        """Adaptive KL learning rate (ppo.py:133-150); KL mean averaged over ranks."""
        if self.desired_kl is None or self.schedule != "adaptive":
            return
        with torch.inference_mode():
            kl = torch.sum(
                torch.log(sigma_batch / old_sigma_batch + 1.0e-5)
                + (torch.square(old_sigma_batch) + torch.square(old_mu_batch - mu_batch))
                / (2.0 * torch.square(sigma_batch)) - 0.5, axis=-1)
            kl_mean = gdist.allreduce_mean(torch.mean(kl))
            kl_val = float(kl_mean)  # host decision, as in the reference
            if kl_val > self.desired_kl * 2.0:
                self.learning_rate = max(1e-5, self.learning_rate / 1.5)
            elif self.desired_kl / 2.0 > kl_val > 0.0:
                self.learning_rate = min(1e-2, self.learning_rate * 1.5)
            for g in self.optimizer.param_groups:
                g["lr"] = self.learning_rate

    def _ppo_losses(self, actions_log_prob_batch, old_actions_log_prob_batch, advantages_batch, value_batch,
                    target_values_batch, returns_batch):
        """Clipped surrogate (ppo.py:152-158) and (clipped) value loss (ppo.py:160-169)."""
        ratio = torch.exp(actions_log_prob_batch - torch.squeeze(old_actions_log_prob_batch))
        surrogate = -torch.squeeze(advantages_batch) * ratio
        surrogate_clipped = -torch.squeeze(advantages_batch) * torch.clamp(ratio, 1.0 - self.clip_param,
                                                                           1.0 + self.clip_param)
        surrogate_loss = torch.max(surrogate, surrogate_clipped).mean()
        if self.use_clipped_value_loss:
            value_clipped = target_values_batch + (value_batch - target_values_batch).clamp(-self.clip_param,
                                                                                            self.clip_param)
            value_losses = (value_batch - returns_batch).pow(2)
            value_losses_clipped = (value_clipped - returns_batch).pow(2)
            value_loss = torch.max(value_losses, value_losses_clipped).mean()
        else:
            value_loss = (returns_batch - value_batch).pow(2).mean()
        return surrogate_loss, value_loss

    def _check_all_grads(self, loss, params, grads=None):
        """Find the parameters the loss does not reach (e.g. VisionActorCritic's aux_decoder) and take them out of
        the flat gradient buffer, with `.grad` None: the reference's `zero_grad()` leaves their `.grad` None and
        Adam skips them (ppo.py:178-181), where a bound zero `.grad` would count an Adam step for them (and step
        them by their moments if they ever had any).  Checked once, on the first mini-batch: the set of parameters
        the loss reaches must not change afterwards.  The eager update raises if a dropped parameter later receives a
        gradient (PPO.update); the graphed update differentiates only the parameters kept here."""
        if grads is None:
            grads = torch.autograd.grad(loss, params, retain_graph=True, allow_unused=True)
        self._unused = {id(p) for p, g in zip(params, grads) if g is None}
        for p in self.policy.parameters():
            if id(p) in self._unused:
                p.grad = None
        self._grads_checked = True
        return self.flat_grads()

    def update(self):
        if self.graph_update and self.storage is not None and str(self.device).startswith("cuda") \
                and type(self).update is PPO.update:
            if self._graphed is None:
                self._graphed = _GraphedStep(self)
            out = self._graphed.update()
            if self.fused is not None:  # graph replays write the parameters without bumping their versions
                self.fused.refresh()
            return out
        mean_value_loss = torch.zeros((), device=self.device)
        mean_surrogate_loss = torch.zeros((), device=self.device)
        generator = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs)
        params = list(self.policy.parameters())
        flat = self.flat_grads()
        flat.bind()
        ac = torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.update_autocast_bf16 and
                            str(self.device).startswith("cuda"))
        for (obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch, returns_batch,
             old_actions_log_prob_batch, old_mu_batch, old_sigma_batch, hid_states_batch, masks_batch) in generator:
            if self._use_fused_losses(obs_batch):  # the same losses as one device op each way (fused_loss.py)
                loss, stats = _floss.ppo_loss(
                    self, obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch,
                    returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch)
                surrogate_loss, value_loss = stats[0], stats[1]
                self._adapt_learning_rate_kl(stats[2])
            else:
                surrogate_loss, value_loss, loss = self._torch_losses(
                    ac, obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch,
                    returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch)
            self.optimizer.zero_grad(set_to_none=False)  # (in place: the views of the flat buffer stay bound)
            if not self._grads_checked:
                flat = self._check_all_grads(loss, params)
                flat.bind()
            loss.backward()
            if self._unused and any(p.grad is not None for p in params if id(p) in self._unused):
                raise RuntimeError("PPO.update: a parameter the loss did not reach on the first mini-batch now has a "
                                   "gradient; the set of parameters the loss reaches must be fixed from the first "
                                   "mini-batch (it is checked once: _check_all_grads)")
            gdist.allreduce_grads(params, flat)
            _fadam.clip_grad_norm_(self.optimizer, params, self.max_grad_norm)
            self.optimizer.step()
            mean_value_loss += value_loss.detach()
            mean_surrogate_loss += surrogate_loss.detach()
        num_updates = self.num_learning_epochs * self.num_mini_batches
        self.storage.clear()
        return {
            "value_function": float(mean_value_loss) / num_updates,
            "surrogate": float(mean_surrogate_loss) / num_updates,
        }

    def _use_fused_losses(self, obs) -> bool:
        return (self.fused_losses and obs.is_cuda and not self.update_autocast_bf16
                and _floss.fused_losses_ok(self.policy, obs))

    def _adapt_learning_rate_kl(self, kl_mean):
        """_adapt_learning_rate from the mini-batch's KL mean (computed by the fused losses)."""
        if self.desired_kl is None or self.schedule != "adaptive":
            return
        kl_val = float(gdist.allreduce_mean(kl_mean.detach()))  # host decision, as in the reference
        if kl_val > self.desired_kl * 2.0:
            self.learning_rate = max(1e-5, self.learning_rate / 1.5)
        elif self.desired_kl / 2.0 > kl_val > 0.0:
            self.learning_rate = min(1e-2, self.learning_rate * 1.5)
        for g in self.optimizer.param_groups:
            g["lr"] = self.learning_rate

    def _torch_losses(self, ac, obs_batch, critic_obs_batch, actions_batch, target_values_batch, advantages_batch,
                      returns_batch, old_actions_log_prob_batch, old_mu_batch, old_sigma_batch):
        """ppo.py:103-169 as torch ops (CPU, autocast, other policies)."""
        with ac:
                self.policy.act(obs_batch)
                actions_log_prob_batch = self.policy.get_actions_log_prob(actions_batch)
                value_batch = self.policy.evaluate(critic_obs_batch)
                mu_batch = self.policy.action_mean
                sigma_batch = self.policy.action_std
                entropy_batch = self.policy.entropy
        self._adapt_learning_rate(mu_batch.float(), sigma_batch.float(), old_mu_batch, old_sigma_batch)
        surrogate_loss, value_loss = self._ppo_losses(actions_log_prob_batch.float(), old_actions_log_prob_batch,
                                                      advantages_batch, value_batch.float(), target_values_batch,
                                                      returns_batch)
        loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_batch.float().mean()
        return surrogate_loss, value_loss, loss


class _GraphedStep:
    """PPO.update's mini-batch step as hipGraph replays (the same operations as the eager loop).

    Per mini-batch the eager loop launches ~150 small kernels and reads the KL back to the host for the
    adaptive learning rate (ppo.py:133-150).  Here the learning-rate rule runs on the device (the same
    comparisons, in fp32), Adam takes the rate as a device tensor (FlatAdam's lr pointer, or torch's
    `capturable=True` with fused_adam off), and the step
    (mini-batch gathers from the storage by a static index buffer, forward, losses, backward, grad
    clipping, Adam) is captured once and replayed per mini-batch.  Capture needs warm-up steps; the
    parameters, the optimizer state and the rate are snapshotted before and restored after, so training
    is unchanged.  `learning_rate` is read back once per update, for the log.

    Gradients: `torch.autograd.grad` into the views of one flat buffer (gdist.FlatGrads, bound as the
    parameters' `.grad` before capture and never rebound), so the captured step does not depend on how
    autograd's gradient accumulation treats an existing `.grad` (an out-of-place accumulation during
    capture rebinds `.grad` and leaves the graph writing a buffer nobody holds).  The mini-batch's local KL
    mean is written into the flat buffer's extra slot.

    Two segments: A = gathers, forward, KL, losses, backward (into the flat buffer); B = learning-rate rule,
    clip, Adam.  The rate only enters Adam, so computing it after the backward changes nothing.  With one
    rank both segments of every mini-batch of an epoch are one graph (each step gathers by its own slice of the
    update's permutation), replayed once per epoch.  With several ranks (any backend) they are two graphs and the exchange
    runs eagerly between them: ONE in-place all-reduce of the flat buffer carries the gradients and the KL
    mean together.  No collective is ever captured."""

    _PACK = True  # gather the mini-batch from the storage's packed sample rows when it has them

    def __init__(self, alg: "PPO"):
        self.alg = alg
        st, dev = alg.storage, alg.device
        self.T, self.N = st.num_transitions_per_env, st.num_envs
        self.mb = self.T * self.N // alg.num_mini_batches
        self.params = list(alg.policy.parameters())
        self.lr = torch.tensor(float(alg.learning_rate), device=dev, dtype=torch.float32)
        old = alg.optimizer
        if isinstance(old, _fadam.FlatAdam):  # the same launches eager or captured: the rate as a device tensor
            self.opt = old
            self.opt.param_groups[0]["lr"] = self.lr
        else:
            self.opt = optim.Adam(self.params, lr=self.lr, capturable=True)
            if old.state:  # resumed from a checkpoint: keep Adam's moments and step counts
                self.opt.load_state_dict(old.state_dict())
            for g in self.opt.param_groups:  # (load_state_dict brings the eager groups' settings)
                g["lr"] = self.lr
                g["capturable"] = True
        alg.optimizer = self.opt
        self.flat = alg.flat_grads()
        self.nmb = alg.num_mini_batches
        # the update's permutation (rollout_storage.py:152-191: one draw, the same mini-batch partition every epoch);
        # one rank: ONE graph holds an epoch's mini-batch steps, each gathering by its own slice of this buffer (no
        # per-step index copy or replay launch); several ranks: per-step graphs read `idx`, refilled per step
        self.perm = torch.zeros(self.nmb * self.mb, dtype=torch.long, device=dev)
        self.idx = self.perm[:self.mb]
        # packed sample rows (None: gathered field by field); a subclass gathering its own fields sets _PACK False and
        # never allocates the buffer
        self.cols = st.sample_columns() if self._PACK else None
        # persistent: the graphs read it (the storage's own packed buffer, shared with the eager generator)
        self.pack = st.pack_samples(out=st.packed_buffer()) if self.cols is not None else None
        self.acc = torch.zeros(2, device=dev)  # the update's sums of the surrogate and value means
        self.one = torch.ones((), device=dev)
        self.segmented = gdist.is_dist() or alg.graph_update_segmented
        self.per_step = self.segmented or alg.graph_update_per_step
        # epoch graph + packed rows: the samples in the update's permutation order, gathered ONCE per update (every
        # epoch uses the same partition, rollout_storage.py:152-191), so mini-batch i is the contiguous row slice i and
        # the captured steps gather nothing (the per-step gathers were latency-bound launches, one per step)
        self.pack_perm = torch.empty_like(self.pack) if self.pack is not None and not self.per_step else None
        self.graph = None  # one rank: an epoch's steps (per_step: one step)
        self.graph_b = None  # segmented: graph = segment A, graph_b = segment B

    def _gather(self, idx):
        """The mini-batch's fields by a static index buffer: one row gather of the packed samples (refilled
        before every update's replays, RolloutStorage.pack_samples), or one gather per field for wide rows.  idx a
        (lo, hi) pair: rows lo .. hi of the permuted packed samples (pack_perm), views, no gather."""
        st = self.alg.storage
        if isinstance(idx, tuple):
            g = self.pack_perm[idx[0]:idx[1]]
            return tuple(g[:, a:b] for a, b in self.cols)
        if self.cols is not None:
            g = self.pack.index_select(0, idx)
            return tuple(g[:, a:b] for a, b in self.cols)
        return tuple(x.index_select(0, idx) for x in st.sample_sources())

    def _adaptive(self) -> bool:
        return self.alg.desired_kl is not None and self.alg.schedule == "adaptive"

    def _seg_a(self, idx=None):
        alg, pol = self.alg, self.alg.policy
        obs, priv, act, val, adv, ret, logp, mu, sig = self._gather(self.idx if idx is None else idx)
        obs, priv = obs.float(), priv.float()
        if alg._use_fused_losses(obs):  # (fused_loss.py: one device op each way, the means and the loss finished
            # there: the step's loss sums accumulate in self.acc, the KL mean lands in the flat buffer's extra slot)
            # (the gradients land in the flat buffer's views directly while the sink is set: linear._GRAD_SINK)
            _lin._GRAD_SINK = {id(p): v for p, v in zip(self.flat.params, self.flat.views)}
            try:
                loss, _ = _floss.ppo_loss(alg, obs, priv, act, val, adv, ret, logp, mu, sig, acc=self.acc,
                                          kl_out=self.flat.extra[:1] if self._adaptive() else None, seed=self.one)
            finally:
                _lin._GRAD_SINK = None
            self._backward(loss)
            return
        # the eager loop's policy.act also draws a sample it never uses; torch.normal's check of the std
        # reads back to the host, which a capture forbids, so only the distribution is set here
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=alg.update_autocast_bf16):
            pol.update_distribution(obs)
            logp_b = pol.get_actions_log_prob(act)
            value_b = pol.evaluate(priv)
            mu_b, sigma_b, entropy_b = pol.action_mean, pol.action_std, pol.entropy
        logp_b, value_b, mu_b, sigma_b, entropy_b = (t.float() for t in (logp_b, value_b, mu_b, sigma_b, entropy_b))
        if self._adaptive():
            with torch.no_grad():
                kl = torch.sum(torch.log(sigma_b / sig + 1.0e-5)
                               + (torch.square(sig) + torch.square(mu - mu_b)) / (2.0 * torch.square(sigma_b)) - 0.5,
                               axis=-1)
                self.flat.extra[0].copy_(torch.mean(kl))
        surrogate_loss, value_loss = alg._ppo_losses(logp_b, logp, adv, value_b, val, ret)
        loss = surrogate_loss + alg.value_loss_coef * value_loss - alg.entropy_coef * entropy_b.mean()
        self.acc.add_(torch.stack([surrogate_loss.detach(), value_loss.detach()]))
        self._backward(loss)

    def _backward(self, loss):
        alg = self.alg
        if not alg._grads_checked:  # (first warm-up step, before any capture)
            grads = torch.autograd.grad(loss, self.params, retain_graph=True, allow_unused=True)
            self.flat = alg._check_all_grads(loss, self.params, grads)
            self.flat.bind()
        # (the seed gradient from a persistent 1: no fill launch in the captured step; the fused MLP backward writes
        # its gradients into their flat views directly, linear._GRAD_SINK, and only the others are copied)
        _lin._GRAD_SINK = {id(p): v for p, v in zip(self.flat.params, self.flat.views)}
        try:
            grads = torch.autograd.grad(loss, self.flat.params, grad_outputs=self.one)
        finally:
            _lin._GRAD_SINK = None
        pairs = [(v, g) for v, g in zip(self.flat.views, grads) if g.data_ptr() != v.data_ptr()]
        if pairs:
            torch._foreach_copy_([v for v, _ in pairs], [g for _, g in pairs])

    def _seg_b(self):
        alg = self.alg
        if isinstance(self.opt, _fadam.FlatAdam):  # the rate rule, the clip and Adam: two launches (gr_adam_clip_step)
            self.opt.clip_and_step(alg.max_grad_norm, kl=self.flat.extra if self._adaptive() else None,
                                   desired_kl=alg.desired_kl)
            return
        if self._adaptive():  # on the rank-averaged KL mean once the flat buffer has been all-reduced: the
            # comparisons of ppo.py:133-150 on the device, one launch (gr_adaptive_lr)
            _lin._lib_call("gr_adaptive_lr", self.flat.extra.data_ptr(), self.lr.data_ptr(),
                           C.c_double(alg.desired_kl), C.c_double(1e-5), C.c_double(1e-2), _lin._stream(self.lr))
        _fadam.clip_grad_norm_(self.opt, self.params, alg.max_grad_norm)
        self.opt.step()

    def _capture(self):
        # snapshot (parameters, optimizer state, rate), warm up on a side stream, capture, restore
        snap_p = [p.detach().clone() for p in self.params]
        # (the module's buffers too: the warm-up and captured steps' BatchNorm running statistics and batch counts)
        bufs = list(self.alg.policy.buffers())
        snap_bufs = [b.detach().clone() for b in bufs]
        snap_lr = self.lr.clone()
        snap_acc = self.acc.clone()
        self.flat.bind()  # Adam and the clip read the gradients from these views (static addresses)
        snap_o = {id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in self.opt.state[p].items()}
                  for p in self.params}
        self.perm.copy_(torch.arange(self.perm.numel(), device=self.perm.device))
        self._permute_pack()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        _lin._FORCE_FN = True  # bias gradients by gr_column_sum in the captured step (linear.bias_grad)
        try:
            with torch.cuda.stream(s):
                for _ in range(3):  # (no collective in the warm-up: its results are discarded)
                    self._seg_a()
                    self._seg_b()
            torch.cuda.current_stream().wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            if self.segmented:
                with torch.cuda.graph(self.graph, stream=s):
                    self._seg_a()
                self.graph_b = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph_b, stream=s, pool=self.graph.pool()):
                    self._seg_b()
            elif self.per_step:
                with torch.cuda.graph(self.graph, stream=s):
                    self._seg_a()
                    self._seg_b()
            else:  # an epoch: every mini-batch step, each on its slice of the permutation
                with torch.cuda.graph(self.graph, stream=s):
                    for i in range(self.nmb):
                        lo, hi = i * self.mb, (i + 1) * self.mb
                        self._seg_a((lo, hi) if self.pack_perm is not None else self.perm[lo:hi])
                        self._seg_b()
        finally:
            _lin._FORCE_FN = False
        with torch.no_grad():
            for p, v in zip(self.params, snap_p):
                p.copy_(v)
            for p in self.params:
                for k, v in snap_o[id(p)].items():
                    if torch.is_tensor(v):
                        self.opt.state[p][k].copy_(v)
            for b, v in zip(bufs, snap_bufs):
                b.copy_(v)
            self.lr.copy_(snap_lr)
            self.acc.copy_(snap_acc)

    def _permute_pack(self):
        if self.pack_perm is not None:
            torch.index_select(self.pack, 0, self.perm, out=self.pack_perm)

    def _refresh_sources(self):
        """Before an update's replays: this rollout's samples, packed in place (the graphs read the buffer)."""
        if self.pack is not None:
            self.alg.storage.pack_samples(out=self.pack)

    def _stats(self, num_updates):
        sl, vl = self.acc.tolist()
        return {"value_function": vl / num_updates, "surrogate": sl / num_updates}

    def update(self):
        alg = self.alg
        n = alg.num_mini_batches
        perm = torch.randperm(n * self.mb, device=self.perm.device)  # rollout_storage.py:152-191, drawn first
        self._refresh_sources()
        if self.graph is None:
            had_state = bool(self.opt.state)
            if not had_state:  # Adam's first step creates its state: take it with zero gradients, then undo
                snap_p = [p.detach().clone() for p in self.params]
                self.flat.bind()
                self.flat.flat.zero_()
                self.opt.step()
                with torch.no_grad():
                    for p, v in zip(self.params, snap_p):
                        p.copy_(v)
                    for p in self.params:
                        for k, v in self.opt.state[p].items():
                            if torch.is_tensor(v):
                                v.zero_()
            self._capture()
        self.lr.fill_(float(alg.learning_rate))
        self.acc.zero_()
        if not self.per_step:
            self.perm.copy_(perm)
            self._permute_pack()
        for _ in range(alg.num_learning_epochs):
            if not self.per_step:  # one replay per epoch
                self.graph.replay()
                continue
            for i in range(n):
                self.idx.copy_(perm[i * self.mb:(i + 1) * self.mb])
                self.graph.replay()
                if self.graph_b is not None:
                    self.flat.allreduce_()  # eager, on the current stream's order: gradients + KL mean, one message
                    self.graph_b.replay()
        num_updates = alg.num_learning_epochs * n
        alg.learning_rate = float(self.lr)
        alg.storage.clear()
        return self._stats(num_updates)
