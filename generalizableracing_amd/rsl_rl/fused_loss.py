"""The PPO losses of a mini-batch as one device op (gr_ppo_loss_forward / gr_ppo_loss_backward, gr_update.hip).

PPO.update (standalone/rsl_rl/ext/algorithms/ppo.py:103-190) evaluates, per mini-batch, the Gaussian log prob of
the stored actions under the new policy (rsl_rl ActorCritic.get_actions_log_prob), the adaptive-rate KL
(ppo.py:133-150), the clipped surrogate and the clipped value loss (ppo.py:152-169): in torch some 50 launches of
[rows] / [rows, 4] tensors forward and as many backward, each a few microseconds, together ~0.45 ms of every
mini-batch step at 65 536 envs (profiles/round03_update65536_graphed_kernel_stats.csv).  Here: one launch and a
fixed-order reduction each way, graph-capturable, on the row-strided columns of the packed mini-batch.  The
arithmetic follows the torch ops it replaces (fp32; ties of torch.max split the gradient, clamp passes it on its
closed interval); the entropy term depends on the std only and stays in torch.
"""
from __future__ import annotations

import ctypes as C
import math

import torch


class GrPpoLossArgs(C.Structure):
    """Mirror of gr_ppo_loss_args (include/gr.h)."""
    _fields_ = [("rows", C.c_int64), ("k", C.c_int32), ("clipped_value", C.c_int32), ("clip", C.c_float)] + [
        (n, C.c_void_p) for n in ("mu", "std", "value", "act", "logp_old", "adv", "value_old", "ret", "mu_old",
                                  "sig_old")] + [
        (n, C.c_int64) for n in ("ld_mu", "ld_value", "ld_act", "ld_logp_old", "ld_adv", "ld_value_old", "ld_ret",
                                 "ld_mu_old", "ld_sig_old")]


def _ld(t: torch.Tensor) -> int:
    if t.dim() == 2 and t.stride(1) != 1:
        raise ValueError("fused PPO loss: rows must have unit column stride")
    return int(t.stride(0))


def _args(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, clip, clipped_value):
    a = GrPpoLossArgs()
    a.rows, a.k = mu.shape[0], mu.shape[1]
    a.clipped_value, a.clip = int(bool(clipped_value)), float(clip)
    for name, t in (("mu", mu), ("std", std), ("value", value), ("act", act), ("logp_old", logp_old), ("adv", adv),
                    ("value_old", value_old), ("ret", ret), ("mu_old", mu_old), ("sig_old", sig_old)):
        setattr(a, name, t.data_ptr())
        if name != "std":
            setattr(a, "ld_" + name, _ld(t))
    return a


def _call(name, *args):
    from .. import _abi

    rc = getattr(_abi.load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (status {rc})")


class _PPOLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, clip, clipped_value):
        from .. import _abi

        std = std.contiguous()
        a = _args(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, clip, clipped_value)
        rows = mu.shape[0]
        part = torch.empty(_abi.load().gr_ppo_loss_partials(rows), device=mu.device, dtype=torch.float32)
        sums = torch.empty(3, device=mu.device, dtype=torch.float32)
        stream = _abi.raw_stream(mu.device)
        _call("gr_ppo_loss_forward", C.addressof(a), part.data_ptr(), sums.data_ptr(), stream)
        ctx.save_for_backward(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old)
        ctx.clip, ctx.clipped_value = clip, clipped_value
        out = sums / rows  # the means (torch's mean: sum / rows)
        kl = out[2].clone()
        ctx.mark_non_differentiable(kl)
        return out[0].clone(), out[1].clone(), kl

    @staticmethod
    def backward(ctx, g_surr, g_value, g_kl):
        from .. import _abi

        mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old = ctx.saved_tensors
        a = _args(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, ctx.clip, ctx.clipped_value)
        rows, k = mu.shape
        dev = mu.device
        zero = torch.zeros((), device=dev)
        g = torch.stack([g_surr if g_surr is not None else zero, g_value if g_value is not None else zero]).float()
        dmu = torch.empty(rows, k, device=dev, dtype=torch.float32)
        dvalue = torch.empty(rows, device=dev, dtype=torch.float32)
        part = torch.empty(_abi.load().gr_ppo_loss_partials(rows), device=dev, dtype=torch.float32)
        dstd = torch.empty(k, device=dev, dtype=torch.float32)
        stream = _abi.raw_stream(dev)
        _call("gr_ppo_loss_backward", C.addressof(a), g.data_ptr(), dmu.data_ptr(), dvalue.data_ptr(), part.data_ptr(),
              dstd.data_ptr(), stream)
        return (dmu, dstd, dvalue.view(value.shape), None, None, None, None, None, None, None, None, None)


class _PPOLossCombinedFn(torch.autograd.Function):
    """The combined loss surrogate + value_coef * value (ppo.py:171-172) and its gradient, finished on the device
    (gr_ppo_loss_forward_loss / gr_ppo_loss_backward_loss): no torch glue between the losses and autograd (the
    means' division, the clones, the coefficient's multiply and add, the gradient stack).  Outputs: the loss and
    the non-differentiable [surrogate, value, KL] means; `acc` [2] (optional) accumulates the surrogate and value
    means, `kl_out` [1] (optional) receives the KL mean."""

    @staticmethod
    def forward(ctx, mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, clip, clipped_value,
                value_coef, acc, kl_out, seed):
        from .. import _abi

        std = std.contiguous()
        a = _args(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, clip, clipped_value)
        rows, k = mu.shape
        dev = mu.device
        npart = _abi.load().gr_ppo_loss_partials(rows)
        part = torch.empty(npart, device=dev, dtype=torch.float32)
        sums = torch.empty(3, device=dev, dtype=torch.float32)
        loss = torch.empty((), device=dev, dtype=torch.float32)
        stats = torch.empty(3, device=dev, dtype=torch.float32)
        stream = _abi.raw_stream(dev)
        accp, klp = (acc.data_ptr() if acc is not None else None), (kl_out.data_ptr() if kl_out is not None else None)
        ctx.pre = None
        if seed is not None:
            # the backward's per-row gradients in the forward's pass (gr_ppo_loss_forward_backward), for the
            # upstream gradient the caller will seed autograd with (the graph-captured step's persistent one)
            dmu = torch.empty(rows, k, device=dev, dtype=torch.float32)
            dvalue = torch.empty(rows, device=dev, dtype=torch.float32)
            dpart = torch.empty(npart, device=dev, dtype=torch.float32)
            dstd = _std_sink(std, k)
            _call("gr_ppo_loss_forward_backward", C.addressof(a), seed.data_ptr(), C.c_float(value_coef),
                  part.data_ptr(), sums.data_ptr(), loss.data_ptr(), stats.data_ptr(), accp, klp, dmu.data_ptr(),
                  dvalue.data_ptr(), dpart.data_ptr(), dstd.data_ptr(), stream)
            ctx.pre = (seed.data_ptr(), dmu, dstd, dvalue.view(value.shape))
        else:
            _call("gr_ppo_loss_forward_loss", C.addressof(a), part.data_ptr(), sums.data_ptr(), C.c_float(value_coef),
                  loss.data_ptr(), stats.data_ptr(), accp, klp, stream)
        ctx.save_for_backward(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old)
        ctx.clip, ctx.clipped_value, ctx.value_coef = clip, clipped_value, float(value_coef)
        ctx.mark_non_differentiable(stats)
        ctx.set_materialize_grads(False)  # (no zero gradient filled in for the stats)
        return loss, stats

    @staticmethod
    def backward(ctx, g_loss, g_stats):
        from .. import _abi

        if g_loss is None:
            return (None,) * 16
        if ctx.pre is not None and g_loss.data_ptr() == ctx.pre[0]:  # computed in the forward, for this seed
            return ctx.pre[1:] + (None,) * 13
        mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old = ctx.saved_tensors
        a = _args(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old, ctx.clip, ctx.clipped_value)
        rows, k = mu.shape
        dev = mu.device
        g = g_loss.float().contiguous()
        dmu = torch.empty(rows, k, device=dev, dtype=torch.float32)
        dvalue = torch.empty(rows, device=dev, dtype=torch.float32)
        part = torch.empty(_abi.load().gr_ppo_loss_partials(rows), device=dev, dtype=torch.float32)
        dstd = _std_sink(std, k)
        _call("gr_ppo_loss_backward_loss", C.addressof(a), g.data_ptr(), C.c_float(ctx.value_coef), dmu.data_ptr(),
              dvalue.data_ptr(), part.data_ptr(), dstd.data_ptr(), _abi.raw_stream(dev))
        return (dmu, dstd, dvalue.view(value.shape)) + (None,) * 13


def _std_sink(std, k):
    """The std gradient's buffer: its view in the graph-captured step's flat gradient buffer when the std is the
    parameter itself (linear._GRAD_SINK; the step then copies no gradient), else a new tensor."""
    from . import linear as _lin

    sink = _lin._GRAD_SINK.get(id(std)) if _lin._GRAD_SINK is not None else None
    if sink is not None and sink.dtype == torch.float32 and sink.is_contiguous() and sink.numel() == k:
        return sink.view(k)
    return torch.empty(k, device=std.device, dtype=torch.float32)


def _policy_std(pol):
    """The policy's action std [k] as a differentiable function of its parameter (ActorCritic._std without the
    expand over the batch, whose backward would be a reduction)."""
    return pol.std if pol.noise_std_type == "scalar" else torch.exp(pol.log_std)


def policy_outputs(alg, obs, critic_obs):
    """(action mean, value) of the mini-batch: both MLPs through the whole-network MFMA kernels when they cover
    them (linear.fused_mlps: one launch per direction for actor and critic), else module by module."""
    from . import linear as _lin

    pol = alg.policy
    nets, xs = [pol.actor, pol.critic], [obs, critic_obs]
    if getattr(alg, "fused_mlp", False) and _lin.networks_fusable(nets, xs):
        return _lin.fused_mlps(nets, xs)
    return pol.actor(obs), pol.critic(critic_obs)


def ppo_loss(alg, obs, critic_obs, act, value_old, adv, ret, logp_old, mu_old, sig_old, acc=None, kl_out=None,
             seed=None):
    """(loss, [surrogate, value, KL] means) of one mini-batch: loss = surrogate + value_loss_coef * value
    (- entropy_coef * entropy) as in ppo.py:171-172, differentiable; the same values as ppo_losses.  seed: the
    device tensor autograd will be seeded with (the loss's gradient), when known now and the loss is the root: the
    losses' backward then runs inside the forward's pass (gr_ppo_loss_forward_backward)."""
    pol = alg.policy
    mu, value = policy_outputs(alg, obs, critic_obs)
    std = _policy_std(pol)
    if alg.entropy_coef != 0.0:  # (the loss is not the root then: its gradient is not the seed)
        seed = None
    loss, stats = _PPOLossCombinedFn.apply(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old,
                                           float(alg.clip_param), bool(alg.use_clipped_value_loss),
                                           float(alg.value_loss_coef), acc, kl_out, seed)
    if alg.entropy_coef != 0.0:  # Normal.entropy summed over the actions: the same for every sample
        ent = (0.5 + 0.5 * math.log(2.0 * math.pi) + torch.log(std)).sum()
        loss = loss - alg.entropy_coef * ent
    return loss, stats


def fused_losses_ok(policy, obs: torch.Tensor) -> bool:
    """rsl_rl's ActorCritic (state-independent std) with <= 8 actions, CUDA fp32 observations, outside autocast."""
    from .actor_critic import ActorCritic

    return (type(policy) is ActorCritic and obs.is_cuda and obs.dtype == torch.float32
            and policy.actor[-1].out_features <= 8 and not torch.is_autocast_enabled("cuda"))


def ppo_losses(alg, obs, critic_obs, act, value_old, adv, ret, logp_old, mu_old, sig_old):
    """(surrogate_loss, value_loss, entropy_mean, kl_mean, mu, sigma) of one mini-batch, the losses differentiable:
    the policy's actor and critic forward (the fused MLPs on tall batches), then gr_ppo_loss_*.  The same values
    as PPO.update's policy.act / get_actions_log_prob / evaluate / _ppo_losses / _adapt_learning_rate (ppo.py
    :103-169), without the unused action sample."""
    pol = alg.policy
    mu, value = policy_outputs(alg, obs, critic_obs)
    std = pol._std(mu[:1])[0]  # [k]: the scalar or exp(log) std, differentiable
    surr, vloss, kl = _PPOLossFn.apply(mu, std, value, act, logp_old, adv, value_old, ret, mu_old, sig_old,
                                       float(alg.clip_param), bool(alg.use_clipped_value_loss))
    ent = None
    if alg.entropy_coef != 0.0:  # Normal.entropy summed over the actions: the same for every sample
        ent = (0.5 + 0.5 * math.log(2.0 * math.pi) + torch.log(std)).sum()
    return surr, vloss, ent, kl, mu, std
