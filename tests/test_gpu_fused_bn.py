"""Fused training-mode BatchNorm + activation (gr_bn_act_forward / _backward, rsl_rl/fused_bn.py) against
torch's batch_norm + activation, on the GPU.

Tolerance: the batch statistics are fp64 sums over up to millions of rows (torch: fp32 Welford), so the
outputs agree to ~1e-6 of their scale; the test holds y to 1e-5 and the running statistics to 1e-5
relative.  Gradients: LeakyReLU's derivative jumps at 0, and a pre-activation within rounding of 0 may fall
on different sides here and in torch (torch rounds (x - mean) * invstd * w + b with its own contraction),
so gx is held to 1e-4 of its scale on all but at most 1e-6 of its elements (each such element is off by
at most |gy| (1 - slope) invstd |w|), and gw / gb (sums over M rows, which such an element moves by O(1)
against a scale of O(sqrt M)) to 2e-3."""
from __future__ import annotations

import copy
import os
import sys

import pytest
import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl.fused_bn import batch_norm_act, reference_batch_norm_act  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _close(got, want, tol):
    scale = float(want.abs().max()) + 1e-6
    err = float((got - want).abs().max())
    assert err <= tol * scale, (err, scale)


@pytest.mark.parametrize("m,c,act", [(2, 16, "lrelu"), (1000, 16, "lrelu"), (4097, 32, "elu"), (300000, 64, "lrelu"),
                                     (3 * 10**6, 16, "lrelu"), (77, 8, "elu"), (5, 4, "lrelu")])
def test_matches_torch(m, c, act):
    torch.manual_seed(m + c)
    bn = nn.BatchNorm2d(c).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    a = nn.LeakyReLU(0.01) if act == "lrelu" else nn.ELU()
    ref_bn = copy.deepcopy(bn)
    x = (3.0 + 2.0 * torch.randn(m, c, device=DEV)).requires_grad_(True)  # offset mean: the shifted sums
    xr = x.detach().clone().requires_grad_(True)
    y = batch_norm_act(bn, a, x)
    yr = reference_batch_norm_act(ref_bn, a, xr)
    _close(y, yr, 1e-5)
    for got, want in ((bn.running_mean, ref_bn.running_mean), (bn.running_var, ref_bn.running_var)):
        assert float(((got - want).abs() / want.abs().clamp_min(1e-3)).max()) < 1e-5
    gy = torch.randn_like(y)
    y.backward(gy)
    yr.backward(gy)
    scale = float(xr.grad.abs().max()) + 1e-6
    off = (x.grad - xr.grad).abs() > 1e-4 * scale
    assert int(off.sum()) <= max(2, int(1e-6 * off.numel())), int(off.sum())
    _close(bn.weight.grad, ref_bn.weight.grad, 2e-3)
    _close(bn.bias.grad, ref_bn.bias.grad, 2e-3)


def test_deterministic():
    torch.manual_seed(1)
    bn = nn.BatchNorm2d(32).to(DEV)
    a = nn.LeakyReLU(0.01)
    x = torch.randn(500000, 32, device=DEV)
    outs = []
    for _ in range(2):
        xi = x.clone().requires_grad_(True)
        b = copy.deepcopy(bn)
        y = batch_norm_act(b, a, xi)
        y.backward(torch.ones_like(y))
        outs.append((y.detach(), xi.grad, b.weight.grad))
    for u, v in zip(*outs):
        assert torch.equal(u, v)


def test_vision_policy_fused_vs_torch():
    """VisionActorCritic features and parameter gradients with the fused op == with torch's ops."""
    from generalizableracing_amd.rsl_rl.vision_actor_critic import VisionActorCritic

    torch.manual_seed(2)
    n = 256
    pol = VisionActorCritic(16 + 72 * 96, 16 + 72 * 96, 4, actor_hidden_dims=[128, 128], critic_hidden_dims=[128, 128],
                            activation="lrelu").to(DEV)
    ref = copy.deepcopy(pol)
    ref.fused_bn = False
    obs = torch.rand(n, 16 + 72 * 96, device=DEV) * 5.0
    f = pol.features(obs)
    fr = ref.features(obs)
    _close(f, fr, 1e-4)
    (f.square().sum() + pol.actor(f).sum()).backward()
    (fr.square().sum() + ref.actor(fr).sum()).backward()
    for (name, p), (_, q) in zip(pol.named_parameters(), ref.named_parameters()):
        if p.grad is None:
            assert q.grad is None, name
            continue
        _close(p.grad, q.grad, 2e-3)
    for (name, b), (_, c) in zip(pol.named_buffers(), ref.named_buffers()):
        if b.dtype.is_floating_point:
            assert float((b - c).abs().max()) <= 1e-5 * (float(c.abs().max()) + 1e-6), name
        else:
            assert torch.equal(b, c), name
