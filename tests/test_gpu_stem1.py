"""The vision stem's first block from the image (gr_stem1_forward / _backward via rsl_rl/fused_bn.py's
stem1_bn_act): Conv2d(1, 16, 3, stride 3) -> BatchNorm2d (batch statistics) -> LeakyReLU / ELU on the patch rows
of VisionActorCritic.stem_gemm, against a float64 evaluation of the same math (patch gather + GEMM + batch norm
+ activation, autograd for the gradients).

Tolerances: y is held to 1e-5 of its scale (fp32 conv, fp64 statistics), the running statistics to 1e-5
relative; the three parameter gradients reduce over up to 1.6 M rows with the BatchNorm backward's cancellation,
so they are held to 1e-4 of their norm.  Repeats must be bit-identical (fixed-order reductions, no atomics)."""
from __future__ import annotations

import os
import sys

import pytest
import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl.fused_bn import stem1_bn_act  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _vision_tables():
    from generalizableracing_amd.rsl_rl.vision_actor_critic import VisionActorCritic

    pol = VisionActorCritic(16 + 72 * 96, 16 + 72 * 96, 4, actor_hidden_dims=[32], critic_hidden_dims=[32])
    a, b, na, nb, _, _, pix16 = pol._patch_index(DEV)
    return 72 * 96, na, nb, pix16


def _synthetic_tables(hw, na, nb, seed):
    g = torch.Generator().manual_seed(seed)
    return hw, na, nb, torch.randint(0, hw, ((na + nb) * 9,), generator=g, dtype=torch.int16).to(DEV)


def _reference(img, pix, na, nb, w, bw, bb, eps, act, gy):
    """float64: rows = every image's table-a cells, then every image's table-b cells (stem_gemm's order)."""
    n = img.shape[0]
    idx = pix.long()
    x64 = img.double()
    pa = x64[:, idx[: na * 9]].reshape(n * na, 9)
    pb = x64[:, idx[na * 9:]].reshape(n * nb, 9)
    w64 = w.detach().double().reshape(16, 9).requires_grad_(True)
    bw64 = bw.detach().double().requires_grad_(True)
    bb64 = bb.detach().double().requires_grad_(True)
    conv = torch.cat([pa, pb]) @ w64.t()
    mean = conv.mean(0)
    var = conv.var(0, unbiased=False)
    z = (conv - mean) / torch.sqrt(var + eps) * bw64 + bb64
    y = act(z)[: n * na]
    (y * gy.double()).sum().backward()
    m = conv.shape[0]
    return y.detach(), mean.detach(), (var * m / max(m - 1, 1)).detach(), w64.grad, bw64.grad, bb64.grad


def _run(img, pix, na, nb, act, seed):
    torch.manual_seed(seed)
    conv = nn.Conv2d(1, 16, 3, 3, bias=False).to(DEV)
    bn = nn.BatchNorm2d(16, momentum=None).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    bn.num_batches_tracked.add_(1)
    y = stem1_bn_act(bn, act, conv.weight, img, pix, na, nb)
    gy = torch.randn_like(y)
    y.backward(gy)
    return conv, bn, y.detach(), gy


def _rel(a, b):
    return float((a.double() - b).norm() / (b.norm() + 1e-30))


CASES = [("vision", 3, "lrelu"), ("vision", 2048, "lrelu"), ("vision", 97, "elu"),
         ("syn", 7, "lrelu"), ("syn1", 1, "elu"), ("syn", 301, "elu")]


@pytest.mark.parametrize("table,nimg,actname", CASES)
def test_stem1_against_float64(table, nimg, actname):
    if table == "vision":
        hw, na, nb, pix = _vision_tables()
    elif table == "syn":
        hw, na, nb, pix = _synthetic_tables(144, 5, 3, nimg)  # na, nb < 16: tiles span images and tables
    else:
        hw, na, nb, pix = _synthetic_tables(9, 1, 0, nimg)  # one image, one cell: a single row
    act = nn.LeakyReLU(0.01) if actname == "lrelu" else nn.ELU()
    g = torch.Generator(device=DEV).manual_seed(nimg)
    obs = torch.rand(nimg, hw + 20, device=DEV, generator=g) * 5.0
    img = obs[:, 4: 4 + hw]  # row stride hw + 20, offset 4: as the rollout's observation rows
    conv, bn, y, gy = _run(img, pix, na, nb, act, nimg)
    y64, mean64, var64, gw64, gbw64, gbb64 = _reference(img, pix, na, nb, conv.weight, bn.weight, bn.bias, bn.eps,
                                                         act, gy)
    assert y.shape == y64.shape
    scale = float(y64.abs().max()) + 1e-6
    assert float((y.double() - y64).abs().max()) <= 1e-5 * scale
    # momentum None, num_batches_tracked 1: the running statistics are this batch's
    assert float(((bn.running_mean.double() - mean64).abs() / mean64.abs().clamp_min(1e-3)).max()) < 1e-5
    if var64.numel() and nimg * (na + nb) > 1:
        assert float(((bn.running_var.double() - var64).abs() / var64.abs().clamp_min(1e-3)).max()) < 1e-5
    assert _rel(conv.weight.grad.reshape(16, 9), gw64) < 1e-4, _rel(conv.weight.grad.reshape(16, 9), gw64)
    assert _rel(bn.weight.grad, gbw64) < 1e-4
    assert _rel(bn.bias.grad, gbb64) < 1e-4


def test_stem1_deterministic():
    hw, na, nb, pix = _vision_tables()
    img = torch.rand(512, hw, device=DEV) * 5.0
    runs = []
    for _ in range(2):
        conv, bn, y, _ = _run(img, pix, na, nb, nn.LeakyReLU(0.01), 5)
        runs.append((y, conv.weight.grad, bn.weight.grad, bn.bias.grad, bn.running_mean, bn.running_var))
    for u, v in zip(*runs):
        assert torch.equal(u, v)

