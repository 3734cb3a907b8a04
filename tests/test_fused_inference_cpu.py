"""Fused policy inference (gr_policy.hip) on CPU: the weight packing and the kernel's fragment dataflow.

The GPU kernel computes every layer transposed with v_mfma_f32_16x16x32_bf16 and feeds each layer's
accumulator tiles to the next layer as B fragments with a permuted k order; the host packs W2 / W3 in
that order (rsl_rl/fused_inference.py).  This test replays that dataflow lane by lane in numpy (the
documented MFMA operand / result maps) on the packed tensors and compares it with the fp32 torch
module, so a packing or permutation error fails here, before any GPU run.  The -m gpu twin compares
the kernel itself (tests/test_gpu_fused_inference.py)."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl import ActorCritic  # noqa: E402
from generalizableracing_amd.rsl_rl.fused_inference import mlp_layers, pack_w1, pack_w2, pack_w3  # noqa: E402


def bf16(x):
    return torch.as_tensor(np.asarray(x, np.float32)).to(torch.bfloat16).float().numpy().astype(np.float64)


def mfma_16x16x32(a, b):
    """a, b: [64, 8] lane fragments (A[l & 15][8 (l >> 4) + j], B[8 (l >> 4) + j][l & 15]) -> [64, 4] result
    (lane l, reg r = D[4 (l >> 4) + r][l & 15])."""
    A = np.zeros((16, 32))
    B = np.zeros((32, 16))
    for lane in range(64):
        for j in range(8):
            A[lane & 15, 8 * (lane >> 4) + j] = a[lane, j]
            B[8 * (lane >> 4) + j, lane & 15] = b[lane, j]
    D = A @ B
    out = np.zeros((64, 4))
    for lane in range(64):
        for r in range(4):
            out[lane, r] = D[4 * (lane >> 4) + r, lane & 15]
    return out


def act(x, kind):
    return np.where(x > 0, x, 0.01 * x) if kind == 0 else np.where(x > 0, x, np.expm1(x))


def emulate(lin, code, X):
    """the kernel's dataflow for one column tile of 16 envs (X [16, D])"""
    H = lin[0].out_features
    T, S = H // 16, H // 32
    w1 = pack_w1(lin[0].weight).float().numpy().astype(np.float64)
    w2 = pack_w2(lin[1].weight).float().numpy().astype(np.float64)
    w3 = pack_w3(lin[2].weight).float().numpy().astype(np.float64)
    b1, b2, b3 = (l.bias.detach().double().numpy() for l in lin)
    D = X.shape[1]
    xb = np.zeros((64, 8))
    for lane in range(64):
        for j in range(8):
            k = 8 * (lane >> 4) + j
            xb[lane, j] = X[lane & 15, k] if k < D else 0.0
    xb = bf16(xb)
    lanes = np.arange(64)

    def bias_act(y, b, row0):
        rows = row0 + 4 * (lanes >> 4)[:, None] + np.arange(4)[None, :]
        return act(y + b[rows], code)

    h1 = np.zeros((S, 64, 8))
    for t in range(0, T, 2):
        y0 = bias_act(mfma_16x16x32(w1[t], xb), b1, 16 * t)
        y1 = bias_act(mfma_16x16x32(w1[t + 1], xb), b1, 16 * t + 16)
        h1[t // 2] = bf16(np.concatenate([y0, y1], axis=1))
    h2 = np.zeros((S, 64, 8))
    for t in range(0, T, 2):
        acc0 = sum(mfma_16x16x32(w2[t, s], h1[s]) for s in range(S))
        acc1 = sum(mfma_16x16x32(w2[t + 1, s], h1[s]) for s in range(S))
        h2[t // 2] = bf16(np.concatenate([bias_act(acc0, b2, 16 * t), bias_act(acc1, b2, 16 * t + 16)], axis=1))
    o = sum(mfma_16x16x32(w3[s], h2[s]) for s in range(S))
    out = lin[2].out_features
    return np.stack([o[lane, :out] + b3 for lane in range(16)])  # [16 envs, out]


@pytest.mark.parametrize("hidden,activation", [(256, "lrelu"), (128, "elu")])
def test_fragment_dataflow_matches_torch(hidden, activation):
    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [hidden, hidden], [hidden, hidden], activation)
    X = torch.randn(16, 16) * 2.0
    for seq, n_out in ((pol.actor, 4), (pol.critic, 1)):
        lin, code = mlp_layers(seq)
        want = seq(X).detach().double().numpy()
        got = emulate(lin, code, X.numpy().astype(np.float64))
        assert got.shape == (16, n_out)
        scale = np.abs(want).max() + 1e-3
        assert np.abs(got - want).max() < 2e-2 * scale, (np.abs(got - want).max(), scale)


def test_packing_is_a_permutation():
    torch.manual_seed(1)
    H = 256
    w = torch.randn(H, H)
    p = pack_w2(w).float()
    # every (row, k) of W2 appears exactly once, with the bf16 value of that entry
    assert p.numel() == H * H
    assert torch.equal(torch.sort(p.flatten()).values, torch.sort(w.to(torch.bfloat16).float().flatten()).values)
    w3 = torch.randn(4, H)
    p3 = pack_w3(w3).float()
    assert (p3 != 0).sum() == 4 * H
    w1 = torch.randn(H, 16)
    p1 = pack_w1(w1).float()
    assert (p1 != 0).sum() == H * 16


def test_unsupported_policies_rejected():
    with pytest.raises(ValueError):
        mlp_layers(ActorCritic(16, 16, 4, [256, 256, 256], [256, 256, 256], "lrelu").actor)
    with pytest.raises(ValueError):
        mlp_layers(ActorCritic(16, 16, 4, [64, 64], [64, 64], "lrelu").actor)
    with pytest.raises(ValueError):
        mlp_layers(ActorCritic(16, 16, 4, [256, 256], [256, 256], "tanh").actor)


def test_fused_rollout_has_no_cpu_path():
    """algorithm.fused_rollout_inference is HIP-only: on a CPU device PPO refuses it at storage init."""
    from generalizableracing_amd.rsl_rl.ppo import PPO

    alg = PPO(ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu"), device="cpu", fused_rollout_inference=True)
    with pytest.raises(RuntimeError):
        alg.init_storage("rl", 8, 4, [16], [16], [4])
