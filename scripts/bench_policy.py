"""Fused MFMA policy inference (gr_policy_forward) alone: per-launch us, TFLOP/s and the error vs the fp32
module, at 65 536 envs.  GR_LIB_PATH selects a timing variant build (scripts/build_variants.sh).

    python scripts/bench_policy.py [--envs 65536] [--hidden 256] [--precision bf16|fp32]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl import ActorCritic  # noqa: E402
from generalizableracing_amd.rsl_rl.fused_inference import FusedPolicyInference  # noqa: E402


def run(n=65536, hidden=256, reps=64, device="cuda:0", precision="bf16"):
    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [hidden, hidden], [hidden, hidden], "lrelu").to(device)
    fused = FusedPolicyInference(pol, n, device, precision=precision)
    obs = torch.randn(n, 16, device=device)
    for _ in range(4):
        fused.act(obs, obs)
    torch.cuda.synchronize()
    with torch.no_grad():
        m_ref, v_ref = pol.actor(obs), pol.critic(obs)
    err = max(float((fused.action_mean - m_ref).abs().max()) / (float(m_ref.abs().max()) + 1e-3),
              float((fused.values - v_ref).abs().max()) / (float(v_ref.abs().max()) + 1e-3))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fused.act(obs, obs)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    flops = 2 * n * 2 * (16 * hidden + hidden * hidden + hidden * 4)
    # the torch fp32 equivalent (actor + critic forward + sampling), for reference
    with torch.no_grad():
        for _ in range(3):
            pol.act(obs), pol.evaluate(obs)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(8):
            a = pol.act(obs)
            pol.evaluate(obs)
            pol.get_actions_log_prob(a)
        e1.record()
        e1.synchronize()
    torch_us = e0.elapsed_time(e1) * 1e3 / 8
    peak = 2.5e15 if precision == "bf16" else 157.3e12  # dense MFMA peak of the operand type
    return {"lib": os.environ.get("GR_LIB_PATH", "tree"), "precision": precision, "envs": n, "hidden": hidden,
            "kernel_us": us, "TFLOPs": flops / (us * 1e-6) / 1e12, "frac_of_mfma_peak": flops / (us * 1e-6) / peak,
            "max_rel_err_vs_fp32": err, "torch_fp32_us": torch_us}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    a = ap.parse_args()
    print(json.dumps(run(a.envs, a.hidden, precision=a.precision)))
