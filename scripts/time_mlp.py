"""Time the update's MLP forward + backward for actor and critic at the update's mini-batch sizes: the whole-network
kernels (linear.fused_mlps: gr_mlp_forward / gr_mlp_backward) against the round-3 per-layer path (MLP modules:
fused first layer / head around hipBLASLt).  HIP events around 20 repetitions on the current stream; prints one JSON
line per (rows, path).  Run it under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python scripts/time_mlp.py [--rows 24576 393216] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl import linear as lin  # noqa: E402
from generalizableracing_amd.rsl_rl.actor_critic import ActorCritic  # noqa: E402

PEAK = 157.3


def flops(rows, h=256, d=16):
    """Useful flops of forward + backward (weight and input gradients below the first layer) of both networks."""
    fwd = 2 * rows * ((d * h + h * h + h * 4) + (d * h + h * h + h))
    wgrad = fwd
    igrad = 2 * rows * ((h * h + h * 4) + (h * h + h))
    return fwd + wgrad + igrad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[24576, 393216])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--mask", action="store_true", help="the backward reads h1's sign bits (mlp_bwd256h), not the rows")
    ap.add_argument("--fused-only", action="store_true")
    a = ap.parse_args()
    lin._H1_MASKS = a.mask
    dev = "cuda:0"
    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(dev)
    nets = [pol.actor, pol.critic]
    params = [p for n in nets for p in n.parameters()]
    for rows in a.rows:
        buf = torch.randn(rows, 48, device=dev)
        xa, xc = buf[:, :16], buf[:, 16:32]
        ga, gc = torch.randn(rows, 4, device=dev), torch.randn(rows, 1, device=dev)
        for path in (("fused_mlp",) if a.fused_only else ("fused_mlp", "per_layer")):
            def step():
                if path == "fused_mlp":
                    ya, yc = lin.fused_mlps(nets, [xa, xc])
                else:
                    ya, yc = pol.actor(xa), pol.critic(xc)
                torch.autograd.grad((ya * ga).sum() + (yc * gc).sum(), params)

            lin._FORCE_FN = True
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                step()
            e1.record()
            e1.synchronize()
            lin._FORCE_FN = False
            us = e0.elapsed_time(e1) * 1e3 / a.reps
            tfs = flops(rows) / (us * 1e-6) / 1e12
            print(json.dumps({"rows": rows, "path": path, "us_fwd_bwd": us, "TFLOPs": tfs, "frac_fp32_peak": tfs / PEAK}),
                  flush=True)


if __name__ == "__main__":
    main()
