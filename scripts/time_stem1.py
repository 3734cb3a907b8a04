"""Time the vision stem's first block (gr_stem1_forward / _backward) at one PPO mini-batch of images (4 096 envs x
24 steps / 4 mini-batches = 24 576 images of 72 x 96): HIP events around `reps` forward and backward calls.
GR_LIB_PATH selects a variant build (scripts/build_patched.py, e.g. variants/stem1_valu: the per-row VALU kernels).

    python scripts/time_stem1.py [--nimg 24576] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl.fused_bn import stem1_bn_act  # noqa: E402
from generalizableracing_amd.rsl_rl.vision_actor_critic import VisionActorCritic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nimg", type=int, default=24576)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda:0"
    pol = VisionActorCritic(16 + 72 * 96, 16 + 72 * 96, 4, actor_hidden_dims=[32], critic_hidden_dims=[32])
    _, _, na, nb, _, _, pix = pol._patch_index(dev)
    torch.manual_seed(0)
    obs = torch.rand(a.nimg, 16 + 72 * 96, device=dev) * 5.0
    img = obs[:, 16:]
    conv = nn.Conv2d(1, 16, 3, 3, bias=False).to(dev)
    bn = nn.BatchNorm2d(16).to(dev)
    act = nn.LeakyReLU(0.01)
    gy = torch.randn(a.nimg * na, 16, device=dev)
    for _ in range(3):
        y = stem1_bn_act(bn, act, conv.weight, img, pix, na, nb)
        y.backward(gy)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd = bwd = 0.0
    for _ in range(a.reps):
        ev[0].record()
        y = stem1_bn_act(bn, act, conv.weight, img, pix, na, nb)
        ev[1].record()
        y.backward(gy)
        ev[2].record()
        ev[2].synchronize()
        fwd += ev[0].elapsed_time(ev[1])
        bwd += ev[1].elapsed_time(ev[2])
    rows = a.nimg * (na + nb)
    print(json.dumps({"lib": os.environ.get("GR_LIB_PATH", "libgr.so"), "nimg": a.nimg, "rows": rows,
                      "forward_us": fwd * 1e3 / a.reps, "backward_us": bwd * 1e3 / a.reps,
                      "image_bytes": a.nimg * 72 * 96 * 4, "y_bytes": a.nimg * na * 16 * 4,
                      "gw_sum": float(conv.weight.grad.double().abs().sum())}))


if __name__ == "__main__":
    main()
