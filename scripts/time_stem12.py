"""Time the vision stem's first block + conv2 (fused_bn.stem12_bn_act_conv: gr_stem1_forward, the conv2 GEMM, and the
fused backward gr_stem12_backward) at one PPO mini-batch of images (24 576 of 72 x 96): HIP events around `reps`
forward + backward calls.  Run under rocprofv3 for the per-kernel split (or --pmc counters).

    python scripts/time_stem12.py [--nimg 24576] [--reps 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl.fused_bn import stem12_bn_act_conv  # noqa: E402
from generalizableracing_amd.rsl_rl.vision_actor_critic import VisionActorCritic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nimg", type=int, default=24576)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stored-y1", action="store_true", help="the round-5 backward (y1 stored, conv2's weight gradient "
                    "by gr_patch_wgrad) instead of gr_stem12_backward_w2")
    a = ap.parse_args()
    if a.stored_y1:
        from generalizableracing_amd.rsl_rl import fused_bn

        fused_bn.STEM12_W2 = False
    dev = "cuda:0"
    pol = VisionActorCritic(16 + 72 * 96, 16 + 72 * 96, 4, actor_hidden_dims=[32], critic_hidden_dims=[32])
    _, _, na, nb, _, n2, pix = pol._patch_index(dev)
    torch.manual_seed(0)
    obs = torch.rand(a.nimg, 16 + 72 * 96, device=dev) * 5.0
    img = obs[:, 16:]
    conv = nn.Conv2d(1, 16, 3, 3, bias=False).to(dev)
    conv2 = nn.Conv2d(16, 32, 3, 3, bias=False).to(dev)
    bn = nn.BatchNorm2d(16).to(dev)
    act = nn.LeakyReLU(0.01)
    gz2 = torch.randn(a.nimg * n2, 32, device=dev)

    def step():
        w2 = conv2.weight.permute(0, 2, 3, 1).reshape(32, 144)
        z2 = stem12_bn_act_conv(bn, act, conv.weight, w2, img, pix, na, nb)
        z2.backward(gz2)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"nimg": a.nimg, "reps": a.reps, "stored_y1": a.stored_y1, "ms_fwd_bwd": e0.elapsed_time(e1) / a.reps}))


if __name__ == "__main__":
    main()
