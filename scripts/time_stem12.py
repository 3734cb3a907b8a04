"""Time the vision stem's first block + conv2 (fused_bn.stem12_bn_act_conv: the statistics pass + stem12g_kernel forward,
gr_stem12_backward_w2's stem12w_kernel backward) at one PPO mini-batch of images (24 576 of 72 x 96): HIP events around
`reps` forward + backward calls.  Run under rocprofv3 for the per-kernel split (or --pmc counters).

    python scripts/time_stem12.py [--nimg 24576] [--reps 20] [--stored-y1] [--no-moments] [--roofline]

`roofline(nimg)` (bench.py's vision leg) times the forward and the backward separately and states each against its
bound from the algorithmic bytes and flops per image:
  forward  = statistics pass (image read, conv1 of all 768 cells) + stem12g (image read, conv1 of the 720 table-a
             cells, BN + act, conv2; z2 written);
  backward = stem12w (image + gz2 read; conv1 recomputed, conv2's input and weight gradients, conv1's weight-gradient
             sums: with the forward's pixel moments only A1 = sum gz x pixels) + its two small fixed-order reductions.
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

HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFS = 157.3
H, W, C1, C2 = 72, 96, 16, 32
CELLS, CELLS_A, PATCHES = 768, 720, 80  # conv1 outputs per image; those under a conv2 patch; conv2 outputs
IMG_BYTES = H * W * 4
Z2_BYTES = PATCHES * C2 * 4
CONV1 = 2 * C1 * 9            # flops per conv1 output cell
CONV2 = 2 * PATCHES * C2 * C1 * 9  # flops of conv2 (forward; each backward product the same)
# per image: (bytes, useful flops)
STATS = (IMG_BYTES, CELLS * CONV1)
STEM12G = (IMG_BYTES + Z2_BYTES, CELLS_A * CONV1 + CONV2)
STEM12W = (IMG_BYTES + Z2_BYTES, CELLS * CONV1 + 2 * CONV2 + CELLS_A * CONV1 + CELLS * CONV1)
# with the forward's pixel moments (fused_bn.STEM12_MOMENTS): conv1 recomputed on the table-a cells, conv2's two
# products, A1; A2 / A3 come from the moments
STEM12W_MOM = (IMG_BYTES + Z2_BYTES, CELLS_A * CONV1 + 2 * CONV2 + CELLS_A * CONV1)


def _setup(nimg, dev="cuda:0"):
    pol = VisionActorCritic(16 + H * W, 16 + H * W, 4, actor_hidden_dims=[32], critic_hidden_dims=[32])
    _, _, na, nb, _, n2, pix = pol._patch_index(dev)
    torch.manual_seed(0)
    obs = torch.rand(nimg, 16 + H * W, device=dev) * 5.0
    conv = nn.Conv2d(1, C1, 3, 3, bias=False).to(dev)
    conv2 = nn.Conv2d(C1, C2, 3, 3, bias=False).to(dev)
    bn = nn.BatchNorm2d(C1).to(dev)
    act = nn.LeakyReLU(0.01)
    gz2 = torch.randn(nimg * n2, C2, device=dev)

    def forward():
        w2 = conv2.weight.permute(0, 2, 3, 1).reshape(C2, 9 * C1)
        return stem12_bn_act_conv(bn, act, conv.weight, w2, obs[:, 16:], pix, na, nb)

    return forward, gz2


def _bound(per_img, nimg, us):
    by, fl = per_img[0] * nimg, per_img[1] * nimg
    t_hbm, t_mfma = by / (HBM_PEAK_GBS * 1e9) * 1e6, fl / (FP32_MFMA_PEAK_TFS * 1e12) * 1e6
    bound = "mfma" if t_mfma >= t_hbm else "hbm"
    return {"us": us, "bytes": by, "flops": fl, "achieved_GBps": by / (us * 1e-6) / 1e9,
            "achieved_TFLOPs": fl / (us * 1e-6) / 1e12, "bound": bound,
            "frac": (t_mfma if bound == "mfma" else t_hbm) / us}


def roofline(nimg=24576, reps=10):
    """Forward and backward of the stem's first block + conv2 at `nimg` images, each timed with HIP events over `reps`
    calls, against the HBM / fp32-MFMA bound of its algorithmic bytes and flops."""
    forward, gz2 = _setup(nimg)
    for _ in range(2):
        forward().backward(gz2)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps + 1)]
    ev[0].record()
    for r in range(reps):
        z2 = forward()
        ev[2 * r + 1].record()
        z2.backward(gz2)
        ev[2 * r + 2].record()
    torch.cuda.synchronize()
    fwd = sum(ev[2 * r].elapsed_time(ev[2 * r + 1]) for r in range(reps)) * 1e3 / reps
    bwd = sum(ev[2 * r + 1].elapsed_time(ev[2 * r + 2]) for r in range(reps)) * 1e3 / reps
    f = _bound((STATS[0] + STEM12G[0], STATS[1] + STEM12G[1]), nimg, fwd)
    from generalizableracing_amd.rsl_rl import fused_bn

    b = _bound(STEM12W_MOM if fused_bn.STEM12_MOMENTS else STEM12W, nimg, bwd)
    return {"images": nimg, "forward": f, "backward": b,
            "note": "forward = statistics pass + stem12g_kernel (+ bn_stats_final); backward = stem12w_kernel (+ its two "
                    "fixed-order reductions); bytes / flops algorithmic per image (scripts/time_stem12.py, DESIGN §4c), "
                    "HIP events around each phase"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nimg", type=int, default=24576)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--stored-y1", action="store_true", help="the round-5 pair (y1 stored by stem12f_kernel, conv2's "
                    "weight gradient by gr_patch_wgrad) instead of stem12g / gr_stem12_backward_w2")
    ap.add_argument("--roofline", action="store_true", help="the forward / backward split against their bounds")
    ap.add_argument("--no-moments", action="store_true", help="the backward sums A2 / A3 itself (round-6 first form) "
                    "instead of taking them from the forward's pixel moments")
    a = ap.parse_args()
    from generalizableracing_amd.rsl_rl import fused_bn

    if a.stored_y1:
        fused_bn.STEM12_W2 = False
    if a.no_moments:
        fused_bn.STEM12_MOMENTS = False
    if a.roofline:
        print(json.dumps(roofline(a.nimg)))
        return
    forward, gz2 = _setup(a.nimg)
    for _ in range(3):
        forward().backward(gz2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        forward().backward(gz2)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"nimg": a.nimg, "reps": a.reps, "stored_y1": a.stored_y1, "ms_fwd_bwd": e0.elapsed_time(e1) / a.reps}))


if __name__ == "__main__":
    main()
