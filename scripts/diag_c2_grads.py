"""Diagnostic (GPU box): per-parameter error of the first mini-batch gradient of the C2 PPO update on cuda:0 vs the
build's CPU path (which equals the reference's to 3e-7), eager; with and without TallLinear's split-K."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import make_golden_ppo_c2 as mk  # noqa: E402
import ppo_c2_golden as pc2  # noqa: E402
from generalizableracing_amd.rsl_rl import ActorCritic, linear  # noqa: E402
from generalizableracing_amd.rsl_rl.ppo import PPO  # noqa: E402


def first_grads(device, split=True):
    data = mk.rollout_inputs()
    roll = PPO(mk.deterministic_sampling(mk.make_policy(ActorCritic)), None, device="cpu", **mk.HP)
    roll.init_storage("rl", mk.N, mk.T, [16], [16], [4])
    obs, cobs, rew, dones, tout, last, eps = data[0]
    with torch.inference_mode():
        for t in range(mk.T):
            roll.policy._eps = eps[t]
            roll.act(obs[t], cobs[t])
            roll.process_env_step(rew[t], dones[t], {"time_outs": tout[t]})
        roll.compute_returns(last)
    upd = PPO(mk.make_policy(ActorCritic), None, device=device, **mk.HP)
    upd.init_storage("rl", mk.N, mk.T, [16], [16], [4])
    for name, v in vars(roll.storage).items():
        if torch.is_tensor(v):
            getattr(upd.storage, name).copy_(v)
    upd.storage.step = roll.storage.step
    old = linear.SPLIT
    if not split:
        linear.SPLIT = 1 << 30
    grads = []
    torch.manual_seed(200)
    try:
        with pc2.cpu_randperm(), pc2.record_grads(upd, grads, count=1):
            upd.update()
    finally:
        linear.SPLIT = old
    names = [n for n, _ in upd.policy.named_parameters()]
    sizes = [p.numel() for p in upd.policy.parameters()]
    return grads[0].double(), names, sizes


gp = pc2.load()
want = torch.from_numpy(gp["ppo_it0_grad_mb0"]).double()
out = {}
for dev, split in (("cpu", True), ("cuda:0", True), ("cuda:0", False)):
    g, names, sizes = first_grads(dev, split)
    off, per = 0, {}
    for n, k in zip(names, sizes):
        a, b = g[off:off + k], want[off:off + k]
        per[n] = float((a - b).norm() / max(float(b.norm()), 1e-30))
        off += k
    out[f"{dev} split={split}"] = {"total": float((g - want).norm() / want.norm()), "per_param": per}
    print(dev, split, out[f"{dev} split={split}"]["total"], flush=True)
print(json.dumps(out, indent=1))
