"""Diagnostic (GPU box): where the actor's hidden-layer gradients of the C2 first mini-batch lose accuracy on cuda:0.
Intermediate tensors of the forward and their gradients, GPU fp32 vs CPU fp64, plain nn.Linear layers."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import make_golden_ppo_c2 as mk  # noqa: E402
from generalizableracing_amd.rsl_rl import ActorCritic  # noqa: E402
from generalizableracing_amd.rsl_rl.ppo import PPO  # noqa: E402

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
st = roll.storage
torch.manual_seed(200)
idx = torch.randperm(mk.N * mk.T)[: mk.N * mk.T // 4]


def run(dev, dtype):
    pol = mk.plain_linear(mk.make_policy(ActorCritic)).to(dev, dtype)
    f = lambda x: x.flatten(0, 1)[idx].to(dev, dtype)  # noqa: E731
    o, c, a, v, adv, ret, lp = (f(getattr(st, k)) for k in ("observations", "privileged_observations", "actions",
                                                             "values", "advantages", "returns", "actions_log_prob"))
    acts = {}
    hooks = []
    def hook(mod, inp, out, i):
        out.retain_grad()
        acts[f"a{i}"] = out

    for i, m in enumerate(pol.actor):
        m.register_forward_hook(lambda mod, inp, out, i=i: hook(mod, inp, out, i))
    pol.update_distribution(o)
    logp = pol.get_actions_log_prob(a)
    val = pol.evaluate(c)
    alg = PPO(pol, None, device=dev, **mk.HP)
    s, vl = alg._ppo_losses(logp, lp, adv, val, v, ret)
    (s + vl).backward()
    out = {k: (x.detach().double().cpu(), x.grad.double().cpu()) for k, x in acts.items()}
    out["params"] = [(n, p.grad.double().cpu()) for n, p in pol.named_parameters()]
    return out


ref = run("cpu", torch.float64)
for dev in ("cpu", "cuda:0") if torch.cuda.is_available() else ("cpu",):
    got = run(dev, torch.float32)
    print("=====", dev)
    for k in ref:
        if k == "params":
            continue
        (x, g), (xr, gr) = got[k], ref[k]
        flips = int(((x > 0) != (xr > 0)).sum())
        print(f"{k}: value {float((x - xr).norm() / xr.norm()):.2e}  grad {float((g - gr).norm() / gr.norm()):.2e}  "
              f"sign flips vs float64 {flips}, |x| < 1e-6: {int((xr.abs() < 1e-6).sum())}")
    for (n, g), (_, gr) in zip(got["params"], ref["params"]):
        print(f"  {n:16s} {float((g - gr).norm() / gr.norm()):.2e}")
