"""Golden vectors for VisionActorCritic, produced by the REFERENCE's own module
(standalone/rsl_rl/ext/modules/vision_actor_critic.py:43-144) — TEST INFRASTRUCTURE.

Run in the development container (the reference is mounted read-only at /root/reference; it never travels to
the GPU box, only the .npz this writes does):

    python tests/golden/make_golden_vision.py

The module file imports upstream rsl_rl (`rsl_rl.modules.actor_critic_recurrent`: ActorCritic,
ActorCriticRecurrent, Memory; `rsl_rl.utils.unpad_trajectories`), which is not installed.  A minimal stub stands
in: `ActorCritic` restated from rsl-rl-lib 2.2 (actor / critic nn.Sequential MLPs with the upstream key names,
a scalar std parameter, a Normal distribution, summed log prob); the recurrent names raise if reached (they are
not on VisionActorCritic's path).  Everything the fixture pins — the conv stem, its BatchNorms, the state
encoder, the feature sum and activation, act_inference / update_distribution / evaluate — runs the reference's
own code over that base.

Inputs: 256 observation rows [16 state terms | 72 x 96 depth image] (policy and critic groups) of the CPU oracle
env with its depth camera (tests/oracle_vecenv.py, obstacle tracks) after 6 random-action steps, so the images
are real renders (gates, walls, ground, the 10 m clip); both groups use the noise-free image (stored once).  The module is the registered recipe's
(agents/rsl_rl_ppo_cfg.py:43-52,80-104: img_res (72, 96), dim_hidden_input 192, heads [128, 128], lrelu,
use_auxiliary_loss) with seeded weights and randomised BatchNorm affine parameters and running statistics.

Recorded:
  * the state_dict the comparison loads (every parameter and buffer);
  * eval mode: act_inference -> (mean, feat), update_distribution -> (mean, stddev), evaluate -> value;
  * train mode: update_distribution(policy rows) -> mean, log_prob(actions).sum(-1), evaluate(critic rows);
    the BatchNorm running statistics after those two forwards; the gradient of every parameter of the scalar
    loss  sum(mean * g_mu) + mean(log_prob * w) + sum(value * g_v)  (fixed random g_mu, w, g_v).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn
from torch.distributions import Normal

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import il_shim  # noqa: E402
from vision_golden import observation_rows, randomise, run  # noqa: E402

OUT = os.path.join(HERE, "golden_vision.npz")
VAC = os.path.join(il_shim.REF, "standalone/rsl_rl/ext/modules/vision_actor_critic.py")
N, OBS, H, W = 256, 16 + 72 * 96, 72, 96


class UpstreamActorCritic(nn.Module):
    """rsl-rl-lib 2.2 `rsl_rl.modules.ActorCritic`, restated (the reference subclasses it; not vendored): MLPs
    Linear -> act -> ... -> Linear named actor.* / critic.*, std = init_noise_std * ones, Normal(mean, std)."""
    is_recurrent = False

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=(256, 256, 256),
                 critic_hidden_dims=(256, 256, 256), activation="elu", init_noise_std=1.0, **kwargs):
        super().__init__()
        acts = {"elu": nn.ELU, "selu": nn.SELU, "relu": nn.ReLU, "lrelu": nn.LeakyReLU, "tanh": nn.Tanh,
                "sigmoid": nn.Sigmoid}

        def mlp(inp, hidden, out):
            layers = [nn.Linear(inp, hidden[0]), acts[activation]()]
            for i in range(len(hidden)):
                if i == len(hidden) - 1:
                    layers.append(nn.Linear(hidden[i], out))
                else:
                    layers += [nn.Linear(hidden[i], hidden[i + 1]), acts[activation]()]
            return nn.Sequential(*layers)

        self.actor = mlp(num_actor_obs, list(actor_hidden_dims), num_actions)
        self.critic = mlp(num_critic_obs, list(critic_hidden_dims), 1)
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        Normal.set_default_validate_args(False)

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)


def load_reference_vac():
    for n in ("rsl_rl", "rsl_rl.modules", "rsl_rl.modules.actor_critic_recurrent", "rsl_rl.utils"):
        sys.modules[n] = types.ModuleType(n)
    acr = sys.modules["rsl_rl.modules.actor_critic_recurrent"]
    acr.ActorCritic = UpstreamActorCritic
    acr.ActorCriticRecurrent = type("ActorCriticRecurrent", (nn.Module,), {"__init__": il_shim._unsupported})
    acr.Memory = il_shim._unsupported
    sys.modules["rsl_rl.utils"].unpad_trajectories = il_shim._unsupported
    return il_shim.load("grref_vision_actor_critic", VAC).VisionActorCritic


def policy_kwargs():
    """The registered recipe's policy (agents/rsl_rl_ppo_cfg.py:43-52, use_auxiliary_loss :103)."""
    return dict(img_res=(H, W), dim_hidden_input=192, actor_hidden_dims=[128, 128], critic_hidden_dims=[128, 128],
                activation="lrelu", init_noise_std=1.0, noise_std_type="scalar", use_auxiliary_loss=True)


def main():
    Ref = load_reference_vac()
    pol, cri = observation_rows()
    torch.manual_seed(0)
    ref = Ref(OBS, OBS, 4, **policy_kwargs())
    g = torch.Generator().manual_seed(5)
    randomise(ref, g)
    actions = torch.randn(N, 4, generator=g)
    g_mu, w, g_v = torch.randn(N, 4, generator=g), torch.randn(N, generator=g), torch.randn(N, 1, generator=g)
    sd = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    rec = run(ref, pol, cri, actions, g_mu, w, g_v)
    out = {"obs_policy_state": pol[:, :16], "obs_critic": cri, "actions": actions, "g_mu": g_mu, "w": w, "g_v": g_v}
    out.update({"sd:" + k: v for k, v in sd.items()})
    out.update(rec)
    # the same module and inputs in float64: the reference's own fp32 round-off is then visible (its conv1 weight
    # gradient, a BatchNorm backward reduced over ~200 000 rows, is ~7e-5 off its float64 value)
    ref64 = Ref(OBS, OBS, 4, **policy_kwargs()).double()
    ref64.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in sd.items()})
    rec64 = run(ref64, pol.double(), cri.double(), actions.double(), g_mu.double(), w.double(), g_v.double())
    # (stored rounded to fp32: 6e-8 relative, far below the tolerances it serves)
    out.update({"f64:" + k: v.float() for k, v in rec64.items() if not k.startswith("after:")})
    arrays = {k: np.ascontiguousarray(v.cpu().numpy()) for k, v in out.items()}
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: {len(arrays)} arrays; eval mean[0] {arrays['eval_mean'][0]}, loss "
          f"{float(arrays['train_loss'].reshape(())):.6f}")


if __name__ == "__main__":
    main()
