"""ActorCritic — the rsl_rl MLP policy the runner instantiates
(rsl_rl.modules.ActorCritic, used via standalone/rsl_rl/ext/runners/on_policy_runner.py:15,57-60;
rsl_rl is not vendored in the reference, rsl-rl-lib ~2.2-2.3 semantics restated).

Gaussian policy with a state-independent std (noise_std_type "scalar" or
"log"), separate actor / critic MLPs, log-prob and entropy summed over the 4
CTBR actions.  GEMMs run on hipBLASLt through torch.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.distributions import Normal

from .linear import MLP, TallLinear


def resolve_nn_activation(name: str) -> nn.Module:
    table = {
        "elu": nn.ELU(), "selu": nn.SELU(), "relu": nn.ReLU(), "crelu": nn.CELU(),
        "lrelu": nn.LeakyReLU(), "tanh": nn.Tanh(), "sigmoid": nn.Sigmoid(),
    }
    if name not in table:
        raise ValueError(f"Invalid activation function '{name}'.")
    return table[name]


def _mlp(inp: int, hidden: list, out: int, act: str) -> nn.Sequential:
    # TallLinear = nn.Linear (same parameters / state_dict keys) with a row-split weight gradient; MLP =
    # nn.Sequential whose last LeakyReLU + Linear fuse on the update's tall batches (linear.py)
    layers = [TallLinear(inp, hidden[0]), resolve_nn_activation(act)]
    for i in range(len(hidden)):
        if i == len(hidden) - 1:
            layers.append(TallLinear(hidden[i], out))
        else:
            layers.append(TallLinear(hidden[i], hidden[i + 1]))
            layers.append(resolve_nn_activation(act))
    return MLP(*layers)


class ActorCritic(nn.Module):
    is_recurrent = False

    def __init__(self, num_actor_obs, num_critic_obs, num_actions, actor_hidden_dims=(256, 256, 256),
                 critic_hidden_dims=(256, 256, 256), activation="elu", init_noise_std=1.0,
                 noise_std_type: str = "scalar", **kwargs):
        if kwargs:
            print("ActorCritic.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs)))
        super().__init__()
        self.actor = _mlp(num_actor_obs, list(actor_hidden_dims), num_actions, activation)
        self.critic = _mlp(num_critic_obs, list(critic_hidden_dims), 1, activation)
        self.noise_std_type = noise_std_type
        if noise_std_type == "scalar":
            self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        elif noise_std_type == "log":
            self.log_std = nn.Parameter(torch.log(init_noise_std * torch.ones(num_actions)))
        else:
            raise ValueError(f"Unknown standard deviation type: {noise_std_type}. Should be 'scalar' or 'log'")
        self.distribution = None
        Normal.set_default_validate_args(False)

    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def _std(self, mean):
        if self.noise_std_type == "scalar":
            return self.std.expand_as(mean)
        return torch.exp(self.log_std).expand_as(mean)

    def update_distribution(self, observations):
        mean = self.actor(observations)
        self.distribution = Normal(mean, self._std(mean))

    def act(self, observations, **kwargs):
        self.update_distribution(observations)
        d = self.distribution
        if d.loc.is_cuda:
            # Normal.sample is torch.normal(loc, scale), whose `std >= 0` check reads back to the host on every
            # call; its draw is normal_(0, 1) into a fresh tensor, then mul_(std).add_(mean): the same bits here,
            # without the synchronisation
            with torch.no_grad():
                return torch.randn(d.loc.shape, dtype=d.loc.dtype, device=d.loc.device).mul_(d.scale).add_(d.loc)
        return d.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_inference(self, observations):
        return self.actor(observations)

    def evaluate(self, critic_observations, **kwargs):
        return self.critic(critic_observations)

    def load_state_dict(self, state_dict, strict=True):
        super().load_state_dict(state_dict, strict=strict)
        return True  # rsl_rl: "resumed training"


class EmpiricalNormalization(nn.Module):
    """rsl_rl.modules.EmpiricalNormalization (running mean/var until `until` samples)."""

    def __init__(self, shape, eps=1e-2, until=None):
        super().__init__()
        self.eps = eps
        self.until = until
        self.register_buffer("_mean", torch.zeros(shape).unsqueeze(0))
        self.register_buffer("_var", torch.ones(shape).unsqueeze(0))
        self.register_buffer("_std", torch.ones(shape).unsqueeze(0))
        self.register_buffer("count", torch.tensor(0, dtype=torch.long))

    def forward(self, x):
        if self.training:
            self.update(x)
        return (x - self._mean) / (self._std + self.eps)

    @torch.jit.unused
    def update(self, x):
        if self.until is not None and self.count >= self.until:
            return
        count_x = x.shape[0]
        self.count += count_x
        rate = count_x / self.count
        var_x = torch.var(x, dim=0, unbiased=False, keepdim=True)
        mean_x = torch.mean(x, dim=0, keepdim=True)
        delta_mean = mean_x - self._mean
        self._mean += rate * delta_mean
        self._var += rate * (var_x - self._var + delta_mean * (mean_x - self._mean))
        self._std = torch.sqrt(self._var)
