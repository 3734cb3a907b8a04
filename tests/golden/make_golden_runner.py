"""Golden vectors for the rsl_rl training loop, produced by the REFERENCE's own OnPolicyRunner
(standalone/rsl_rl/ext/runners/on_policy_runner.py) driving this repo's VecEnv surface.

Run in the development container (the reference is mounted read-only at /root/reference; it never travels to
the GPU box):

    python tests/golden/make_golden_runner.py

The env is the CPU-oracle VecEnv of the tests (tests/oracle_vecenv.py: the same `RslRlVecEnvWrapper` tuples
as the HIP env: get_observations -> (obs, {"observations": {policy, critic, aux}}), step -> (obs, rew,
dones long, extras{observations, time_outs, log})), so the fixture pins that the reference's runner loop runs
on this surface, and what it computes over two learning iterations: the policy parameters, the adaptive
learning rate, the losses and the episode logs it reads from extras["log"].

rsl_rl is not installed, so its names are bound as in make_golden_ppo.py: `rsl_rl.modules.ActorCritic` /
`EmpiricalNormalization` to the build's restatements of the upstream modules (the policy both sides step),
the reference's own PPO / PPOL2C2 / storages from its tree, and stubs for what the loop only logs with
(`store_code_state`, the tensorboard writer: tensorboard is not installed; the stub records the scalars).
"""
from __future__ import annotations

import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # the oracle's ctypes module (tests/conftest.py does the same)

import il_shim  # noqa: E402
from make_golden_ppo import load_reference  # noqa: E402

OUT = os.path.join(HERE, "golden_runner.npz")
EXT = os.path.join(il_shim.REF, "standalone/rsl_rl/ext")
NUM_ENVS, ITERS = 64, 2


def runner_cfg():
    """The reference's QuadcopterPPORunnerCfg (agents/rsl_rl_ppo_cfg.py) with small hidden layers and 8 steps
    per env, as the dict `OnPolicyRunner` receives from `agent_cfg.to_dict()`."""
    return {
        "num_steps_per_env": 8, "max_iterations": ITERS, "save_interval": 1000, "empirical_normalization": False,
        "experiment_name": "racing_ppo", "logger": "tensorboard", "seed": 42,
        "policy": {"class_name": "ActorCritic", "init_noise_std": 1.0, "actor_hidden_dims": [32, 32],
                   "critic_hidden_dims": [32, 32], "activation": "lrelu"},
        "algorithm": {"class_name": "PPO", "value_loss_coef": 1.0, "use_clipped_value_loss": True, "clip_param": 0.2,
                      "entropy_coef": 0.0, "num_learning_epochs": 5, "num_mini_batches": 4, "learning_rate": 5.0e-4,
                      "schedule": "adaptive", "gamma": 0.99, "lam": 0.95, "desired_kl": 0.01, "max_grad_norm": 1.0},
    }


class RecordingWriter:
    """Stand-in for torch.utils.tensorboard.SummaryWriter: keeps every scalar."""
    scalars: dict = {}

    def __init__(self, *a, **k):
        RecordingWriter.scalars = {}

    def add_scalar(self, key, value, step):
        RecordingWriter.scalars.setdefault(key, {})[int(step) if float(step).is_integer() else float(step)] = float(value)

    def close(self):
        pass


def load_reference_runner():
    RefPPO, RefL2C2 = load_reference()
    from generalizableracing_amd.rsl_rl import ActorCritic, VisionActorCritic
    from generalizableracing_amd.rsl_rl.actor_critic import EmpiricalNormalization

    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = RecordingWriter
    sys.modules["torch.utils.tensorboard"] = tb
    for n in ("rsl_rl.env",):
        sys.modules.setdefault(n, types.ModuleType(n))
    sys.modules["rsl_rl"].__file__ = os.path.join(EXT, "__init__.py")
    sys.modules["rsl_rl.env"].VecEnv = object
    m = sys.modules["rsl_rl.modules"]
    m.ActorCritic, m.ActorCriticRecurrent, m.EmpiricalNormalization = ActorCritic, il_shim._unsupported, EmpiricalNormalization
    sys.modules["rsl_rl.utils"].store_code_state = lambda *a, **k: []
    mods = types.ModuleType("standalone.rsl_rl.ext.modules")
    mods.VisionActorCritic = VisionActorCritic
    mods.VisionActorCriticRecurrent = mods.StudentTeacher = mods.VisionStudentTeacher = il_shim._unsupported
    sys.modules["standalone.rsl_rl.ext.modules"] = mods
    algs = types.ModuleType("standalone.rsl_rl.ext.algorithms")
    algs.PPO, algs.PPOL2C2, algs.Distillation, algs.PPOLCP = RefPPO, RefL2C2, il_shim._unsupported, il_shim._unsupported
    sys.modules["standalone.rsl_rl.ext.algorithms"] = algs
    return il_shim.load("grref_on_policy_runner", os.path.join(EXT, "runners/on_policy_runner.py")).OnPolicyRunner


def main():
    from oracle_vecenv import OracleVecEnv

    Runner = load_reference_runner()
    torch.manual_seed(0)
    env = OracleVecEnv(num_envs=NUM_ENVS)
    with tempfile.TemporaryDirectory() as d:
        runner = Runner(env, runner_cfg(), log_dir=d, device="cpu")
        rec = {"init_params": torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()])}
        runner.learn(ITERS, init_at_random_ep_len=False)
    rec["params"] = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()])
    rec["learning_rate"] = torch.tensor(float(runner.alg.learning_rate), dtype=torch.float64)
    sc = RecordingWriter.scalars
    keys = sorted(k for k in sc if k.startswith(("Loss/", "Episode_", "Curriculum/", "Metrics/", "Policy/")))
    for k in keys:
        rec["scalar:" + k] = torch.tensor([sc[k].get(it, float("nan")) for it in range(ITERS)], dtype=torch.float64)
    out = {k: np.ascontiguousarray(v.detach().cpu().numpy()) for k, v in rec.items()}
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(out)} arrays, lr {float(rec['learning_rate']):.3e}, {len(keys)} logged scalars")


if __name__ == "__main__":
    main()
