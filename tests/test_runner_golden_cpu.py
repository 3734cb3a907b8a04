"""The build's OnPolicyRunner against the reference's own runner loop (tests/golden/make_golden_runner.py:
standalone/rsl_rl/ext/runners/on_policy_runner.py driving the same CPU-oracle VecEnv surface, two learning
iterations): same initial and final policy parameters, adaptive learning rate, and logged losses."""
import os

import numpy as np
import pytest
import torch

from generalizableracing_amd.rsl_rl import OnPolicyRunner
from oracle_vecenv import OracleVecEnv

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "golden_runner.npz")


def runner_cfg():
    # the dict of make_golden_runner.runner_cfg (the generator imports the reference, so it is not imported here)
    return {
        "num_steps_per_env": 8, "max_iterations": 2, "save_interval": 1000, "empirical_normalization": False,
        "experiment_name": "racing_ppo", "logger": "tensorboard", "seed": 42,
        "policy": {"class_name": "ActorCritic", "init_noise_std": 1.0, "actor_hidden_dims": [32, 32],
                   "critic_hidden_dims": [32, 32], "activation": "lrelu"},
        "algorithm": {"class_name": "PPO", "value_loss_coef": 1.0, "use_clipped_value_loss": True, "clip_param": 0.2,
                      "entropy_coef": 0.0, "num_learning_epochs": 5, "num_mini_batches": 4, "learning_rate": 5.0e-4,
                      "schedule": "adaptive", "gamma": 0.99, "lam": 0.95, "desired_kl": 0.01, "max_grad_norm": 1.0},
    }


def _scalars(log_dir):
    out = {}
    for root, _, files in os.walk(log_dir):
        if "scalars.csv" in files:
            for line in open(os.path.join(root, "scalars.csv")):
                step, key, value = line.rstrip("\n").split(",", 2)
                out.setdefault(key, {})[int(float(step))] = float(value)
    return out


@pytest.mark.skipif(not os.path.exists(GOLDEN), reason="golden_runner.npz not generated")
def test_runner_matches_reference_runner(tmp_path):
    g = dict(np.load(GOLDEN))
    torch.manual_seed(0)
    env = OracleVecEnv(num_envs=64)
    runner = OnPolicyRunner(env, runner_cfg(), log_dir=str(tmp_path), device="cpu")
    p0 = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).numpy()
    np.testing.assert_array_equal(p0, g["init_params"])  # same module tree, same draws
    runner.learn(2, init_at_random_ep_len=False)
    p1 = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).numpy()
    # two rollouts of the oracle env + two PPO updates (5 epochs x 4 mini-batches, Adam): fp32 CPU arithmetic
    np.testing.assert_allclose(p1, g["params"], rtol=1e-5, atol=1e-6)
    lr = float(np.asarray(g["learning_rate"]).reshape(-1)[0])
    assert abs(float(runner.alg.learning_rate) - lr) <= 1e-9 * lr
    sc = _scalars(str(tmp_path))
    checked = 0
    for k in g:
        if not k.startswith("scalar:"):
            continue
        key = k[len("scalar:"):]
        assert key in sc, f"{key} not logged"
        ours = np.array([sc[key].get(it, np.nan) for it in range(2)])
        np.testing.assert_allclose(ours, g[k], rtol=1e-5, atol=1e-7, err_msg=key)
        checked += 1
    assert checked >= 4
