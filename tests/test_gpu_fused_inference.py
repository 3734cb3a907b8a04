"""Fused MFMA rollout inference (gr_policy_forward) against the fp32 torch ActorCritic on the GPU.

Tolerance: bf16 operands (8-bit mantissa) with fp32 accumulation over K = 16 / 256 / 256: the mean
and the value must agree with the fp32 module to 2 % of the output scale; the log prob must be the
one torch's Normal gives for the kernel's own (mean, std, action) to 1e-4."""
from __future__ import annotations

import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.rsl_rl import ActorCritic  # noqa: E402
from generalizableracing_amd.rsl_rl.fused_inference import FusedPolicyInference  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("hidden,activation,n", [(256, "lrelu", 65536 + 17), (128, "elu", 1000)])
def test_matches_fp32_module(hidden, activation, n):
    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [hidden, hidden], [hidden, hidden], activation, init_noise_std=0.7).to(DEV)
    fused = FusedPolicyInference(pol, n, DEV, seed=3)
    obs = torch.randn(n, 16, device=DEV) * 2.0
    cobs = torch.randn(n, 16, device=DEV) * 2.0
    act, val, logp, mean, sigma = fused.act(obs, cobs)
    torch.cuda.synchronize()
    with torch.no_grad():
        m_ref, v_ref = pol.actor(obs), pol.critic(cobs)
    for got, want in ((mean, m_ref), (val, v_ref)):
        scale = float(want.abs().max()) + 1e-3
        err = float((got - want).abs().max())
        assert err < 2e-2 * scale, (err, scale)
    lp_ref = torch.distributions.Normal(mean, sigma).log_prob(act).sum(-1)
    assert float((logp - lp_ref).abs().max()) < 1e-4
    eps = (act - mean) / sigma
    tol = 5.0 / (4 * n) ** 0.5  # 5 standard errors
    assert abs(float(eps.mean())) < tol and abs(float(eps.std()) - 1.0) < 2 * tol
    # a second call draws fresh noise; the same seed and counter reproduce it
    a1 = act.clone()
    fused.act(obs, cobs)
    assert not torch.equal(a1, fused.actions)
    other = FusedPolicyInference(pol, n, DEV, seed=3)
    other.act(obs, cobs)
    torch.cuda.synchronize()
    assert torch.equal(a1, other.actions)


def test_refresh_after_update_and_graph_capture():
    torch.manual_seed(1)
    n = 4096
    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(DEV)
    fused = FusedPolicyInference(pol, n, DEV)
    obs = torch.randn(n, 16, device=DEV)
    fused.act(obs, obs)
    torch.cuda.synchronize()
    m0 = fused.action_mean.clone()
    with torch.no_grad():
        for p in pol.actor.parameters():
            p.add_(0.05 * torch.randn_like(p))
    fused.refresh()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fused.act(obs, obs)  # warm-up outside capture (even call count)
        fused.act(obs, obs)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fused.act(obs, obs)
        fused.act(obs, obs)
    g.replay()
    torch.cuda.synchronize()
    with torch.no_grad():
        want = pol.actor(obs)
    assert not torch.allclose(m0, fused.action_mean)
    assert float((fused.action_mean - want).abs().max()) < 2e-2 * (float(want.abs().max()) + 1e-3)
    c0 = fused.counters.clone()
    a0 = fused.actions.clone()
    g.replay()
    torch.cuda.synchronize()
    assert int(fused.counters.max()) == int(c0.max()) + 2  # the device counter advances inside the graph
    assert not torch.equal(a0, fused.actions)


@pytest.mark.parametrize("graph_update", [False, True])
def test_ppo_rollout_with_fused_inference(graph_update):
    """PPO with algorithm.fused_rollout_inference on the HIP env: the stored rollout matches the fp32 module,
    the log probs are those of the stored (mean, sigma, action), and an update is picked up by the next act."""
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg
    from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper
    from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg

    torch.manual_seed(2)
    n = 2048
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV)
    cfg.algorithm.fused_rollout_inference = True
    cfg.algorithm.graph_update = graph_update  # replays do not bump parameter versions: PPO refreshes
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    alg, pol = runner.alg, runner.alg.policy
    assert alg.fused is not None
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    steps = 3
    with torch.inference_mode():
        for k in range(steps):
            a = alg.act(obs, cobs)
            m_ref, v_ref = pol.actor(obs), pol.critic(cobs)
            for got, want in ((alg.fused.action_mean, m_ref), (alg.fused.values, v_ref)):
                assert float((got - want).abs().max()) < 2e-2 * (float(want.abs().max()) + 1e-3)
            obs, rew, dones, infos = env.step(a)
            cobs = infos["observations"]["critic"]
            alg.process_env_step(rew, dones, infos)
    st = alg.storage
    lp = torch.distributions.Normal(st.mu[:steps], st.sigma[:steps]).log_prob(st.actions[:steps]).sum(-1)
    assert float((lp - st.actions_log_prob[:steps, :, 0]).abs().max()) < 1e-4
    assert torch.isfinite(st.values[:steps]).all()
    # a full iteration: the update changes the weights in place, the next act repacks them
    st.clear()
    runner.learn(1)
    with torch.inference_mode():
        alg.act(obs, cobs)
        want = pol.actor(obs)
    assert float((alg.fused.action_mean - want).abs().max()) < 2e-2 * (float(want.abs().max()) + 1e-3)
