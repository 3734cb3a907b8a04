"""PPOL2C2 + RolloutStorageL2C2 (standalone/rsl_rl/ext/algorithms/ppo_l2c2.py,
storage/rollout_storage_l2c2.py) on CPU: the next-observation pairing, the smoothness
loss restated by hand, the zero-observation skip, and a full runner iteration."""
import math

import torch

from generalizableracing_amd.rsl_rl import (ActorCritic, OnPolicyRunner, PPOL2C2, QuadcopterL2C2PPORunnerCfg,
                                            RolloutStorageL2C2)
from oracle_vecenv import OracleVecEnv


def _fill(st, T, N, obs, dones):
    for t in range(T):
        tr = RolloutStorageL2C2.Transition()
        tr.observations = obs[t]
        tr.privileged_observations = obs[t] * 2.0
        tr.actions = torch.full((N, 2), float(t))
        tr.rewards = torch.ones(N)
        tr.dones = dones[t]
        tr.values = torch.zeros(N, 1)
        tr.actions_log_prob = torch.zeros(N)
        tr.action_mean = torch.zeros(N, 2)
        tr.action_sigma = torch.ones(N, 2)
        st.add_transitions(tr)


def test_storage_pairs_next_observation():
    """rollout_storage_l2c2.py:131-167: (T-1)*N samples, next_obs = obs[t+1] of the same env,
    cont = 1 - done[t]."""
    T, N, D = 5, 3, 4
    st = RolloutStorageL2C2("rl", N, T, [D], [D], [2], "cpu")
    obs = torch.arange(T * N * D, dtype=torch.float32).view(T, N, D)
    dones = torch.zeros(T, N, dtype=torch.long)
    dones[1, 2] = 1
    dones[3, 0] = 1
    _fill(st, T, N, obs, dones)
    st.compute_returns(torch.zeros(N, 1), 0.99, 0.95)
    batches = list(st.mini_batch_generator(num_mini_batches=1, num_epochs=1))
    assert len(batches) == 1
    o, c, nxt, cont, act = batches[0][:5]
    assert o.shape == ((T - 1) * N, D)
    flat = obs.view(T * N, D)
    for k in range(o.shape[0]):
        row = int(torch.nonzero((flat == o[k]).all(1))[0])
        t, n = divmod(row, N)
        assert t < T - 1
        assert torch.equal(nxt[k], obs[t + 1, n])
        assert torch.equal(c[k], 2.0 * obs[t, n])
        assert float(cont[k]) == 1.0 - float(dones[t, n])
        assert float(act[k, 0]) == float(t)


def test_smoothness_coefficients():
    """ppo_l2c2.py:176-178 with the constructor defaults (0.1, 1.0, 0.1)."""
    pol = ActorCritic(4, 4, 2, [8], [8], "lrelu")
    alg = PPOL2C2(pol, device="cpu")
    c_pi, c_v = alg.smooth_coefs()
    assert math.isclose(c_pi, 1.0 * 0.1 / 0.9)
    assert math.isclose(c_v, 0.1 * 0.1 / 0.9)


def test_smooth_loss_matches_hand_restatement():
    torch.manual_seed(1)
    pol = ActorCritic(6, 6, 3, [16, 16], [16, 16], "lrelu")
    alg = PPOL2C2(pol, device="cpu", value_smoothness_coef=0.3, smoothness_upper_bound=2.0,
                  smoothness_lower_bound=0.5)
    B = 32
    o = torch.randn(B, 6)
    o2 = torch.randn(B, 6)
    cont = (torch.rand(B, 1) > 0.3).float()
    pol.act(o)
    mu = pol.action_mean
    v = pol.evaluate(o)
    torch.manual_seed(7)
    loss, smooth = alg.smooth_loss(o, o2, cont, mu, v)
    torch.manual_seed(7)
    w = cont * (torch.rand(B, 1) - 0.5) * 2.0
    assert float(w.abs().max()) <= 1.0
    mix = o + w * (o2 - o)
    eps = 0.5 / (2.0 - 0.5)
    c_pi = 2.0 * eps
    c_v = 0.3 * c_pi
    pl = ((mu - pol.actor(mix)) ** 2).sum(-1).mean()
    vl = ((v - pol.critic(mix)) ** 2).sum(-1).mean()
    torch.testing.assert_close(loss, c_pi * pl + c_v * vl, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(smooth, (mu - pol.actor(o2)).norm(dim=-1).mean(), rtol=1e-6, atol=1e-7)
    # a reset between t and t+1 (cont = 0) leaves the sample unmixed: zero smoothness term
    torch.manual_seed(7)
    loss0, _ = alg.smooth_loss(o, o2, torch.zeros(B, 1), mu, v)
    assert float(loss0.detach()) == 0.0
    # gradient flows into both heads
    loss.backward()
    assert pol.actor[0].weight.grad is not None and pol.critic[0].weight.grad is not None


def test_zero_observation_transition_is_skipped():
    """ppo_l2c2.py:98: a transition whose observation batch is all ~0 is not stored."""
    pol = ActorCritic(4, 4, 2, [8], [8], "lrelu")
    alg = PPOL2C2(pol, device="cpu")
    alg.init_storage("rl", 3, 4, [4], [4], [2])
    for obs in (torch.zeros(3, 4), torch.ones(3, 4)):
        alg.act(obs, obs)
        alg.process_env_step(torch.zeros(3), torch.zeros(3, dtype=torch.long), {})
    assert alg.storage.step == 1


def test_runner_trains_with_l2c2(tmp_path):
    torch.manual_seed(0)
    cfg = QuadcopterL2C2PPORunnerCfg(device="cpu", num_steps_per_env=8, save_interval=1)
    cfg.policy.actor_hidden_dims = [32, 32]
    cfg.policy.critic_hidden_dims = [32, 32]
    assert cfg.to_dict()["algorithm"]["class_name"] == "PPOL2C2"
    assert cfg.to_dict()["algorithm"]["entropy_coef"] == 0.005
    runner = OnPolicyRunner(OracleVecEnv(num_envs=64), cfg.to_dict(), log_dir=str(tmp_path), device="cpu")
    assert isinstance(runner.alg, PPOL2C2)
    runner.learn(2)
    log = runner.last_log
    for k in ("value_function", "surrogate", "smooth_loss"):
        assert math.isfinite(log[k]), k
    assert log["smooth_loss"] > 0.0
    assert (tmp_path / "model_1.pt").exists()


def _drive(alg, obs_seq, sink):
    """The runner's collection loop (on_policy_runner.py learn) over a scripted observation sequence; with `sink`
    the env writes each step's rows into the storage slot and returns that slot (RacingEnv's fp32 sink)."""
    st = alg.storage
    obs = obs_seq[0].clone()
    for t in range(1, len(obs_seq)):
        alg.act(obs, obs * 2.0)
        if sink:
            p, c = st.sink_slot(st.step + 1)
            p.copy_(obs_seq[t])
            c.copy_(obs_seq[t] * 2.0)
            obs = p
        else:
            obs = obs_seq[t].clone()
        alg.process_env_step(torch.ones(obs.shape[0]), torch.zeros(obs.shape[0], dtype=torch.long), {})


def test_observation_sink_with_zero_observation_skip():
    """PPOL2C2 with the observation sink stores the same transitions as the copy path, also across
    ppo_l2c2.py:98's skip of an all-zero observation batch (the skipped transition's successor rows move down a
    slot: RolloutStorage.sink_skipped)."""
    T, N, D = 6, 5, 4
    g = torch.Generator().manual_seed(3)
    obs_seq = [torch.randn(N, D, generator=g) for _ in range(T + 2)]
    obs_seq[2] = torch.zeros(N, D)  # the transition acting on these rows is skipped
    stores = []
    for sink in (True, False):
        torch.manual_seed(0)
        alg = PPOL2C2(ActorCritic(D, D, 2, [8], [8], "lrelu"), device="cpu")
        alg.init_storage("rl", N, T, [D], [D], [2])
        if sink:
            alg.storage.enable_obs_sink()
        torch.manual_seed(1)
        _drive(alg, obs_seq, sink)
        stores.append(alg.storage)
    a, b = stores
    assert a.step == b.step == T
    assert torch.equal(a.observations[:T], b.observations)
    assert torch.equal(a.privileged_observations[:T], b.privileged_observations)
    assert torch.equal(a.actions, b.actions)
    # the stored rows are the scripted ones minus the skipped batch
    want = torch.stack([o for k, o in enumerate(obs_seq[:T + 1]) if k != 2])
    assert torch.equal(b.observations, want)


def test_runner_l2c2_camera_sink_matches_copy():
    """OnPolicyRunner + PPOL2C2 on the camera task (oracle env, [16 | image] rows): with the fp32 observation sink
    the stored rows and the trained parameters equal the copy path's."""
    from generalizableracing_amd.envs.racing_cfg import CameraCfg

    runs = []
    for sink in (True, False):
        torch.manual_seed(0)
        cfg = QuadcopterL2C2PPORunnerCfg(device="cpu", num_steps_per_env=4)
        cfg.policy.actor_hidden_dims = [16]
        cfg.policy.critic_hidden_dims = [16]
        cfg.algorithm.obs_sink = sink
        cam = CameraCfg(width=16, height=8)
        r = OnPolicyRunner(OracleVecEnv(num_envs=8, camera=cam), cfg.to_dict(), log_dir=None, device="cpu")
        assert r.obs_sink is sink
        r.learn(2)
        runs.append(r)
    a, b = runs
    T = a.num_steps_per_env
    assert a.alg.storage.observations.shape[2] == 16 + 16 * 8
    assert torch.equal(a.alg.storage.observations[1:T], b.alg.storage.observations[1:T])
    for (k, x), (_, y) in zip(a.alg.policy.state_dict().items(), b.alg.policy.state_dict().items()):
        assert torch.equal(x, y), k
