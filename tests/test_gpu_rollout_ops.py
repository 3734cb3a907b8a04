"""The rollout loop's bookkeeping ops (rsl_rl/rollout_ops.py, csrc/gr_rollout.hip) bit-exact against the torch
ops they replace: PPO.process_env_step + RolloutStorage.add_transitions (ppo.py:83-95, rollout_storage.py:74-98),
compute_returns' GAE (rollout_storage.py:113-127, against the CPU loop: IEEE fp32 ops, no contraction on either
side), the runner's episode statistics (on_policy_runner.py:128-173), and the sync-free action draw of
ActorCritic.act against torch.normal (Normal.sample) under the same seed."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _storage(n, t, device):
    from generalizableracing_amd.rsl_rl.rollout_storage import RolloutStorage

    return RolloutStorage("rl", n, t, [16], [16], [4], device)


def _transition(n, g, k=4):
    from generalizableracing_amd.rsl_rl.rollout_storage import RolloutStorage

    tr = RolloutStorage.Transition()
    tr.observations = torch.randn(n, 16, generator=g).to(DEV)
    tr.privileged_observations = torch.randn(n, 16, generator=g).to(DEV)
    tr.actions = torch.randn(n, k, generator=g).to(DEV)
    tr.values = torch.randn(n, 1, generator=g).to(DEV)
    tr.actions_log_prob = torch.randn(n, generator=g).to(DEV)
    tr.action_mean = torch.randn(n, k, generator=g).to(DEV)
    tr.action_sigma = torch.rand(k, generator=g).to(DEV).expand(n, k)  # the expanded std (row stride 0)
    return tr


@pytest.mark.parametrize("dones_dtype,bootstrap", [(torch.int64, True), (torch.bool, True), (torch.uint8, False)])
def test_store_transition_matches_torch(dones_dtype, bootstrap):
    from generalizableracing_amd.rsl_rl import rollout_ops as R

    n, T, gamma = 3001, 5, 0.99
    g = torch.Generator().manual_seed(1)
    ref, got = _storage(n, T, DEV), _storage(n, T, DEV)
    for _ in range(T):
        tr = _transition(n, g)
        rewards = torch.randn(n, generator=g).to(DEV)
        rewards[::7] = -0.0
        dones = (torch.rand(n, generator=g) < 0.2).to(dones_dtype).to(DEV)
        tos = (torch.rand(n, generator=g) < 0.3).to(DEV) if bootstrap else None
        assert R.store_ok(got, tr, rewards, dones, tos)
        R.store_transition(got, tr, rewards, dones, tos, gamma)
        tr.rewards = rewards.clone()  # PPO.process_env_step
        tr.dones = dones
        if tos is not None:
            tr.rewards += gamma * torch.squeeze(tr.values * tos.unsqueeze(1).to(DEV), 1)
        ref.add_transitions(tr)
    torch.cuda.synchronize()
    assert got.step == ref.step == T
    for name in ("observations", "privileged_observations", "rewards", "dones", "actions", "values",
                 "actions_log_prob", "mu", "sigma"):
        a, b = getattr(got, name), getattr(ref, name)
        assert a.dtype == b.dtype and torch.equal(a.view(torch.uint8) if a.is_floating_point() else a,
                                                  b.view(torch.uint8) if b.is_floating_point() else b), name


@pytest.mark.parametrize("n,T", [(4096, 24), (1, 1), (777, 3)])
def test_gae_matches_cpu_loop(n, T):
    from generalizableracing_amd.rsl_rl import rollout_ops as R

    g = torch.Generator().manual_seed(2)
    cpu = _storage(n, T, "cpu")
    cpu.rewards.copy_(torch.randn(T, n, 1, generator=g))
    cpu.values.copy_(torch.randn(T, n, 1, generator=g))
    cpu.dones.copy_((torch.rand(T, n, 1, generator=g) < 0.1).byte())
    last = torch.randn(n, 1, generator=g)
    dev = _storage(n, T, DEV)
    for k in ("rewards", "values", "dones"):
        getattr(dev, k).copy_(getattr(cpu, k))
    assert R.gae_ok(dev, last.to(DEV))
    cpu.compute_returns(last, 0.99, 0.95, normalize_advantage=False)
    dev.compute_returns(last.to(DEV), 0.99, 0.95, normalize_advantage=False)
    assert torch.equal(dev.returns.cpu().view(torch.int32), cpu.returns.view(torch.int32))
    assert torch.equal(dev.advantages.cpu().view(torch.int32), cpu.advantages.view(torch.int32))
    # with the normalisation (torch's global mean / std on both sides; reductions may differ in the last ulp; one
    # sample: the unbiased std is NaN on both)
    cpu.compute_returns(last, 0.99, 0.95)
    dev.compute_returns(last.to(DEV), 0.99, 0.95)
    torch.testing.assert_close(dev.advantages.cpu(), cpu.advantages, rtol=1e-5, atol=1e-5, equal_nan=True)


def test_episode_stats_device_matches_host():
    from generalizableracing_amd.rsl_rl.rollout_ops import EpisodeStats

    g = torch.Generator().manual_seed(3)
    n, steps = 5000, 60
    rews = torch.randn(steps, n, generator=g)
    dones = (torch.rand(steps, n, generator=g) < 0.02).long()
    a, b = EpisodeStats(n, "cpu", steps=24), EpisodeStats(n, DEV, steps=24)
    for r, d in zip(rews, dones):
        a.update(r, d)
        b.update(r.to(DEV), d.to(DEV))
    ma, mb = a.means(), b.means()
    assert torch.equal(a.buf_rew, b.buf_rew.cpu()) and torch.equal(a.buf_len, b.buf_len.cpu())
    assert torch.equal(a.cur_rew, b.cur_rew.cpu()) and torch.equal(a.cur_len, b.cur_len.cpu())
    assert ma == pytest.approx(mb, rel=1e-6)


def test_actor_critic_act_draw_matches_torch_normal():
    from generalizableracing_amd.rsl_rl import ActorCritic

    pol = ActorCritic(16, 16, 4).to(DEV)
    obs = torch.randn(4096, 16, device=DEV)
    torch.manual_seed(11)
    a = pol.act(obs)
    torch.manual_seed(11)
    pol.update_distribution(obs)
    b = torch.normal(pol.distribution.loc, pol.distribution.scale)
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_l2c2_mix_matches_torch():
    """gr_l2c2_mix (PPOL2C2's mixed observations, ppo_l2c2.py:179-180) is bit-identical to the torch expression
    obs + w * (next - obs) on the same device, zero weights (a reset) and negative ones included."""
    from generalizableracing_amd.rsl_rl.ppo_l2c2 import _mix

    g = torch.Generator(device="cuda").manual_seed(11)
    for rows, cols in ((1, 4), (1000, 6928), (4097, 16)):
        o = torch.randn(rows, cols, device="cuda", generator=g)
        n = torch.randn(rows, cols, device="cuda", generator=g)
        w = (torch.rand(rows, 1, device="cuda", generator=g) - 0.5) * 2.0
        w[::5] = 0.0
        assert torch.equal(_mix(o, n, w), o + w * (n - o))
