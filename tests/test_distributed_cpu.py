"""Data-parallel path on CPU: world_size 2 over gloo.

Each rank owns its own env shard (distinct env ids -> RNG streams, distinct
track seed); after PPO updates every rank must hold bit-identical parameters
(flat gradient all-reduce, rank-averaged KL for the adaptive LR, rank-0
broadcast at init), and advantage normalisation must use global statistics.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, algorithm="PPO"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import sys

        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.dirname(here), here, os.path.join(os.path.dirname(here), "oracle")]
        from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg
        from generalizableracing_amd.rsl_rl import distributed as gdist
        from oracle_vecenv import OracleVecEnv

        r, lr, ws = gdist.init_from_env("gloo")
        torch.manual_seed(100 + rank)  # different local init: rank 0's params must win the broadcast
        n = 32
        env = OracleVecEnv(num_envs=n, env_id_offset=rank * n, track_seed_offset=rank)
        cfg = QuadcopterPPORunnerCfg(device="cpu", num_steps_per_env=8)
        cfg.algorithm.class_name = algorithm
        cfg.policy.actor_hidden_dims = [16, 16]
        cfg.policy.critic_hidden_dims = [16, 16]
        runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device="cpu")
        runner.learn(2, init_at_random_ep_len=True)
        flat = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()])
        gathered = [torch.zeros_like(flat) for _ in range(ws)]
        dist.all_gather(gathered, flat)
        # global advantage statistics == statistics of the concatenation
        x = torch.randn(10 + 7 * rank, generator=torch.Generator().manual_seed(rank))
        m, s = gdist.global_mean_std(x)
        xs = [torch.randn(10 + 7 * k, generator=torch.Generator().manual_seed(k)) for k in range(ws)]
        cat = torch.cat(xs)
        obs0 = env.orc.obs_policy.copy()
        q.put((rank, all(torch.equal(gathered[0], g) for g in gathered),
               abs(float(m - cat.mean())) < 1e-6 and abs(float(s - cat.std())) < 1e-5,
               runner.alg.learning_rate, obs0[:4].tolist()))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced through the queue
        import traceback

        q.put((rank, "error", traceback.format_exc(), None, None))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("algorithm", ["PPO", "PPOL2C2"])
def test_two_rank_gloo_identical_updates(algorithm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, algorithm)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for r in res:
        assert r[1] != "error", r[2]
    assert all(r[1] for r in res), "parameters diverged across ranks"
    assert all(r[2] for r in res), "advantage statistics are not global"
    assert res[0][3] == res[1][3], "adaptive learning rates diverged"
    assert res[0][4] != res[1][4], "env shards should differ (env ids / track seeds)"


def _dp_alg(sl, n_total, T=8):
    """A PPO over the env columns `sl` of one seeded rollout of n_total envs (identical on every rank)."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl.ppo import PPO

    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [32, 32], [32, 32], "elu")
    g = torch.Generator().manual_seed(1)
    obs = torch.randn(T, n_total, 16, generator=g)
    cobs = torch.randn(T, n_total, 16, generator=g)
    last = torch.randn(n_total, 16, generator=g)
    with torch.no_grad():
        mu = pol.actor(obs)
        sigma = pol.std.expand_as(mu)
        act = mu + sigma * torch.randn(mu.shape, generator=g)
        logp = torch.distributions.Normal(mu, sigma).log_prob(act).sum(-1, keepdim=True)
        val = pol.critic(cobs)
    rew = torch.randn(T, n_total, 1, generator=g)
    done = (torch.rand(T, n_total, 1, generator=g) < 0.05).byte()
    alg = PPO(pol, num_learning_epochs=3, num_mini_batches=1, clip_param=0.2, gamma=0.99, lam=0.95,
              value_loss_coef=1.0, entropy_coef=0.005, learning_rate=5e-4, max_grad_norm=1.0,
              schedule="adaptive", desired_kl=0.01)
    n = sl.stop - sl.start
    alg.init_storage("rl", n, T, [16], [16], [4])
    st = alg.storage
    for name, x in (("observations", obs), ("privileged_observations", cobs), ("actions", act), ("rewards", rew),
                    ("dones", done), ("values", val), ("actions_log_prob", logp), ("mu", mu), ("sigma", sigma)):
        getattr(st, name).copy_(x[:, sl])
    st.step = T
    alg.compute_returns(last[sl])
    return alg


def _dp_worker(rank, world, port, q, n_total):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        import sys

        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [os.path.dirname(here), here]
        from generalizableracing_amd.rsl_rl import distributed as gdist

        gdist.init_from_env("gloo")
        per = n_total // world
        alg = _dp_alg(slice(rank * per, (rank + 1) * per), n_total)
        torch.manual_seed(7)
        out = alg.update()
        assert alg.flat_grads().bound()  # the gradients stayed views of the flat buffer (one in-place all-reduce)
        flat = torch.cat([p.detach().reshape(-1) for p in alg.policy.parameters()])
        q.put((rank, flat.tolist(), alg.learning_rate, out["value_function"]))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc(), None))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_dp_update_matches_single_rank(world):
    """k ranks, each holding 1/k of the envs, apply the update one rank computes on all of them: the
    gradient is averaged in one flat all-reduce, the KL mean and the advantage statistics are global (full
    mini-batches, so the shards' means average to the whole batch's)."""
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here)]
    n_total = 64
    ref = _dp_alg(slice(0, n_total), n_total)
    torch.manual_seed(7)
    out_ref = ref.update()
    want = torch.cat([p.detach().reshape(-1) for p in ref.policy.parameters()])
    moved = (want - torch.cat([p.detach().reshape(-1) for p in _dp_alg(slice(0, n_total), n_total).policy.parameters()]))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, world, port, q, n_total)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert r[1] != "error", r[2]
    for r in res:
        got = torch.tensor(r[1])
        assert (got - want).abs().max() <= 1e-3 * moved.abs().max(), (world, r[0], (got - want).abs().max())
        assert r[2] == ref.learning_rate
    assert all(torch.equal(torch.tensor(res[0][1]), torch.tensor(r[1])) for r in res)
