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
