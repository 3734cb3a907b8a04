"""The graph-captured PPO update at world size > 1 (ppo.py _GraphedStep, segmented form): segment A (forward, KL,
losses, backward into the flat gradient buffer) and segment B (learning-rate rule, clip, Adam) are two hipGraphs and
the exchange (ONE in-place all-reduce of the flat buffer: gradients + KL mean) runs eagerly between them, so no
collective is ever captured.

1. On one rank the segmented form equals the single graph (same kernels, same order).
2. Two gloo ranks sharing the one GPU of the test box, each holding half of a rollout, apply the update one rank
   computes eagerly on the whole rollout (reference arithmetic: ppo.py:103-190), at the capture and at the replay,
   and hold identical parameters and learning rates."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

T = 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rollout(n_total, act="elu"):
    """One seeded synthetic rollout (identical in every process), on the CPU.  act="lrelu": the MLPs take the
    fused device path of the update (rsl_rl/linear.py MLP) on the GPU."""
    from generalizableracing_amd.rsl_rl import ActorCritic

    torch.manual_seed(0)
    pol = ActorCritic(16, 16, 4, [64, 64], [64, 64], act)
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
    data = dict(observations=obs, privileged_observations=cobs, actions=act, rewards=rew, dones=done, values=val,
                actions_log_prob=logp, mu=mu, sigma=sigma)
    return pol, data, last


def _alg(sl, n_total, device, act="elu", **kw):
    from generalizableracing_amd.rsl_rl.ppo import PPO

    pol, data, last = _rollout(n_total, act)
    alg = PPO(pol, device=device, num_learning_epochs=3, num_mini_batches=1, clip_param=0.2, gamma=0.99, lam=0.95,
              value_loss_coef=1.0, entropy_coef=0.005, learning_rate=5e-4, max_grad_norm=1.0, schedule="adaptive",
              desired_kl=0.01, **kw)
    n = sl.stop - sl.start
    alg.init_storage("rl", n, T, [16], [16], [4])
    return alg, data, last, sl


def _fill(alg, data, last, sl):
    st = alg.storage
    with torch.no_grad():  # (as the runner's rollout: the storage is written outside autograd)
        for name, x in data.items():
            getattr(st, name).copy_(x[:, sl].to(st.observations.device))
        st.step = T
        alg.compute_returns(last[sl].to(st.observations.device))


def _params(alg):
    return torch.cat([p.detach().reshape(-1).cpu() for p in alg.policy.parameters()])


def _updates(alg, data, last, sl, reps=2):
    out = []
    for rep in range(reps):  # capture, then replay
        _fill(alg, data, last, sl)
        torch.manual_seed(7 + rep)
        alg.update()
        out.append((_params(alg), alg.learning_rate))
    return out


@pytest.mark.parametrize("act", ["elu", "lrelu"])
def test_segmented_equals_single_graph(act):
    n = 512
    res = []
    for seg in (False, True):
        alg, data, last, sl = _alg(slice(0, n), n, "cuda:0", act, graph_update=True, graph_update_segmented=seg)
        res.append(_updates(alg, data, last, sl))
        assert (alg._graphed.graph_b is not None) is seg
    p0 = _params(_alg(slice(0, n), n, "cpu", act)[0])
    for (pa, la), (pb, lb) in zip(*res):
        moved = float((pa - p0).abs().max())
        assert moved > 0 and float((pa - pb).abs().max()) <= 1e-6 * moved
        assert la == lb


def _worker(rank, world, port, q, n_total, act):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    try:
        sys.path.insert(0, ROOT)
        from generalizableracing_amd.rsl_rl import distributed as gdist

        gdist.init_from_env("gloo")
        per = n_total // world
        alg, data, last, sl = _alg(slice(rank * per, (rank + 1) * per), n_total, "cuda:0", act, graph_update=True)
        out = _updates(alg, data, last, sl)
        assert alg._graphed.segmented and alg._graphed.graph_b is not None
        q.put((rank, [(p.tolist(), lr) for p, lr in out]))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover - surfaced through the queue
        import traceback

        q.put((rank, "error:" + traceback.format_exc()))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("act", ["elu", "lrelu"])
def test_two_gloo_ranks_graphed_update_matches_single_rank(act):
    n_total = 1024
    ref, data, last, sl = _alg(slice(0, n_total), n_total, "cpu", act)
    p0 = _params(ref)
    want = _updates(ref, data, last, sl)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, n_total, act)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=280) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not isinstance(v, str), v
    for rep, (wp, wl) in enumerate(want):
        # norms: Adam turns the round-off of a near-zero gradient element (CPU reference vs GPU shards) into an
        # update of up to a learning rate, so single elements may differ by that much
        moved = float((wp - p0).norm())
        got = [torch.tensor(res[r][rep][0]) for r in range(2)]
        assert torch.equal(got[0], got[1]), rep  # the ranks stay bit-identical
        assert float((got[0] - wp).norm()) <= 1e-2 * moved, (rep, float((got[0] - wp).norm()), moved)
        assert res[0][rep][1] == res[1][rep][1]
        assert abs(res[0][rep][1] - wl) <= 1e-6 * wl, (rep, res[0][rep][1], wl)
