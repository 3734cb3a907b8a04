"""PPOL2C2 with algorithm.graph_update (ppo_l2c2._GraphedStepL2C2) on the reference's registered recipe (depth
camera + VisionActorCritic with the fused stem + PPOL2C2): the update's mini-batch steps captured once per epoch
and replayed must give the eager update's parameters, BatchNorm running statistics, learning rate and losses from
the same rollout, at the first call (capture) and the next (replay) (the running statistics, like the parameters,
within 5 % of how far the update moved them).

The smoothness loss's uniform draw is the one input the two cannot share (the graphs draw from torch's graph-safe
generator), so the comparison substitutes a fixed draw (u = 0.75: every mixed row 0.5 of the way to its successor)
in both; a second test keeps the real draw and holds the graphed update to the eager one's direction.  Tolerance as
tests/test_gpu_graph_update.py (fp32 device learning rate, another gradient accumulation order): parameters within
5 % of their movement (norms over all; 15 % per tensor, and the worst tensor within twice what a one-ulp perturbation
of the eager update itself produces), the value loss 1e-4 relative, the smoothness loss 2e-3, the surrogate 5e-5 (or
each within four times the one-ulp control's own difference).  Step by step: after
the first mini-batch step the flat gradient within 1e-5 and the parameters within 1e-6 of the eager loop's; Adam's
device step counters advance by exactly epochs x mini-batches (no step skipped or repeated).  Both the plain
storage layout and the observation-sink layout (T + 1 slots, the recipe's default) are covered."""
import copy
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner  # noqa: E402
from generalizableracing_amd.rsl_rl.config import QuadcopterVisionPPORunnerCfg  # noqa: E402
from generalizableracing_amd.rsl_rl.ppo_l2c2 import PPOL2C2  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _pair(n, steps, fixed_mix, obs_sink=False, per_step=False, control=False, also_per_step=False):
    """The eager algorithm (the runner's), a graph-captured copy (per_step: one graph per mini-batch step instead of
    one per epoch) and, with control, a second EAGER copy whose parameters are moved by one ulp (the round-off
    control); all three hold the same rollout.  obs_sink: the rollout is collected as the runner collects it with the
    observation sink (the env writes each transition's rows into storage slot t + 1; T + 1 slots), and the copies'
    storages take that layout too (sink flags included).  also_per_step: the control slot holds a graphed copy with
    per-step graphs instead (against the epoch-graph copy alg_g)."""
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV),
                                                    camera=CameraCfg())))
    cfg = QuadcopterVisionPPORunnerCfg(device=DEV, num_steps_per_env=steps)
    cfg.algorithm.obs_sink = obs_sink
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    assert runner.obs_sink == obs_sink
    alg = runner.alg
    kw = dict(cfg.to_dict()["algorithm"])
    kw.pop("class_name")
    kw.pop("obs_sink", None)
    od = env.num_obs

    def copy_alg(graph_update, step_graphs=per_step):
        a = PPOL2C2(copy.deepcopy(alg.policy), device=DEV, **dict(kw, graph_update=graph_update,
                                                                 graph_update_per_step=step_graphs and graph_update))
        a.init_storage("rl", n, steps, [od], [od], [4])
        if obs_sink:
            a.storage.enable_obs_sink()
        return a

    alg_g = copy_alg(True)
    alg_c = copy_alg(False) if control else copy_alg(True, True) if also_per_step else None
    copies = [a for a in (alg_g, alg_c) if a is not None]
    if fixed_mix:
        for a in [alg] + copies:
            a._mix_uniform = lambda c: torch.full_like(c, 0.75)
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    st = alg.storage
    if obs_sink:
        st.discard_sink()
    with torch.inference_mode():
        for _ in range(steps):
            a = alg.act(obs, cobs)
            if obs_sink:  # (as OnPolicyRunner.learn: this step's rows land in the next transition's slot)
                env.set_obs_sink(*st.sink_slot(st.step + 1))
            obs, rew, dones, infos = env.step(a)
            cobs = infos["observations"]["critic"]
            alg.process_env_step(rew, dones, infos)
        if obs_sink:
            env.set_obs_sink(None)
        alg.compute_returns(cobs)
    if obs_sink:
        assert st.observations.shape[0] == steps + 1 and st.prefilled[steps]
    for c in copies:
        for name, v in vars(st).items():
            if torch.is_tensor(v):
                getattr(c.storage, name).copy_(v)
        c.storage.prefilled = list(st.prefilled)
        # (the rollout's train-mode forwards moved the BatchNorm running statistics of the eager policy)
        c.policy.load_state_dict(alg.policy.state_dict())
    if control:
        with torch.no_grad():  # one ulp away from the eager parameters (toward +inf; zeros stay zero)
            for p in alg_c.policy.parameters():
                p.copy_(torch.where(p != 0, torch.nextafter(p, torch.full_like(p, float("inf"))), p))
    return env, alg, alg_g, alg_c


def _buffers(pol):
    return {k: v for k, v in pol.state_dict().items() if "running" in k or "num_batches" in k}


def _adam_steps(alg):
    """Adam's per-parameter step counts (FlatAdam keeps them on the device, written by every captured step)."""
    return {i: float(alg.optimizer.state[p]["step"]) if alg.optimizer.state[p] else 0.0
            for i, p in enumerate(alg.policy.parameters()) if p.grad is not None}


def _sync(src, dst):
    """dst takes src's parameters, Adam moments and step counts, BatchNorm statistics and learning rate."""
    with torch.no_grad():
        for pe, pg in zip(src.policy.parameters(), dst.policy.parameters()):
            pg.copy_(pe)
            se, sg = src.optimizer.state[pe], dst.optimizer.state[pg]
            if not se:  # (a parameter the loss does not reach: no gradient, no eager Adam state; the graphed
                # update's zero-gradient first step gave it zero moments, never stepped again)
                assert not sg or float(sg["exp_avg"].abs().max()) == 0.0
                continue
            for key in ("exp_avg", "exp_avg_sq", "step"):
                sg[key].copy_(se[key])
        for k, v in _buffers(src.policy).items():
            dst.policy.state_dict()[k].copy_(v)
    dst.learning_rate = src.learning_rate


def _divergence(alg, other, p0):
    """Per parameter tensor: (name, |other - eager|, |eager - start|) after an update (norms)."""
    out = []
    for (name, pe), po, q in zip(alg.policy.named_parameters(), other.policy.parameters(), p0):
        out.append((name, float((pe.detach() - po.detach()).norm()), float((pe.detach() - q).norm())))
    return out


@pytest.mark.parametrize("obs_sink", [False, True])
def test_graphed_l2c2_update_matches_eager(obs_sink):
    """The whole update, at the first call (capture) and the next (replay), the epoch graph against the eager loop.
    Adam's device step counters advance by exactly num_learning_epochs x num_mini_batches in both (the epoch graph
    replays every mini-batch step once, no more, no fewer).

    A whole update is 20 Adam steps of a chaotic map (a bias element whose gradient sums to ~0 takes an lr-sized step
    whose sign is round-off), so the bound is measured, not assumed: a control copy runs the EAGER update again
    from parameters one ulp away, and the graphed update's worst tensor must stay within twice the control's worst
    divergence (+1 %), every tensor within 15 % of its movement and all together within 5 % (printed).
    The step-level tie is test_graphed_l2c2_first_step_matches_eager."""
    torch.manual_seed(3)
    n, steps = 512, 8
    env, alg, alg_g, alg_c = _pair(n, steps, fixed_mix=True, obs_sink=obs_sink, control=True)
    assert alg.policy.fused_bn
    nsteps = alg.num_learning_epochs * alg.num_mini_batches
    for rep in range(2):  # capture, then replay
        st_state = list(alg.storage.prefilled)
        for a in (alg, alg_g, alg_c):
            a.storage.step = steps
            a.storage.prefilled = list(st_state)
        p0 = [p.detach().clone() for p in alg.policy.parameters()]
        b0 = {k: v.clone() for k, v in _buffers(alg.policy).items()}
        s0e, s0g = _adam_steps(alg), _adam_steps(alg_g)
        le, lg, lc = [], [], []
        for a, out in ((alg, le), (alg_g, lg), (alg_c, lc)):
            torch.manual_seed(7 + rep)
            out.append(a.update())
        le, lg, lc = le[0], lg[0], lc[0]
        # the device step counters: every mini-batch step ran exactly once
        s1e, s1g = _adam_steps(alg), _adam_steps(alg_g)
        assert set(s1e) == set(s1g) and len(s1e) >= len(p0) - 3
        for i in s1e:
            assert s1e[i] - s0e.get(i, 0.0) == nsteps, (rep, i, s0e.get(i), s1e[i])
            assert s1g[i] - s0g.get(i, 0.0) == nsteps, (rep, i, s0g.get(i), s1g[i])
            assert s1g[i] == s1e[i]
        div_g, div_c = _divergence(alg, alg_g, p0), _divergence(alg, alg_c, p0)
        worst_g = sorted(((d / m if m else 0.0), name) for name, d, m in div_g)[-3:]
        worst_c = sorted(((d / m if m else 0.0), name) for name, d, m in div_c)[-3:]
        print(f"obs_sink={obs_sink} rep={rep}: graphed-vs-eager worst {worst_g}; one-ulp eager control worst {worst_c}")
        # measured: graphed-vs-eager worst tensor 1.2 % / 2.2 % of its movement against a one-ulp eager control of 3.5 % /
        # 5.5 % (gpurun_out/r6b), and on another rollout draw 7.6 % against 11 % (r6r): the update's own round-off
        # sensitivity exceeds the graphed path's difference and depends on the data, so the graphed update is held to
        # the control (worst tensor within 2x the control's + 1 %) and to 15 % per tensor
        assert worst_g[-1][0] <= 2.0 * worst_c[-1][0] + 0.01, (rep, worst_g, worst_c)
        per_tensor = 0.15
        n_moved, tot_moved, tot_diff = 0, 0.0, 0.0
        for name, diff, moved in div_g:
            # (the conv biases ahead of a BatchNorm get no gradient: those stay put in both)
            assert diff <= per_tensor * moved, (rep, name, diff, moved)
            n_moved += moved > 0.0
            tot_moved += moved * moved
            tot_diff += diff * diff
        assert n_moved >= len(p0) - 3, (n_moved, len(p0))
        assert tot_diff <= 0.05 ** 2 * tot_moved, (rep, tot_diff ** 0.5, tot_moved ** 0.5)
        be, bg, bc = _buffers(alg.policy), _buffers(alg_g.policy), _buffers(alg_c.policy)
        assert set(be) == set(bg) and len(be) >= 9
        bad = []
        for k in be:
            if "num_batches" in k:
                if not torch.equal(be[k], bg[k]):
                    bad.append((k, int(be[k]), int(bg[k])))
            else:
                # as the parameters: within 5 % of how far the update moved them, or within twice the one-ulp
                # control's difference (+1 %): the statistics are taken with the chaotic parameters (r6v:
                # stem.4.running_var at 7 % of its movement)
                moved, diff = float((be[k] - b0[k]).norm()), float((bg[k] - be[k]).norm())
                ctrl = float((bc[k] - be[k]).norm())
                if not (moved > 0.0 and diff <= max(0.05 * moved, 2.0 * ctrl + 0.01 * moved)):
                    bad.append((k, diff, moved))
        assert not bad, (rep, bad)
        assert abs(alg.learning_rate - alg_g.learning_rate) <= 1e-6 * alg.learning_rate
        # the losses: within fixed bounds (value 1e-4 relative, smoothness 2e-3 relative (a mean of squared distances
        # between two nearly equal policy outputs, ~1e-3), surrogate 5e-5) or within four times what the one-ulp control
        # moved them (the later mini-batches' round-off, amplified as above, shows in them too; the control is one
        # sample of that spread: on rollout r6t the smoothness loss moved 2.1x the control's)
        for key, fixed in (("value_function", 1e-4 * abs(le["value_function"])),
                           ("smooth_loss", 2e-3 * abs(le["smooth_loss"])), ("surrogate", 5e-5)):
            assert abs(le[key] - lg[key]) <= max(fixed, 4.0 * abs(le[key] - lc[key])), (rep, key, le, lg, lc)
        if obs_sink:  # (the last observations opened the next rollout in both, slot T into slot 0)
            assert alg_g.storage.prefilled == alg.storage.prefilled
            assert torch.equal(alg_g.storage.observations, alg.storage.observations)
        _sync(alg, alg_g)  # the next update starts from identical states
        _sync(alg, alg_c)
        with torch.no_grad():
            for p in alg_c.policy.parameters():
                p.copy_(torch.where(p != 0, torch.nextafter(p, torch.full_like(p, float("inf"))), p))
    assert alg_g._graphed is not None and alg_g._graphed.graph is not None and not alg_g._graphed.per_step
    # (the row indices the graphed steps read the storage through stay inside it: successors at + N)
    gs = alg_g._graphed
    assert int(gs.perm.max()) + gs.N < alg_g.storage.observations.shape[0] * gs.N
    env.close()


class _Stop(Exception):
    pass


class _OneReplay:
    """A captured graph that replays once more and then stops the update (the state after ONE mini-batch step)."""

    def __init__(self, graph):
        self.graph = graph

    def replay(self):
        self.graph.replay()
        raise _Stop


def test_graphed_l2c2_first_step_matches_eager():
    """The graphed mini-batch step tied to the eager one step by step: after the FIRST mini-batch step of an update
    (per-step graphs: the same captured operations as the epoch graph, one step per replay), the flat gradient
    (after the clip, which both apply in place) within 1e-5 relative and every parameter tensor after the Adam step
    within 1e-6 relative of the eager loop's.  Taken at the second update, after a full first one on both and a
    state sync (Adam moments warm: a fresh first step is lr * sign(g), see the whole-update test)."""
    torch.manual_seed(5)
    n, steps = 512, 8
    env, alg, alg_g, _ = _pair(n, steps, fixed_mix=True, per_step=True)
    for a in (alg, alg_g):
        a.storage.step = steps
    torch.manual_seed(7)
    alg.update()
    torch.manual_seed(7)
    alg_g.update()
    gs = alg_g._graphed
    assert gs is not None and gs.per_step and gs.graph_b is None
    _sync(alg, alg_g)
    for a in (alg, alg_g):
        a.storage.step = steps
    real_step = alg.optimizer.step

    def one_step(*args, **kw):
        real_step(*args, **kw)
        raise _Stop

    alg.optimizer.step = one_step
    torch.manual_seed(8)
    with pytest.raises(_Stop):
        alg.update()
    del alg.optimizer.step
    gs.graph = _OneReplay(gs.graph)
    torch.manual_seed(8)
    with pytest.raises(_Stop):
        alg_g.update()
    gs.graph = gs.graph.graph
    torch.cuda.synchronize()
    fe, fg = alg.flat_grads(), gs.flat
    # the gradients over the parameters the loss reaches (the flat buffers' views, in the same order; the trailing KL
    # slot only the graphed step writes)
    assert len(fe.views) == len(fg.views) and fe.flat.numel() == fg.flat.numel()
    n_used = fe.flat.numel() - fe.extra.numel()
    ge, gg = fe.flat[:n_used].double(), fg.flat[:n_used].double()
    assert float(ge.abs().max()) > 0.0
    rel_g = float((ge - gg).abs().max() / ge.abs().max())
    worst = []
    for (name, pe), pg in zip(alg.policy.named_parameters(), alg_g.policy.parameters()):
        rel = float((pe.detach().double() - pg.detach().double()).abs().max()
                    / pe.detach().double().abs().max().clamp_min(1e-30))
        worst.append((rel, name))
    worst.sort()
    print(f"first mini-batch step: flat gradient rel {rel_g:.3g}; parameters worst {worst[-3:]}")
    assert rel_g <= 1e-5, rel_g
    assert worst[-1][0] <= 1e-6, worst[-3:]
    env.close()


def test_l2c2_epoch_graph_equals_per_step_graph_bitwise():
    """The default graphed L2C2 update (one graph per epoch, each mini-batch step on its slice of the permutation) and
    one graph per mini-batch step (graph_update_per_step, the form test_graphed_l2c2_first_step_matches_eager ties to
    the eager loop step by step) run the same kernels in the same order: parameters, BatchNorm statistics, Adam
    moments and step counts and losses identical bit for bit, at capture and at replay (fixed mix draw)."""
    torch.manual_seed(6)
    n, steps = 512, 8
    env, alg, alg_e, alg_s = _pair(n, steps, fixed_mix=True, also_per_step=True)

    def state(a):
        sd = a.optimizer.state_dict()
        return ([p.detach() for p in a.policy.parameters()] + list(_buffers(a.policy).values())
                + [t for st in sd["state"].values() for t in st.values() if torch.is_tensor(t)])

    for rep in range(2):
        for a in (alg_e, alg_s):
            a.storage.step = steps
        torch.manual_seed(13 + rep)
        le = alg_e.update()
        torch.manual_seed(13 + rep)
        ls = alg_s.update()
        assert not alg_e._graphed.per_step and alg_s._graphed.per_step
        assert le == ls, (rep, le, ls)
        for x, y in zip(state(alg_e), state(alg_s)):
            assert torch.equal(x, y), rep
        assert alg_e.learning_rate == alg_s.learning_rate
    env.close()


def test_graphed_l2c2_update_draws_fresh_uniforms():
    """With the real draw the graphed steps take their uniforms from torch's graph-safe generator: every replayed
    mini-batch step draws anew (four distinct draws per epoch graph, new ones on the next update), uniform on
    [0, 1); the losses stay finite and the value loss near the eager update's."""
    torch.manual_seed(4)
    n, steps = 512, 8
    env, alg, alg_g, _ = _pair(n, steps, fixed_mix=False)
    nmb, mb = alg_g.num_mini_batches, (steps - 1) * n // alg_g.num_mini_batches
    rec = torch.zeros(nmb, mb, device=DEV)
    calls = [0]

    def recorder(c):
        u = torch.rand_like(c)
        rec[calls[0] % nmb].copy_(u.reshape(-1))
        calls[0] += 1
        return u

    alg_g._mix_uniform = recorder
    seen = []
    for rep in range(2):
        alg_g.storage.step = alg.storage.step = steps
        le = alg.update()
        lg = alg_g.update()
        assert all(torch.isfinite(torch.tensor(list(lg.values())))), lg
        assert abs(le["value_function"] - lg["value_function"]) <= 0.05 * abs(le["value_function"]), (le, lg)
        r = rec.clone()
        assert float(r.min()) >= 0.0 and float(r.max()) < 1.0
        assert abs(float(r.mean()) - 0.5) < 0.02
        for i in range(nmb):
            for j in range(i):
                assert not torch.equal(r[i], r[j]), (rep, i, j)
        for prev in seen:
            assert not torch.equal(prev, r), rep
        seen.append(r)
    env.close()
