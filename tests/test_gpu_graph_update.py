"""PPO update with algorithm.graph_update (ppo.py _GraphedStep): the mini-batch step captured once in a
hipGraph and replayed must give the eager update's parameters, learning rate and losses from the same
rollout, at the first call (capture) and the next (replay).  Tolerance: fp32 round-off.  The learning
rate lives in an fp32 device tensor instead of a Python float, and Adam's capturable path forms its
bias corrections from device tensors: over the 20 Adam steps of an update the parameters agree to
~2 % of the update itself (measured 8e-6 on parameters of scale 0.25 moved by ~5e-4 per step)."""
import copy
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg  # noqa: E402
from generalizableracing_amd.rsl_rl.ppo import PPO  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_graphed_update_matches_eager():
    torch.manual_seed(3)
    n = 2048
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV)
    cfg.algorithm.obs_sink = False  # the storages are copied slot for slot
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    alg = runner.alg
    kw = dict(cfg.to_dict()["algorithm"])
    kw.pop("class_name")
    kw["graph_update"] = True
    alg_g = PPO(copy.deepcopy(alg.policy), device=DEV, **kw)
    alg_g.init_storage("rl", n, cfg.num_steps_per_env, [16], [16], [4])
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    with torch.inference_mode():
        for _ in range(cfg.num_steps_per_env):
            a = alg.act(obs, cobs)
            obs, rew, dones, infos = env.step(a)
            cobs = infos["observations"]["critic"]
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(cobs)
    for name, v in vars(alg.storage).items():
        if torch.is_tensor(v):
            getattr(alg_g.storage, name).copy_(v)
    for rep in range(2):  # capture, then replay
        alg_g.storage.step = alg.storage.step = cfg.num_steps_per_env
        p0 = [p.detach().clone() for p in alg.policy.parameters()]
        torch.manual_seed(7 + rep)
        le = alg.update()
        torch.manual_seed(7 + rep)
        lg = alg_g.update()
        for pe, pg, q in zip(alg.policy.parameters(), alg_g.policy.parameters(), p0):
            moved = float((pe.detach() - q).abs().max())
            diff = float((pe.detach() - pg.detach()).abs().max())
            assert moved > 0.0 and diff <= 0.05 * moved, (rep, diff, moved)
        assert abs(alg.learning_rate - alg_g.learning_rate) <= 1e-6 * alg.learning_rate
        assert abs(le["value_function"] - lg["value_function"]) <= 1e-4 * abs(le["value_function"])
        # the surrogate is a nearly cancelling mean of +-A * ratio (|A| ~ 1, mean ~ 0.02) over 20 mini-batches
        # whose parameters differ by up to the 5 % above: an absolute bound, as tests/ppo_c2_golden.py's
        assert abs(le["surrogate"] - lg["surrogate"]) <= 5e-5, (le["surrogate"], lg["surrogate"])
        # the next update (graph replay) starts from identical states: round-off differences would
        # otherwise grow through Adam's normalisation of near-zero gradients
        with torch.no_grad():
            for pe, pg in zip(alg.policy.parameters(), alg_g.policy.parameters()):
                pg.copy_(pe)
                se, sg = alg.optimizer.state[pe], alg_g.optimizer.state[pg]
                for key in ("exp_avg", "exp_avg_sq", "step"):
                    sg[key].copy_(se[key])
        alg_g.learning_rate = alg.learning_rate
    assert alg_g._graphed is not None and alg_g._graphed.graph is not None


def test_bf16_autocast_update_follows_fp32():
    """algorithm.update_autocast_bf16 (with the graphed step): not the reference's fp32 arithmetic, so held
    to the fp32 update's direction: per parameter tensor, the cosine between the two updates > 0.9, and
    the same adaptive learning rate."""
    torch.manual_seed(4)
    n = 4096
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV)
    cfg.algorithm.obs_sink = False  # the storages are copied slot for slot
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    alg = runner.alg
    kw = dict(cfg.to_dict()["algorithm"])
    kw.pop("class_name")
    kw.update(graph_update=True, update_autocast_bf16=True)
    alg_b = PPO(copy.deepcopy(alg.policy), device=DEV, **kw)
    alg_b.init_storage("rl", n, cfg.num_steps_per_env, [16], [16], [4])
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    with torch.inference_mode():
        for _ in range(cfg.num_steps_per_env):
            a = alg.act(obs, cobs)
            obs, rew, dones, infos = env.step(a)
            cobs = infos["observations"]["critic"]
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(cobs)
    for name, v in vars(alg.storage).items():
        if torch.is_tensor(v):
            getattr(alg_b.storage, name).copy_(v)
    p0 = [p.detach().clone() for p in alg.policy.parameters()]
    torch.manual_seed(9)
    le = alg.update()
    torch.manual_seed(9)
    lb = alg_b.update()
    for pe, pb, q in zip(alg.policy.parameters(), alg_b.policy.parameters(), p0):
        de, db = (pe.detach() - q).flatten(), (pb.detach() - q).flatten()
        cos = float(torch.dot(de, db) / (de.norm() * db.norm() + 1e-20))
        assert cos > 0.9, cos
    assert all(torch.isfinite(torch.tensor(list(lb.values()))))
    assert abs(le["value_function"] - lb["value_function"]) <= 0.05 * abs(le["value_function"])


def test_graphed_update_across_iterations():
    """Three rollout + compute_returns + update iterations, graphed vs eager, each on its own storage.
    compute_returns runs on the graphed algorithm's storage every iteration, so a graph whose gathers
    were baked against an earlier iteration's advantages / returns allocation would read stale data
    (the surrogate loss then disagrees from the second iteration on)."""
    torch.manual_seed(5)
    n = 2048
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV)
    cfg.algorithm.obs_sink = False  # the storages are copied slot for slot
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    alg = runner.alg
    kw = dict(cfg.to_dict()["algorithm"])
    kw.pop("class_name")
    kw["graph_update"] = True
    alg_g = PPO(copy.deepcopy(alg.policy), device=DEV, **kw)
    alg_g.init_storage("rl", n, cfg.num_steps_per_env, [16], [16], [4])
    raw = ("observations", "privileged_observations", "actions", "rewards", "dones", "values",
           "actions_log_prob", "mu", "sigma")
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    adv_ptr = alg_g.storage.advantages.data_ptr()
    for it in range(3):
        with torch.inference_mode():
            for _ in range(cfg.num_steps_per_env):
                a = alg.act(obs, cobs)
                obs, rew, dones, infos = env.step(a)
                cobs = infos["observations"]["critic"]
                alg.process_env_step(rew, dones, infos)
            alg.compute_returns(cobs)
            for name in raw:
                getattr(alg_g.storage, name).copy_(getattr(alg.storage, name))
            alg_g.storage.step = cfg.num_steps_per_env
            alg_g.compute_returns(cobs)
        assert alg_g.storage.advantages.data_ptr() == adv_ptr  # written in place every iteration
        torch.testing.assert_close(alg_g.storage.advantages, alg.storage.advantages, rtol=1e-5, atol=1e-5)
        p0 = [p.detach().clone() for p in alg.policy.parameters()]
        torch.manual_seed(11 + it)
        le = alg.update()
        torch.manual_seed(11 + it)
        lg = alg_g.update()
        for pe, pg, q in zip(alg.policy.parameters(), alg_g.policy.parameters(), p0):
            # norms, not maxima: Adam turns the round-off of a near-zero gradient element into an update of
            # up to lr in either direction, so single elements may differ by a learning rate
            moved = float((pe.detach() - q).norm())
            diff = float((pe.detach() - pg.detach()).norm())
            assert moved > 0.0 and diff <= 0.05 * moved, (it, diff, moved)
        assert abs(le["value_function"] - lg["value_function"]) <= 1e-4 * abs(le["value_function"]), (it, le, lg)
        # the surrogate is a mean of +-A * ratio over normalised advantages (|A| ~ 1) that nearly cancels
        # (~0.01): the < 5 % parameter round-off of the later mini-batches shows in it at ~1e-5 absolute,
        # while a stale advantages buffer would change it at the scale of the terms themselves
        assert abs(le["surrogate"] - lg["surrogate"]) <= 2e-3 * abs(le["surrogate"]) + 5e-5, (it, le, lg)
        with torch.no_grad():
            for pe, pg in zip(alg.policy.parameters(), alg_g.policy.parameters()):
                pg.copy_(pe)
                se, sg = alg.optimizer.state[pe], alg_g.optimizer.state[pg]
                for key in ("exp_avg", "exp_avg_sq", "step"):
                    sg[key].copy_(se[key])
        alg_g.learning_rate = alg.learning_rate


def test_graphed_checkpoint_loads_into_torch_adam(tmp_path):
    """after a graphed update (FlatAdam's group holds the rate as a device tensor) a checkpoint's
    optimizer state must load into a plain torch.optim.Adam — what the reference runner does on resume
    (on_policy_runner.py:319) — and step it; and resume into FlatAdam with the same moments."""
    from generalizableracing_amd.rsl_rl.flat_adam import FlatAdam

    torch.manual_seed(6)
    n = 1024
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV, num_steps_per_env=8)
    cfg.algorithm.graph_update = True
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    runner.learn(2)
    alg = runner.alg
    assert isinstance(alg.optimizer, FlatAdam) and torch.is_tensor(alg.optimizer.param_groups[0]["lr"])
    path = tmp_path / "model.pt"
    runner.save(str(path))
    ck = torch.load(str(path), weights_only=True)
    osd = ck["optimizer_state_dict"]
    g = osd["param_groups"][0]
    assert isinstance(g["lr"], float) and g["capturable"] is False
    for st in osd["state"].values():
        assert st["step"].device.type == "cpu" and st["step"].dim() == 0 and float(st["step"]) >= 1
    pol = copy.deepcopy(alg.policy)
    adam = torch.optim.Adam(pol.parameters(), lr=1e-3)
    adam.load_state_dict(copy.deepcopy(osd))  # (torch Adam adopts the loaded tensors and steps them in place)
    for p in pol.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    adam.step()  # the first foreach step raised 'lr as a Tensor is not supported' before the fix
    assert all(torch.isfinite(p).all() for p in pol.parameters())
    # and back into FlatAdam: same moments and step counts
    fa = FlatAdam(list(alg.policy.parameters()), lr=1e-3)
    fa.load_state_dict(osd)
    for p, q in zip(alg.policy.parameters(), fa.param_groups[0]["params"]):
        s0, s1 = alg.optimizer.state[p], fa.state[q]
        assert torch.equal(s0["exp_avg"], s1["exp_avg"]) and torch.equal(s0["exp_avg_sq"], s1["exp_avg_sq"])
        assert float(s0["step"]) == float(s1["step"])
    env.close()


def test_flat_adam_clip_keeps_nan_like_torch():
    """a non-finite gradient makes torch's clip coefficient NaN and clip_grad_norm_ turns every gradient
    NaN; FlatAdam's clip must fail the same way (not leave the finite tensors unscaled)."""
    from generalizableracing_amd.rsl_rl.flat_adam import FlatAdam

    torch.manual_seed(1)
    ps = [torch.nn.Parameter(torch.randn(300, device=DEV)) for _ in range(3)]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, q in zip(ps, qs):
        p.grad = torch.randn_like(p)
        q.grad = p.grad.clone()
    ps[1].grad[7] = float("nan")
    qs[1].grad[7] = float("nan")
    fa = FlatAdam(ps, lr=1e-3)
    n_fa = fa.clip_grad_norm_(1.0)
    n_t = torch.nn.utils.clip_grad_norm_(qs, 1.0)
    torch.cuda.synchronize()
    assert torch.isnan(n_fa) and torch.isnan(n_t)
    for p, q in zip(ps, qs):
        assert torch.isnan(p.grad).all() and torch.isnan(q.grad).all()


def test_epoch_graph_equals_per_step_graph_bitwise():
    """The default graphed update (one graph per epoch, every mini-batch step on its slice of the permutation) runs
    the same kernels in the same order as one graph per mini-batch step (graph_update_per_step): parameters, Adam
    moments and step counts, learning rate and losses are identical bit for bit, at capture and at replay."""
    torch.manual_seed(5)
    n = 2048
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV))))
    cfg = QuadcopterPPORunnerCfg(device=DEV)
    cfg.algorithm.obs_sink = False
    cfg.algorithm.graph_update = True
    runner = OnPolicyRunner(env, cfg.to_dict(), log_dir=None, device=DEV)
    alg = runner.alg
    kw = dict(cfg.to_dict()["algorithm"])
    kw.pop("class_name")
    kw["graph_update_per_step"] = True
    alg_s = PPO(copy.deepcopy(alg.policy), device=DEV, **kw)
    alg_s.init_storage("rl", n, cfg.num_steps_per_env, [16], [16], [4])
    obs, extras = env.get_observations()
    cobs = extras["observations"]["critic"]
    with torch.inference_mode():
        for _ in range(cfg.num_steps_per_env):
            a = alg.act(obs, cobs)
            obs, rew, dones, infos = env.step(a)
            cobs = infos["observations"]["critic"]
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(cobs)
    for name, v in vars(alg.storage).items():
        if torch.is_tensor(v):
            getattr(alg_s.storage, name).copy_(v)

    def state_tensors(a):
        sd = a.optimizer.state_dict()
        out = [t for st in sd["state"].values() for t in st.values() if torch.is_tensor(t)]
        return [p.detach() for p in a.policy.parameters()] + out

    for rep in range(2):  # capture, then replay
        alg_s.storage.step = alg.storage.step = cfg.num_steps_per_env
        torch.manual_seed(11 + rep)
        le = alg.update()
        torch.manual_seed(11 + rep)
        ls = alg_s.update()
        assert not alg._graphed.per_step and alg_s._graphed.per_step
        te, ts = state_tensors(alg), state_tensors(alg_s)
        assert len(te) == len(ts) > 8
        for k, (x, y) in enumerate(zip(te, ts)):
            assert torch.equal(x, y), (rep, k)
        assert alg.learning_rate == alg_s.learning_rate
        assert le == ls, (le, ls)
    env.close()
