"""The HIP kernels with every random draw on, against the reference's own startup-DR, reset, command and observation
code fed the same draws (tests/golden/make_golden_noise.py; comparisons in tests/noise_golden.py): gr_init's startup
domain randomisation, gr_reset of every env (pose facing the start gate, drag DR, thrust error, curriculum, the
resampled noisy gates, the noisy observation), and one gr_step in which envs pass their gates (the update's new gate
noise, the observation noise).  Also bit for bit against the oracle."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import noise_golden as NG  # noqa: E402
import oracle  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv  # noqa: E402

DEV = "cuda:0"


def _env(n):
    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=1,
                                 terrain=TerrainCfg(obstacles=False)))
    g = env.gr_config
    assert g.obs_noise and g.add_gate_noise and g.dr_startup and g.random_drag
    return env


def _load(env, e, cnt):
    st, ist = oracle.envs_to_planes(e, env.state.shape[0])
    env.state.copy_(torch.from_numpy(st).to(DEV))
    env.istate.copy_(torch.from_numpy(ist).to(DEV))
    env._counters.fill_(cnt)


def _kernel_envs(env):
    torch.cuda.synchronize()
    return oracle.planes_to_envs(env.state.cpu().numpy(), env.istate.cpu().numpy())


def test_kernel_startup_dr_matches_reference():
    g, _ = NG.load()
    env = _env(g["S_Kp"].shape[0])
    e = _kernel_envs(env)
    NG.check_startup(g, e)
    orc = oracle.from_env(env)
    orc.init()
    for k in NG.startup_fields():
        assert np.array_equal(np.ascontiguousarray(e[k]).view(np.uint32),
                              np.ascontiguousarray(orc.envs[k]).view(np.uint32)), k
    env.close()


def test_kernel_reset_draws_match_reference():
    g, _ = NG.load()
    pre, prev_crit, cnt = NG.reset_pre(g)
    env = _env(len(pre))
    _load(env, pre, cnt)
    obs, _ = env.reset()
    e = _kernel_envs(env)
    pol, cri = obs["policy"].cpu().numpy(), obs["critic"].cpu().numpy()
    NG.check_reset(g, e, pol, cri)
    orc = oracle.from_env(env)
    orc.envs[:] = pre
    orc.obs_critic[:] = prev_crit
    orc.counter[0] = cnt
    orc.reset(None)
    assert np.array_equal(pol[:, :12].view(np.uint32), orc.obs_policy[:, :12].view(np.uint32))
    for k in ("p", "q", "v", "w", "k2", "k1", "thr_err", "noise_level", "level", "gate_id"):
        assert np.array_equal(np.ascontiguousarray(e[k]).view(np.uint32),
                              np.ascontiguousarray(orc.envs[k]).view(np.uint32)), k
    env.close()


def test_kernel_noisy_step_matches_reference():
    g, ge = NG.load()
    e, acts = NG.step_pre(ge)
    env = _env(len(e))
    cnt = int(g["G_cnt"][0])
    _load(env, e, cnt)
    obs, _, _, _, _ = env.step(torch.from_numpy(acts).to(DEV))
    got = _kernel_envs(env)
    pol = obs["policy"].cpu().numpy()
    assert NG.check_step(g, ge, got, pol) > 500
    assert np.array_equal(env._sets[env._cur]["dones"].cpu().numpy().astype(np.uint8), ge["s1_out_dones"])
    orc = oracle.from_env(env)
    orc.envs[:] = e
    orc.counter[0] = cnt
    orc.step(acts)
    assert np.array_equal(pol.view(np.uint32), orc.obs_policy.view(np.uint32))
    env.close()
