"""The HIP step kernel (gr_step through the C ABI) against the REFERENCE's own manager code: the
fixture's pre-step state of 1024 eventful envs per training stage is written into the device state
planes (teacher forcing), one gr_step runs, and the outputs are held to the reference vectors with the
tolerances of tests/env_golden.py — and to the CPU oracle bit for bit."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

import oracle  # noqa: E402
from env_golden import STAGES, check_step, envs_from_fixture  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv  # noqa: E402

DEV = "cuda:0"


@pytest.mark.parametrize("stage", STAGES)
def test_kernel_step_matches_reference_managers(golden_env, stage):
    g = golden_env
    e = envs_from_fixture(g, stage)
    n = e.shape[0]
    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=stage,
                                 terrain=TerrainCfg(obstacles=False),
                                 overrides=dict(obs_noise=0, add_gate_noise=0)))
    assert np.array_equal(env.track_gates[:, :, 0:3].cpu().numpy().reshape(20, 10, 8, 3), g["gate_pos"])
    torch.cuda.synchronize()
    st, ist = oracle.envs_to_planes(e, env.state.shape[0])
    env.state.copy_(torch.from_numpy(st).to(DEV))
    env.istate.copy_(torch.from_numpy(ist).to(DEV))
    a = g[f"s{stage}_in_a"]
    orc = oracle.from_env(env)
    orc.envs[:] = e
    orc.step(a)
    obs, rew, term, tout, _ = env.step(torch.from_numpy(a).to(DEV))
    torch.cuda.synchronize()
    got = oracle.planes_to_envs(env.state.cpu().numpy(), env.istate.cpu().numpy())
    dones = env._sets[env._cur]["dones"].cpu().numpy()
    pol, cri = obs["policy"].cpu().numpy(), obs["critic"].cpu().numpy()
    aux = obs["auxiliary"].cpu().numpy()[:, 0]
    check_step(g, stage, got, rew.cpu().numpy(), term.cpu().numpy(), tout.cpu().numpy(), dones, pol, cri, aux,
               g["start_gate"])
    # and the kernel is the oracle, bit for bit
    assert np.array_equal(rew.cpu().numpy().view(np.uint32), orc.reward.view(np.uint32))
    assert np.array_equal(pol.view(np.uint32), orc.obs_policy.view(np.uint32))
    for k in ("p", "q", "v", "w", "gate_id", "level", "acc"):
        assert np.array_equal(np.ascontiguousarray(got[k]).view(np.uint32),
                              np.ascontiguousarray(orc.envs[k]).view(np.uint32)), k
    env.close()


@pytest.mark.parametrize("stage", STAGES)
def test_kernel_free_run_matches_reference(golden_freerun, stage):
    """20 consecutive gr_step launches from the free-run fixture's initial state (tests/golden/
    make_golden_freerun.py): each step held to the reference's own composition (tests/env_golden.py
    check_free_step) and to the CPU oracle bit for bit."""
    from env_golden import check_free_step, freerun_envs

    g = golden_freerun
    e = freerun_envs(g, stage)
    n = e.shape[0]
    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=DEV), stage=stage,
                                 terrain=TerrainCfg(obstacles=False),
                                 overrides=dict(obs_noise=0, add_gate_noise=0)))
    torch.cuda.synchronize()
    st, ist = oracle.envs_to_planes(e, env.state.shape[0])
    env.state.copy_(torch.from_numpy(st).to(DEV))
    env.istate.copy_(torch.from_numpy(ist).to(DEV))
    orc = oracle.from_env(env)
    orc.envs[:] = e
    acts = g[f"s{stage}_actions"]
    for k in range(acts.shape[0]):
        orc.step(acts[k])
        obs, rew, term, tout, _ = env.step(torch.from_numpy(acts[k]).to(DEV))
        torch.cuda.synchronize()
        got = oracle.planes_to_envs(env.state.cpu().numpy(), env.istate.cpu().numpy())
        dones = env._sets[env._cur]["dones"].cpu().numpy()
        pol, cri = obs["policy"].cpu().numpy(), obs["critic"].cpu().numpy()
        aux = obs["auxiliary"].cpu().numpy()[:, 0]
        check_free_step(g, stage, k, got, rew.cpu().numpy(), term.cpu().numpy(), tout.cpu().numpy(), dones, pol, cri,
                        aux, g["start_gate"])
        assert np.array_equal(rew.cpu().numpy().view(np.uint32), orc.reward.view(np.uint32)), k
        assert np.array_equal(pol.view(np.uint32), orc.obs_policy.view(np.uint32)), k
        for key in ("p", "q", "v", "w", "gate_id", "level", "acc", "ep_len"):
            assert np.array_equal(np.ascontiguousarray(got[key]).view(np.uint32),
                                  np.ascontiguousarray(orc.envs[key]).view(np.uint32)), (k, key)
    env.close()
