"""The CPU oracle over a 20-step FREE RUN of the reference's own step composition
(tests/golden/make_golden_freerun.py): from the fixture's initial state, each step's outputs feed the next, in the
order of ManagerBasedDiffRLEnv.step (extensions/diff.lab/diff/lab/envs/manager_based_diff_rl_env.py:160-267).
Masks exact, state / observations within 1e-5, rewards within 2e-5 of scale, on the envs the fixture compares
(first episode, away from the thresholds: make_golden_freerun.py)."""
import numpy as np
import pytest

import oracle
from env_golden import STAGES, cfg, check_free_step, freerun_envs
from generalizableracing_amd.envs.tracks import build_tracks


@pytest.mark.parametrize("stage", STAGES)
def test_oracle_free_run_matches_reference(golden_freerun, stage):
    g = golden_freerun
    gates, recs, _ = build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42, obstacles=False)
    assert np.array_equal(gates[:, :, 0:3].reshape(20, 10, 8, 3), g["gate_pos"])
    e = freerun_envs(g, stage)
    n = e.shape[0]
    orc = oracle.Oracle(cfg(stage, n), gates, recs)
    orc.envs[:] = e
    acts = g[f"s{stage}_actions"]
    compared = []
    for k in range(acts.shape[0]):
        orc.step(acts[k])
        compared.append(check_free_step(g, stage, k, orc.envs, orc.reward, orc.terminated, orc.time_out, orc.dones,
                                        orc.obs_policy, orc.obs_critic, orc.obs_aux, g["start_gate"]))
    assert compared[-1] > n // 2, compared
