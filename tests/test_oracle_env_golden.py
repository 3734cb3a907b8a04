"""The CPU oracle's env step against the REFERENCE's own manager code (tests/golden/make_golden_env.py):
one teacher-forced step per training stage of 1024 eventful envs, checked for termination / time-out /
done masks, rewards, the post-step state, gate progress, accumulated gates, observations and, for the
envs that reset, the terrain-level and noise-level curriculum and the command reset.

What this pins: the reference's reward terms and weights (mdp/rewards.py:154-253), terminations
(mdp/termination.py), command update / resample (mdp/commands.py:247-350), curricula
(mdp/curriculums.py, commands.py:385-402) and observation terms (mdp/observation.py) as composed by
ManagerBasedDiffRLEnv.step, over the reference's own DiffActions / CTBRController / DroneDynamics.
What it does not: Isaac Lab's manager plumbing and math helpers are restated stand-ins
(tests/golden/il_shim.py), and the contact term is fed the build's own collision count (PhysX / Warp
are absent: "parity unpinned")."""
import numpy as np
import pytest

import oracle
from env_golden import STAGES, cfg, check_step, envs_from_fixture
from generalizableracing_amd.envs.tracks import build_tracks


@pytest.fixture(scope="module")
def tables(golden_env):
    gates, recs, _ = build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42, obstacles=False)
    # the build's gate table is the one the fixture was generated over
    assert np.array_equal(gates[:, :, 0:3].reshape(20, 10, 8, 3), golden_env["gate_pos"])
    assert np.array_equal(recs[:, 2].reshape(20, 10).astype(np.int32), golden_env["start_gate"])
    return gates, recs


@pytest.mark.parametrize("stage", STAGES)
def test_step_matches_reference_managers(golden_env, tables, stage):
    g = golden_env
    e = envs_from_fixture(g, stage)
    n = e.shape[0]
    c = cfg(stage, n)
    assert np.array_equal(oracle.type_starts(c)[:-1], np.searchsorted(e["type"], np.arange(20)))
    orc = oracle.Oracle(c, *tables)
    orc.envs[:] = e
    orc.step(g[f"s{stage}_in_a"])
    check_step(g, stage, orc.envs, orc.reward, orc.terminated, orc.time_out, orc.dones, orc.obs_policy,
               orc.obs_critic, orc.obs_aux, g["start_gate"])
