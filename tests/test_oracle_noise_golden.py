"""The oracle with every random draw on, against the reference's own startup-DR, reset, command and observation code
fed the same draws (tests/golden/make_golden_noise.py; comparisons in tests/noise_golden.py)."""
import numpy as np

import noise_golden as NG
import oracle
from generalizableracing_amd.envs.tracks import build_tracks


def _oracle(n):
    gates, recs, _ = build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42, obstacles=False)
    return oracle.Oracle(NG.cfg(n), gates, recs)


def test_startup_dr_matches_reference():
    g, _ = NG.load()
    n = g["S_Kp"].shape[0]
    orc = _oracle(n)
    orc.init()
    NG.check_startup(g, orc.envs)


def test_reset_draws_match_reference():
    g, _ = NG.load()
    pre, prev_crit, cnt = NG.reset_pre(g)
    orc = _oracle(len(pre))
    orc.envs[:] = pre
    orc.obs_critic[:] = prev_crit
    orc.counter[0] = cnt
    orc.reset(None)
    NG.check_reset(g, orc.envs, orc.obs_policy, orc.obs_critic)


def test_noisy_step_matches_reference():
    g, ge = NG.load()
    envs, acts = NG.step_pre(ge)
    orc = _oracle(len(envs))
    orc.envs[:] = envs
    orc.counter[0] = int(g["G_cnt"][0])
    orc.step(acts)
    assert NG.check_step(g, ge, orc.envs, orc.obs_policy) > 500
    assert np.array_equal(orc.dones.astype(np.uint8), ge["s1_out_dones"])
