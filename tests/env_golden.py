"""Shared helpers of the reference-pinned step tests (tests/golden/make_golden_env.py fixtures):
the fixture's pre-step state as oracle env records, and the comparisons with their tolerances.

Tolerances.  The reference composes fp32 torch ops (bmm, vectorised reductions, world-frame positions =
local + origin) where the build runs one scalar fp32 chain without FMA in the env-local frame, so floats
agree to round-off: 1e-5 of max(1, |x|) for the state and observations (the north star's bar), 2e-5 of
the reward's scale.  Masks, gate ids, accumulated gates and curriculum levels are compared exactly."""
from __future__ import annotations

import numpy as np

import oracle

STAGES = (0, 1, 2)


def cfg(stage, n):
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    return RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=stage,
                        terrain=TerrainCfg(obstacles=False),
                        overrides=dict(obs_noise=0, add_gate_noise=0)).to_gr_config()


def envs_from_fixture(g, stage):
    """gro_env records of the fixture's pre-step state (the lag record holds tanh(a_prev): DESIGN §6)."""
    s = lambda k: g[f"s{stage}_in_{k}"]  # noqa: E731
    n = s("p").shape[0]
    e = np.zeros(n, dtype=oracle.ENV_DTYPE)
    for k in ("p", "q", "v", "w", "alpha", "T", "tau", "thr_err", "noise_level", "k2", "k1", "Kp", "cT", "Kd",
              "m_plant", "ctau", "m_ctrl", "J"):
        e[k] = s(k)
    e["lag"] = oracle.test_math(1, s("a_prev").reshape(-1)).reshape(n, 4)
    for k in ("ep_len", "acc", "gate_id", "level", "type"):
        e[k] = s(k)
    e["epoch"] = 3
    e["azero"] = 0
    return e


def close(got, want, rel=1e-5):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    err = np.abs(got - want) / np.maximum(1.0, np.abs(want))
    return float(err.max()) if err.size else 0.0


def check_step(g, stage, envs_after, reward, terminated, time_out, dones, obs_policy, obs_critic, obs_aux,
               start_gate):
    """Assert one step's outputs against the reference fixture of `stage`."""
    o = lambda k: g[f"s{stage}_out_{k}"]  # noqa: E731
    s = lambda k: g[f"s{stage}_in_{k}"]  # noqa: E731
    assert np.array_equal(terminated.astype(np.uint8), o("terminated")), "terminated"
    assert np.array_equal(time_out.astype(np.uint8), o("time_out")), "time_out"
    assert np.array_equal(np.asarray(dones).astype(np.uint8), o("dones")), "dones"
    rscale = max(1.0, float(np.abs(o("reward")).max()))
    assert np.abs(reward.astype(np.float64) - o("reward")).max() <= 2e-5 * rscale, \
        ("reward", np.abs(reward - o("reward")).max())
    assert np.array_equal(obs_aux.astype(np.float32), o("obs_aux")), "aux"
    live = o("dones") == 0
    e = envs_after
    for k, ref in (("p", "post_p"), ("q", "post_q"), ("v", "post_v"), ("w", "post_w")):
        err = close(e[k][live], o(ref)[live])
        assert err <= 1e-5, (k, err)
    assert np.array_equal(e["gate_id"][live], o("gate_id_after")[live]), "gate ids"
    assert np.array_equal(e["acc"][live], o("acc_after")[live].astype(np.int32)), "accumulated gates"
    for name, got, ref in (("policy", obs_policy, o("obs_policy")), ("critic", obs_critic, o("obs_critic"))):
        err = close(got[live], ref[live])
        assert err <= 1e-5, (name, err)
    # done envs: curriculum + command reset (their new random start state is not comparable)
    d = ~live
    lv_ref = o("level_after")[d]
    det = lv_ref >= 0  # the reference draws a random level above the top one
    assert np.array_equal(e["level"][d][det], lv_ref[det]), "curriculum levels"
    assert ((e["level"][d][~det] >= 0) & (e["level"][d][~det] < 10)).all()
    err = close(e["noise_level"][d], o("noise_level_after")[d], 1e-6)
    assert err <= 1e-6, ("noise level", err)
    want_start = start_gate[e["type"][d], e["level"][d]]
    assert np.array_equal(e["gate_id"][d], want_start), "start gate after reset"
    assert (e["acc"][d] == 0).all()
    assert (e["ep_len"][d] == 0).all()
    assert np.array_equal(e["ep_len"][live], s("ep_len")[live] + 1)


def freerun_envs(g, stage):
    """gro_env records of the free run's initial state (tests/golden/make_golden_freerun.py)."""
    return envs_from_fixture(g, stage)


def check_free_step(g, stage, k, envs_after, reward, terminated, time_out, dones, obs_policy, obs_critic, obs_aux,
                    start_gate):
    """Assert step k of the reference free run on the envs its `valid` mask compares (first episode, away from
    every threshold); returns the number of envs compared."""
    o = lambda key: g[f"s{stage}_out_{key}"][k]  # noqa: E731
    v = o("valid").astype(bool)
    where = f"stage {stage} step {k}"
    for name, got in (("terminated", terminated), ("time_out", time_out), ("dones", dones)):
        assert np.array_equal(np.asarray(got).astype(np.uint8)[v], o(name)[v]), (where, name)
    rscale = max(1.0, float(np.abs(o("reward")[v]).max()))
    assert np.abs(reward[v].astype(np.float64) - o("reward")[v]).max() <= 2e-5 * rscale, (where, "reward")
    assert np.array_equal(obs_aux.astype(np.float32)[v], o("obs_aux")[v]), (where, "aux")
    live = v & (o("dones") == 0)
    e = envs_after
    for key, ref in (("p", "post_p"), ("q", "post_q"), ("v", "post_v"), ("w", "post_w")):
        err = close(e[key][live], o(ref)[live])
        assert err <= 1e-5, (where, key, err)
    assert np.array_equal(e["gate_id"][live], o("gate_id_after")[live]), (where, "gate ids")
    assert np.array_equal(e["acc"][live], o("acc_after")[live].astype(np.int32)), (where, "accumulated gates")
    # noise off: the fixture stores the policy rows only when they differ from the critic rows
    ref_policy = o("obs_policy") if f"s{stage}_out_obs_policy" in g else o("obs_critic")
    for name, got, ref in (("policy", obs_policy, ref_policy), ("critic", obs_critic, o("obs_critic"))):
        err = close(got[live], ref[live])
        assert err <= 1e-5, (where, name, err)
    d = v & (o("dones") != 0)
    lv_ref = o("level_after")[d]
    det = lv_ref >= 0
    assert np.array_equal(e["level"][d][det], lv_ref[det]), (where, "curriculum levels")
    assert close(e["noise_level"][d], o("noise_level_after")[d], 1e-6) <= 1e-6, (where, "noise level")
    assert np.array_equal(e["gate_id"][d], start_gate[e["type"][d], e["level"][d]]), (where, "start gate")
    assert (e["acc"][d] == 0).all() and (e["ep_len"][d] == 0).all()
    return int(v.sum())
