"""Shared parts of the noise-on reference pins (tests/golden/make_golden_noise.py -> golden_noise.npz): the configs,
the fixture's pre-states as oracle env records, and the comparisons.  Run against the oracle by
tests/test_oracle_noise_golden.py and against the HIP kernel by tests/test_gpu_noise_golden.py.

Tolerances: the reference applies each draw in fp32 torch ops in the world frame (positions = local + origin,
quaternion products and rotations in IL's formulas), the build in one scalar fp32 chain in the env-local frame, so
the floats agree to round-off: 1e-5 of max(1, |x|) (the north star's bar); the startup-DR values are one or two ops
(1e-6).  Levels and gate ids exactly."""
from __future__ import annotations

import os

import numpy as np

import oracle
from env_golden import close, envs_from_fixture

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    return np.load(os.path.join(GOLDEN, "golden_noise.npz")), np.load(os.path.join(GOLDEN, "golden_env.npz"))


def cfg(n):
    """Stage 1, gate-only tracks, every draw on (observation noise, gate noise, startup and reset DR)."""
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    c = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=1,
                     terrain=TerrainCfg(obstacles=False)).to_gr_config()
    assert c.obs_noise and c.add_gate_noise and c.dr_startup and c.random_drag
    return c


def startup_fields():
    return ("Kp", "Kd", "cT", "ctau", "m_plant", "J", "thr_err")


def check_startup(g, envs):
    for k in startup_fields():
        err = close(envs[k], g[f"S_{k}"], 1e-6)
        assert err <= 1e-6, ("startup", k, err)


def reset_pre(g):
    """(env records, previous critic rows, counter) the reset part starts from."""
    n = g["R_pre_p"].shape[0]
    e = np.zeros(n, dtype=oracle.ENV_DTYPE)
    for name in oracle.ENV_DTYPE.names:
        e[name] = g[f"R_pre_{name}"]
    return e, g["R_prev_critic"], int(g["R_cnt"][0])


def check_reset(g, envs, obs_policy, obs_critic):
    for k in ("p", "q", "v", "w", "k2", "k1", "thr_err", "noise_level"):
        err = close(envs[k], g[f"R_{k}"])
        assert err <= 1e-5, ("reset", k, err)
    assert np.array_equal(envs["level"], g["R_level"]), "curriculum level"
    assert np.array_equal(envs["gate_id"], g["R_gate_id"]), "start gate"
    assert (envs["acc"] == 0).all() and (envs["ep_len"] == 0).all()
    for name, got, ref in (("policy", obs_policy, g["R_obs_policy12"]), ("critic", obs_critic, g["R_obs_critic12"])):
        err = close(got[:, :12], ref)
        assert err <= 1e-5, ("reset obs", name, err)


def step_pre(ge):
    """The stage-1 golden_env pre-step state (epoch 3) and its actions."""
    return envs_from_fixture(ge, 1), ge["s1_in_a"].astype(np.float32)


def check_step(g, ge, envs, obs_policy):
    live = ge["s1_out_dones"] == 0
    assert np.array_equal(envs["gate_id"][live], g["G_gate_id_after"][live]), "gate ids"
    err = close(obs_policy[live], g["G_obs_policy"][live])
    assert err <= 1e-5, ("noisy policy row", err)
    # the noise is really on: the noisy rows differ from the noise-free reference rows of golden_env
    assert np.abs(obs_policy[live] - ge["s1_out_obs_policy"][live]).max() > 1e-3
    return int(live.sum())
