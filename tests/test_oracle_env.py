"""Known-answer tests of the env logic on the CPU oracle (no GPU).

The manager-level semantics the reference delegates to Isaac Lab (command
update, terminations, reward manager, curriculum, reset) have no reference
test or fixture ("parity unpinned"); they are pinned here by hand-derived
answers at the thresholds the reference uses (gate radius 0.35 m,
|roll| > pi/2, episode length 200, curriculum thresholds 3/2 and 4/3).
"""
import math

import numpy as np
import pytest

import oracle
from generalizableracing_amd import _abi
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg
from generalizableracing_amd.envs.tracks import Track, pack_tracks

DT = 0.03
G0 = (3.0, 0.0, 0.5)  # gate 0 of line_track() in the env-local frame (gate point - env origin)
STILL = -20.0  # tanh(-20) == -1 in fp32: thrust command 0


def line_track(origin_z=1.0, start=0, g=8, spacing=3.0):
    """Gates every `spacing` m along +x at 1.5 m, frames facing +x (euler rxyz (90, 90, 0))."""
    pts = np.zeros((g, 3), np.float32)
    pts[:, 0] = spacing * np.arange(1, g + 1)
    pts[:, 2] = 1.5
    eul = np.tile(np.array([90.0, 90.0, 0.0], np.float32), (g, 1))
    w = np.full(g, 1.0, np.float32)
    return Track(pts, eul, w, w.copy(), np.full(g, 0.2, np.float32), np.full(g, 0.2, np.float32),
                 np.array([0.0, 0.0, origin_z]), start)


def make_oracle(n=1, types=1, levels=10, stage=1, **ov):
    ov.setdefault("obs_noise", 0)
    ov.setdefault("add_gate_noise", 0)
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=stage, overrides=ov)
    cfg.terrain.num_cols = types
    cfg.terrain.num_rows = levels
    c = cfg.to_gr_config()
    gates, recs = pack_tracks([[line_track() for _ in range(levels)] for _ in range(types)], 8, 0.1)
    o = oracle.Oracle(c, gates, recs)
    o.init()
    return o


def place(o, i=0, p=(0, 0, 1.0), q=(1, 0, 0, 0), gate=0, level=3, ep_len=10):
    e = o.envs[i]
    e["p"] = p
    e["q"] = q
    e["v"] = 0
    e["w"] = 0
    e["alpha"] = 0
    e["T"] = 0
    e["tau"] = 0
    e["k1"] = 0
    e["k2"] = 0
    e["gate_id"] = gate
    e["level"] = level
    e["ep_len"] = ep_len
    e["acc"] = 0
    e["azero"] = 1


def still(n=1):
    return np.full((n, 4), [STILL, 0, 0, 0], np.float32)


def test_hover_equilibrium_zero_acceleration():
    c = _abi.default_config()
    n = 1
    s = np.zeros((n, 13), np.float32)
    s[:, 2] = 1.0
    s[:, 3] = 1.0
    par = np.zeros((n, 16), np.float32)
    par[:, 7] = 0.6
    par[:, 12:15] = [0.0015, 0.002, 0.004]
    tt = np.array([[np.float32(0.6) * np.float32(9.81), 0, 0, 0]], np.float32)
    so, _, xo = oracle.test_dynamics(c, 1, s, np.zeros((n, 3)), tt, np.zeros((n, 4)), par, np.zeros((n, 6)))
    assert abs(xo[0, 2]) < 1e-6 and np.abs(so[0, :3] - [0, 0, 1.0]).max() < 1e-7


def test_drone_at_rest_stays_put_without_gravity():
    o = make_oracle(gravity=0.0)
    place(o, p=(0.0, 0.0, 1.0))
    before = o.envs[0]["p"].copy()
    o.step(still())
    assert np.array_equal(o.envs[0]["p"], before) and o.dones[0] == 0


@pytest.mark.parametrize("dist,passes", [(0.349, True), (0.351, False)])
def test_gate_pass_threshold(dist, passes):
    o = make_oracle(gravity=0.0)
    place(o, p=(G0[0] - dist, G0[1], G0[2]), gate=0)
    o.step(still())
    e = o.envs[0]
    assert (e["gate_id"] == 1) == passes and (e["acc"] == 1) == passes
    # success_cross: 20 * 1/(d^2+1) * dt when inside the radius (rewards.py:215-224)
    succ = 20.0 * (1.0 / (dist * dist + 1.0)) * DT if passes else 0.0
    assert o.obs_aux[0] == (1.0 if passes else 0.0)
    assert abs(e["ep_sum"][5] - succ) < 1e-6


@pytest.mark.parametrize("roll,bad", [(1.58, True), (1.56, False), (-1.58, True), (3.0, True)])
def test_bad_pose_termination(roll, bad):
    o = make_oracle(gravity=0.0)
    q = (math.cos(roll / 2), math.sin(roll / 2), 0.0, 0.0)
    place(o, p=(0.0, 0.0, 1.0), q=q)
    o.step(still())
    assert bool(o.terminated[0]) == bad and bool(o.dones[0]) == bad and o.time_out[0] == 0
    if bad:  # the env was reset in-lane
        assert o.envs[0]["ep_len"] == 0


def test_time_out_at_episode_length():
    o = make_oracle(gravity=0.0)
    place(o, p=(0.0, 0.0, 1.0), ep_len=198)
    o.step(still())
    assert o.time_out[0] == 0 and o.envs[0]["ep_len"] == 199
    o.step(still())
    assert o.time_out[0] == 1 and o.terminated[0] == 0 and o.dones[0] == 1
    assert o.envs[0]["ep_len"] == 0 and o.envs[0]["epoch"] >= 1


@pytest.mark.parametrize("acc,level,expect", [(3, 4, 5), (2, 4, 4), (1, 4, 3), (0, 0, 0), (5, 9, None)])
def test_curriculum_levels(acc, level, expect):
    """curriculums.py:25-38 + IL update_env_origins: +1 if gates>=3, -1 if <2, clip 0, >=max -> random."""
    o = make_oracle()
    place(o, level=level)
    o.envs[0]["acc"] = acc
    o.reset(np.ones(1, np.uint8))
    lv = o.envs[0]["level"]
    if expect is None:
        assert 0 <= lv < 10
    else:
        assert lv == expect


@pytest.mark.parametrize("acc,factor", [(4, 1.02), (3, 1.0), (2, 0.97)])
def test_noise_curriculum(acc, factor):
    """curriculums.py:40-54: x1.02 if gates>=4, x0.97 if <3 (stage 1)."""
    o = make_oracle()
    place(o)
    o.envs[0]["acc"] = acc
    o.envs[0]["noise_level"] = 1.0
    o.reset(np.ones(1, np.uint8))
    assert abs(o.envs[0]["noise_level"] - factor) < 1e-7


def test_collision_known_answers():
    o = make_oracle()
    track = 3  # type 0, level 3
    ident = np.array([1, 0, 0, 0], np.float32)
    # gate 0 at G0, 1.0 x 1.0 hole, 0.2 edge, 0.2 thick (the whole collider box fits the slab), hole spanning local y (width) and z (height)
    assert o.collision_count(track, [3.0, 0.0, 0.5], ident) == 0          # through the middle of the hole
    assert o.collision_count(track, [3.0, 0.6, 0.5], ident) == 17         # inside the side bar
    assert o.collision_count(track, [3.0, 0.0, 1.1], ident) == 17         # inside the top bar
    assert 0 < o.collision_count(track, [3.0, 0.45, 0.5], ident) < 17     # straddling the hole edge
    assert o.collision_count(track, [3.5, 0.6, 0.5], ident) == 0          # beside the bar, off the slab
    assert o.collision_count(track, [3.0, 0.9, 0.5], ident) == 0          # outside the outer frame
    # origin_z = 1: ground plane at z = -1 in the env-local frame; collider half-height 0.025
    assert o.collision_count(track, [0.0, 0.0, -0.97], ident) == 0
    assert o.collision_count(track, [0.0, 0.0, -0.999], ident) == 8      # lz = -1 and lz = -0.5 layers
    assert o.collision_count(track, [0.0, 0.0, -1.5], ident) == 17


def test_reset_distribution_faces_start_gate():
    n = 4096
    o = make_oracle(n=n, types=2)
    o.reset(None)
    e = o.envs
    assert np.all(np.abs(e["p"][:, :2]) <= 0.5) and np.all(np.abs(e["p"][:, 2] - 0.5) <= 0.5)
    assert np.all(np.abs(e["v"]) <= 0.1)
    assert np.all(e["ep_len"] == 0) and np.all(e["gate_id"] == 0) and np.all(e["azero"] == 1)
    # body x axis vs direction to the start gate G0: yaw offset U(+-0.7), roll/pitch U(+-0.2)
    q = e["q"].astype(np.float64)
    w, x, y, z = q.T
    fwd = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y + w * z)], 1)
    to_gate = np.stack([3.0 - e["p"][:, 0], -e["p"][:, 1]], 1)
    ang = np.arccos(np.clip((fwd * to_gate).sum(1) / np.linalg.norm(fwd, axis=1) / np.linalg.norm(to_gate, axis=1), -1, 1))
    assert ang.max() < 0.75 and ang.max() > 0.6
    assert np.all(np.abs(np.linalg.norm(q, axis=1) - 1) < 1e-6)
    # drag DR (droneDynamics.py:50-57): k2 = 0.01 m + U(0,0.005), z x U(4, 4.4)
    k2 = e["k2"]
    assert np.all((k2[:, 0] > 0.003) & (k2[:, 0] < 0.02)) and np.all(k2[:, 2] / k2[:, 0] > 2.0)
    thr = e["thr_err"]
    assert abs(thr.mean() - 1) < 1e-3 and 0.008 < thr.std() < 0.012


def test_critic_observation_layout():
    o = make_oracle(gravity=0.0)
    yaw = 0.3
    q = (math.cos(yaw / 2), 0.0, 0.0, math.sin(yaw / 2))
    place(o, p=(0.5, 0.2, 1.2), q=q)
    o.envs[0]["v"] = [1.0, 0.0, 0.0]
    o.observe()
    ob = o.obs_critic[0].astype(np.float64)
    R = np.array([[math.cos(yaw), -math.sin(yaw), 0], [math.sin(yaw), math.cos(yaw), 0], [0, 0, 1]])
    np.testing.assert_allclose(ob[0:3], R.T @ [1, 0, 0], atol=1e-6)                    # v_b
    np.testing.assert_allclose(ob[3:6], R[2], atol=1e-6)                               # R[2,:]
    np.testing.assert_allclose(ob[6:9], R.T @ (np.array(G0) - [0.5, 0.2, 1.2]), atol=1e-6)
    np.testing.assert_allclose(ob[9:12], R.T @ [3.0, 0, 0], atol=1e-6)                # gate -> next gate
    assert np.array_equal(ob[12:16], np.zeros(4))  # last action: zeroed by the action manager reset


def test_rotor_constant_dr():
    """Config C5's rotor-constant DR (not in the reference): the thrust map and kappa of each env are the
    config's x U(0.9, 1.1), drawn once at start-up (off: the config's exactly); with it the gross-thrust clamp
    of the CTBR controller follows the env's own map (controller_diff.py:96-99)."""
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg
    from generalizableracing_amd.envs.tracks import build_tracks

    n = 256
    gates, recs, _ = build_tracks(num_types=4, num_levels=10, num_gates=8, obstacles=False)
    nominal = None
    for on in (0, 1):
        c = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"),
                         terrain=TerrainCfg(num_cols=4, obstacles=False), overrides=dict(dr_rotor=on)).to_gr_config()
        orc = oracle.Oracle(c, gates, recs)
        orc.init()
        rot = orc.envs["rotor"].astype(np.float64)
        base = np.array([c.thrustmap[0], c.thrustmap[1], c.thrustmap[2], c.kappa], np.float32).astype(np.float64)
        if not on:
            assert np.array_equal(rot, np.tile(base, (n, 1)))
            nominal = orc
            continue
        ratio = rot / base
        assert (ratio >= 0.9 - 1e-6).all() and (ratio <= 1.1 + 1e-6).all()
        assert len(np.unique(ratio[:, 0])) > n // 2 and ratio.std(axis=0).min() > 0.05
        # full thrust command: each env clamps at 4 f(w_max) of its own map (thrust filter state T = its clamp)
        for o in (orc, nominal):
            o.reset(None)
            o.envs["T"] = 0.0
            o.envs["cT"] = 0.0  # no filter lag: T = clamp(cmd)
            o.envs["thr_err"] = 10.0
            o.envs["azero"] = 0
            o.envs["lag"] = 1.0
            o.step(np.full((n, 4), 5.0, np.float32))
        w1 = np.float64(c.motor_omega[1])
        want = (rot[:, 0] * w1 * w1 + rot[:, 1] * w1 + rot[:, 2]) * 4.0
        live = orc.dones == 0
        np.testing.assert_allclose(orc.envs["T"][live], want[live].astype(np.float32), rtol=1e-6)
        assert not np.allclose(orc.envs["T"][live], nominal.envs["T"][live])

