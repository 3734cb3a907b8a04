"""Golden vectors for a 20-step FREE RUN of the env step, produced by the REFERENCE's own mdp code.

Run in the development container (the reference is mounted read-only at /root/reference; it never
travels to the GPU box):

    python tests/golden/make_golden_freerun.py

Per training stage, 512 envs start from a seeded pre-step state (drones 1-4 m before a gate, near hover, some
near the end of their episode) and take 20 steps of recorded actions (hover throttle + noise).  Each step is the
teacher-forced composition of make_golden_env.reference_step (the order of ManagerBasedDiffRLEnv.step,
extensions/diff.lab/diff/lab/envs/manager_based_diff_rl_env.py:160-267, over the reference's DiffActions /
CTBRController / DroneDynamics, reward, termination, command, curriculum and observation terms) and the next step
starts from its outputs: the DroneDynamics pose and body rate, its body angular acceleration (the D-term input the
simulator reports), the controller's filter state, the lagged action, episode length, gate id and accumulated
gates.  So the run follows the reference's step ordering across steps, not just within one.

Comparison mask `valid[k]` (what the tests compare at step k): an env is compared from step 0 until, and
including, its first reset (after a reset its start state is random in both); an env whose discrete outcome at
some step sits within round-off of a threshold (gate radius, bad-pose / height bounds, the collision lattice:
make_golden_env.margins_ok) is dropped from that step on.  Observation and gate-pose noise are off (the build's
obs_noise / add_gate_noise switches), as in golden_env.npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import make_golden_env as mge  # noqa: E402

OUT = os.path.join(HERE, "golden_freerun.npz")
N = 512
STEPS = 20
HOVER_A0 = float(np.arctanh(-1.0 / 3.0))  # tanh(a0) * s + s = m g with s = 1.5 m g: the hover throttle


def sample_free_state(rng, st, gate_pose, origin_z, stage):
    """Pre-step state of all envs for a free run (in place)."""
    n = len(st["p"])
    t, lv = st["type"], rng.integers(0, mge.NL, n)
    st["level"][:] = lv
    gid = rng.integers(0, mge.G, n)
    st["gate_id"][:] = gid
    gpos = gate_pose[t, lv, gid, :3].astype(np.float64)
    prev = gate_pose[t, lv, (gid - 1) % mge.G, :3].astype(np.float64)
    back = prev - gpos
    back /= np.maximum(np.linalg.norm(back, axis=1, keepdims=True), 1e-6)
    p = gpos + back * rng.uniform(1.0, 4.0, (n, 1)) + rng.normal(0, 0.3, (n, 3))
    ground = -origin_z[t, lv]
    p[:, 2] = np.maximum(p[:, 2], ground + 0.3)
    roll, pitch = rng.uniform(-0.3, 0.3, n), rng.uniform(-0.3, 0.3, n)
    yaw = np.arctan2(-back[:, 1], -back[:, 0]) + rng.uniform(-0.5, 0.5, n)
    q = mge.il_shim.quat_from_euler_xyz(*(torch.tensor(x, dtype=torch.float32) for x in (roll, pitch, yaw))).numpy()
    st["p"][:] = p
    st["q"][:] = q
    st["v"][:] = -back * rng.uniform(0.0, 3.0, (n, 1)) + rng.normal(0, 0.3, (n, 3))
    st["w"][:] = rng.normal(0, 0.5, (n, 3))
    st["alpha"][:] = rng.normal(0, 2.0, (n, 3))
    st["T"][:] = mge.MASS0 * 9.81 * rng.uniform(0.8, 1.2, n)
    st["tau"][:] = rng.normal(0, 0.002, (n, 3))
    st["a_prev"][:] = np.concatenate([HOVER_A0 + rng.normal(0, 0.2, (n, 1)), rng.normal(0, 0.3, (n, 3))], 1)
    st["thr_err"][:] = 1.0 + rng.normal(0, 0.02, n)
    st["m_ctrl"][:] = mge.MASS0 + rng.uniform(-0.02, 0.02, n)
    st["m_plant"][:] = mge.MASS0 + rng.uniform(-0.02, 0.02, n)
    st["J"][:] = np.array(mge.J0) * rng.uniform(0.9, 1.1, (n, 3))
    z = 4.0 + rng.uniform(0, 0.4, n)
    k2 = 0.01 * st["m_ctrl"][:, None] + rng.uniform(0, 0.005, (n, 3))
    k1 = 0.18 * st["m_ctrl"][:, None] + rng.uniform(0, 0.1, (n, 3))
    k2[:, 2] *= z
    k1[:, 2] *= z
    st["k2"][:], st["k1"][:] = k2, k1
    st["Kp"][:] = 35.0 * rng.uniform(0.9, 1.1, (n, 3))
    st["Kd"][:] = np.array([5e-4, 5e-4, 3e-4]) * rng.uniform(0.9, 1.1, (n, 3))
    st["dT"][:] = 0.03 * rng.uniform(0.8, 1.3, n)
    st["dtau"][:] = 0.03 * rng.uniform(0.8, 1.3, (n, 3))
    max_len = 267 if stage == 2 else 200
    ep = rng.integers(0, max_len - 1, n)
    near_end = rng.random(n) < 0.1  # these time out inside the run
    ep[near_end] = max_len - 1 - rng.integers(0, STEPS, near_end.sum())
    st["ep_len"][:] = ep
    st["acc"][:] = rng.integers(0, 7, n)
    st["noise_level"][:] = rng.uniform(0.8, 1.25, n)


def actions(rng, n):
    a = np.concatenate([HOVER_A0 + rng.normal(0, 0.25, (STEPS, n, 1)), rng.normal(0, 0.4, (STEPS, n, 3))], 2)
    return a.astype(np.float32)


def main():
    import oracle
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    gates, recs, gate_pose, start, origin_z = mge.tables()
    out = {"gate_pos": gate_pose[..., :3], "start_gate": start.astype(np.int32), "origin_z": origin_z}
    for stage in (0, 1, 2):
        cfg = RacingEnvCfg(scene=SceneCfg(num_envs=N), sim=SimCfg(device="cpu"), stage=stage,
                           terrain=TerrainCfg(obstacles=False)).to_gr_config()
        collide = oracle.Oracle(cfg, gates, recs).collision_count
        rng = np.random.default_rng(300 + stage)
        st = {k: np.zeros((N,) + s, np.float64) for k, s in (
            ("p", (3,)), ("q", (4,)), ("v", (3,)), ("w", (3,)), ("alpha", (3,)), ("T", ()), ("tau", (3,)),
            ("a_prev", (4,)), ("a", (4,)), ("thr_err", ()), ("m_ctrl", ()), ("m_plant", ()), ("J", (3,)),
            ("k2", (3,)), ("k1", (3,)), ("Kp", (3,)), ("Kd", (3,)), ("dT", ()), ("dtau", (3,)),
            ("noise_level", ()))}
        for k in ("type", "level", "gate_id", "ep_len", "acc"):
            st[k] = np.zeros(N, np.int64)
        st["type"][:] = torch.div(torch.arange(N), N / mge.NT, rounding_mode="floor").long().numpy()
        sample_free_state(rng, st, gate_pose, origin_z, stage)
        for k in st:
            if st[k].dtype == np.float64:
                st[k] = st[k].astype(np.float32).astype(np.float64)
        acts = actions(rng, N)
        alive = np.ones(N, bool)  # not yet reset, never near a threshold
        recs_k = {}
        init = None
        for k in range(STEPS):
            st["a"] = acts[k].astype(np.float64)
            res, pre = mge.reference_step(st, stage, gate_pose, start, origin_z, collide, carry=True)
            if k == 0:  # the state the reference actually stepped from (local position, body rates, D-term input)
                for key in ("p", "w", "alpha"):
                    st[key] = pre[key]
                init = {key: v.copy() for key, v in st.items()}
                init["cT"] = torch.exp(-mge.DT / torch.tensor(st["dT"], dtype=torch.float32)).numpy()
                init["ctau"] = torch.exp(-mge.DT / torch.tensor(st["dtau"], dtype=torch.float32)).numpy()
            alive &= mge.margins_ok(st, res, gate_pose, origin_z, stage, collide)
            for key in ("reward", "terminated", "time_out", "dones", "post_p", "post_q", "post_v", "post_w",
                        "gate_id_after", "acc_after", "level_after", "noise_level_after", "obs_policy", "obs_critic",
                        "obs_aux"):
                recs_k.setdefault(key, []).append(res[key])
            recs_k.setdefault("valid", []).append(alive.copy())
            d = res["dones"].astype(bool)
            # the next step starts from this step's outputs (DroneDynamics, controller, lag, bookkeeping)
            st["p"], st["q"], st["v"], st["w"] = (res[x].astype(np.float64) for x in ("post_p", "post_q", "post_v",
                                                                                          "post_w"))
            st["alpha"] = res["alpha_b"].astype(np.float64)
            st["T"], st["tau"] = res["ctrl_T"].astype(np.float64), res["ctrl_tau"].astype(np.float64)
            st["a_prev"] = st["a"].copy()
            st["ep_len"] = st["ep_len"] + 1
            st["gate_id"] = res["gate_id_after"].astype(np.int64)
            st["acc"] = res["acc_after"].astype(np.int64)
            alive &= ~d  # compared at its reset step (curriculum, command reset), dropped after
        for key, v in init.items():
            out[f"s{stage}_in_{key}"] = v
        out[f"s{stage}_actions"] = acts
        for key, v in recs_k.items():
            out[f"s{stage}_out_{key}"] = np.stack(v)
        # observation noise is off in this run, so the policy rows equal the critic rows: stored once
        # (tests/env_golden.py reads obs_critic when obs_policy is absent)
        if np.array_equal(out[f"s{stage}_out_obs_policy"], out[f"s{stage}_out_obs_critic"]):
            del out[f"s{stage}_out_obs_policy"]
        val = np.stack(recs_k["valid"])
        dn = np.stack(recs_k["dones"]).astype(bool)
        print(f"stage {stage}: compared at the last step {val[-1].sum()}/{N}; resets inside the run "
              f"{(dn & val).sum()}; gate passes {int((np.diff(np.stack(recs_k['acc_after']), axis=0) > 0).sum())}")
    conv = {}
    for k, v in out.items():
        v = np.asarray(v)
        if v.dtype == np.float64:
            v = v.astype(np.float32)
        elif v.dtype == np.bool_:
            v = v.astype(np.uint8)
        elif v.dtype == np.int64:
            v = v.astype(np.int32)
        conv[k] = np.ascontiguousarray(v)
    np.savez_compressed(OUT, **conv)
    print(f"wrote {OUT}: {sum(v.nbytes for v in conv.values()) / 1e3:.1f} kB raw, {len(conv)} arrays")


if __name__ == "__main__":
    main()
