"""The reference's own step composition timed on this container's CPU cores — a second stated CPU baseline beside
the C-oracle port (SURVEY §8d "CPU baseline").

The step is tests/golden/make_golden_env.reference_step: the reference's mdp code (DiffActions.process_actions with
CTBRController.compute and DroneDynamics.step standing in for PhysX, RacingCommand, the reward / termination /
observation / curriculum terms) composed in ManagerBasedDiffRLEnv.step's order over Isaac Lab stand-ins
(tests/golden/il_shim.py), free-running as make_golden_freerun.py does (each step starts from the last one's
outputs), stage 1, 8-gate tracks without obstacles.  The contact term needs a collision count the reference gets
from PhysX: here the build's C oracle is called per env from Python (its time is reported apart).  Isaac Lab's own
manager overhead and PhysX are not in this figure, so it flatters the reference.

Runs here only (it imports the reference from /root/reference, which never travels to the GPU box):

    python scripts/time_reference_cpu_step.py [--envs 4096] [--steps 200] [--out profiles/round05_reference_cpu_step.json]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import il_shim  # noqa: E402
import make_golden_env as mge  # noqa: E402
import make_golden_freerun as mgf  # noqa: E402


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "round05_reference_cpu_step.json"))
    a = ap.parse_args()
    import oracle
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg

    threads = os.cpu_count()
    torch.set_num_threads(threads)
    mdp = il_shim.load_mdp()  # the reference's modules, loaded once (reference_step would re-execute them per call)
    il_shim.load_mdp = lambda: mdp
    n, stage = a.envs, 1
    gates, recs, gate_pose, start, origin_z = mge.tables()
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=stage,
                       terrain=TerrainCfg(obstacles=False)).to_gr_config()
    orc_collide = oracle.Oracle(cfg, gates, recs).collision_count
    t_coll = [0.0]

    def collide(k, p, q):
        t0 = time.perf_counter()
        c = orc_collide(k, p, q)
        t_coll[0] += time.perf_counter() - t0
        return c

    rng = np.random.default_rng(7)
    st = {k: np.zeros((n,) + s, np.float64) for k, s in (
        ("p", (3,)), ("q", (4,)), ("v", (3,)), ("w", (3,)), ("alpha", (3,)), ("T", ()), ("tau", (3,)),
        ("a_prev", (4,)), ("a", (4,)), ("thr_err", ()), ("m_ctrl", ()), ("m_plant", ()), ("J", (3,)),
        ("k2", (3,)), ("k1", (3,)), ("Kp", (3,)), ("Kd", (3,)), ("dT", ()), ("dtau", (3,)), ("noise_level", ()))}
    for k in ("type", "level", "gate_id", "ep_len", "acc"):
        st[k] = np.zeros(n, np.int64)
    st["type"][:] = torch.div(torch.arange(n), n / mge.NT, rounding_mode="floor").long().numpy()
    mgf.sample_free_state(rng, st, gate_pose, origin_z, stage)
    acts = rng.standard_normal((a.warmup + a.steps, n, 4))
    t_all = 0.0
    for k in range(a.warmup + a.steps):
        if k == a.warmup:
            t_coll[0] = 0.0
        st["a"] = acts[k]
        t0 = time.perf_counter()
        res, _ = mge.reference_step(st, stage, gate_pose, start, origin_z, collide, carry=True)
        dt = time.perf_counter() - t0
        if k >= a.warmup:
            t_all += dt
        # the next step starts from this step's outputs (as make_golden_freerun.py)
        st["p"], st["q"], st["v"], st["w"] = (res[x].astype(np.float64) for x in ("post_p", "post_q", "post_v", "post_w"))
        st["alpha"] = res["alpha_b"].astype(np.float64)
        st["T"], st["tau"] = res["ctrl_T"].astype(np.float64), res["ctrl_tau"].astype(np.float64)
        st["a_prev"] = st["a"].copy()
        st["ep_len"] = np.where(res["dones"].astype(bool), 0, st["ep_len"] + 1)
        st["gate_id"] = res["gate_id_after"].astype(np.int64)
        st["acc"] = res["acc_after"].astype(np.int64)
        lv = res["level_after"].astype(np.int64)
        st["level"] = np.where(lv < 0, 0, lv)
    out = {
        "what": "the reference's step composition (tests/golden/make_golden_env.reference_step: its mdp code over "
                "Isaac Lab stand-ins, DroneDynamics for PhysX), free run, stage 1, 8-gate tracks",
        "num_envs": n, "steps": a.steps, "seconds": t_all,
        "env_steps_per_s": n * a.steps / t_all,
        "collision_seconds": t_coll[0],
        "env_steps_per_s_without_collision": n * a.steps / (t_all - t_coll[0]),
        "collision_note": "per-env Python calls of the build's C oracle (the reference's contact is PhysX)",
        "torch_threads": torch.get_num_threads(), "cores": threads, "cpu_model": cpu_model(),
        "torch": torch.__version__, "host": "development container (the reference cannot travel to the GPU box)",
        "script": "scripts/time_reference_cpu_step.py",
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
