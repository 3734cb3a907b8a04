"""Where a training iteration's rollout goes at small env counts (config C2: 4 096 envs): wall time of the
rollout loop's pieces (policy act, env.step, process_env_step, episode stats), each timed with a device
synchronisation around it, and the loop's host profile (cProfile, no synchronisation) — launch- / host-bound or
GPU-bound.

    python scripts/prof_rollout.py [--envs 4096] [--fused] [--out gpurun_out/rollout.json]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg  # noqa: E402
from generalizableracing_amd.rsl_rl.on_policy_runner import _EpisodeStats  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = "cuda:0"
    venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=a.envs), sim=SimCfg(device=dev))))
    cfg = QuadcopterPPORunnerCfg(device=dev)
    cfg.algorithm.fused_rollout_inference = a.fused
    cfg.algorithm.fused_rollout_precision = "fp32"
    cfg.algorithm.graph_update = True
    runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=dev)
    runner.learn(1, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    alg, env, storage = runner.alg, runner.env, runner.alg.storage
    obs, extras = env.get_observations()
    priv = extras["observations"].get(runner.privileged_obs_type, obs)
    stats = _EpisodeStats(env.num_envs, dev)
    T = runner.num_steps_per_env

    def one_step(obs, priv, timed=None):
        def mark(k, t0):
            if timed is not None:
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                timed[k] = timed.get(k, 0.0) + (t1 - t0)
                return t1
            return t0

        t = time.perf_counter()
        if storage.step >= T:
            storage.clear()
        act = alg.act(obs, priv)
        t = mark("act", t)
        if runner.obs_sink:
            env.set_obs_sink(*storage.sink_slot(storage.step + 1))
        obs, rew, dones, infos = env.step(act)
        t = mark("env_step", t)
        priv = infos["observations"].get(runner.privileged_obs_type, obs) \
            if runner.privileged_obs_type is not None else obs
        alg.process_env_step(rew, dones, infos)
        t = mark("process_env_step", t)
        stats.update(rew, dones)
        mark("stats", t)
        return obs, priv

    res = {"envs": a.envs, "fused_rollout": a.fused}
    with torch.inference_mode():
        storage.clear()
        for _ in range(8):
            obs, priv = one_step(obs, priv)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            obs, priv = one_step(obs, priv)
        torch.cuda.synchronize()
        res["step_us_async"] = (time.perf_counter() - t0) / a.steps * 1e6
        timed = {}
        for _ in range(a.steps):
            obs, priv = one_step(obs, priv, timed)
        res["step_us_synced_parts"] = {k: v / a.steps * 1e6 for k, v in timed.items()}
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.steps):
            obs, priv = one_step(obs, priv)
        pr.disable()
        torch.cuda.synchronize()
    if runner.obs_sink:
        env.set_obs_sink(None)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    print(json.dumps(res, indent=1))
    print(s.getvalue())
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")
        with open(a.out.replace(".json", "_cprofile.txt"), "w") as f:
            f.write(s.getvalue())


if __name__ == "__main__":
    main()
