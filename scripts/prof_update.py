"""One PPO iteration at 65 536 envs (rollout + update) for a rocprofv3 kernel trace: where the update's time goes.

    rocprofv3 --kernel-trace --stats -d <dir> -- python3 scripts/prof_update.py [--fused] [--autocast]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--fused", action="store_true")
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--graph", action="store_true", help="graph-captured update (algorithm.graph_update)")
    ap.add_argument("--split", type=int, default=0, help="override rsl_rl/linear.py SPLIT (rows per chunk)")
    a = ap.parse_args()
    if a.split:
        from generalizableracing_amd.rsl_rl import linear

        linear.SPLIT = a.split
    dev = "cuda:0"
    venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=a.envs), sim=SimCfg(device=dev))))
    cfg = QuadcopterPPORunnerCfg(device=dev)
    cfg.algorithm.fused_rollout_inference = a.fused
    cfg.algorithm.fused_rollout_precision = "fp32"
    cfg.algorithm.graph_update = a.graph
    runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=dev)
    runner.learn(1, init_at_random_ep_len=True)
    torch.cuda.synchronize()
    for _ in range(a.iters):
        t0 = time.perf_counter()
        runner.learn(1)
        torch.cuda.synchronize()
        print(f"iteration {time.perf_counter() - t0:.4f} s  fps {runner.last_log['fps']:.0f}", flush=True)
