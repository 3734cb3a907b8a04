"""Where the vision recipe's training iteration goes (QuadcopterVisionPPORunnerCfg at 4 096 envs): the runner's
collection / learn split, and a host profile (cProfile) of one PPOL2C2.update — host-bound or GPU-bound.

    python scripts/prof_vision_update.py [--envs 4096] [--out gpurun_out/vis_update.json]
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

from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterVisionPPORunnerCfg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=a.envs), sim=SimCfg(device=dev),
                                                    camera=CameraCfg())))
    runner = OnPolicyRunner(env, QuadcopterVisionPPORunnerCfg(device=dev).to_dict(), log_dir=None, device=dev)
    runner.learn(1)  # warm-up
    runner.learn(1)
    res = {"envs": a.envs, "last_log": {k: runner.last_log[k] for k in ("fps", "collection_time", "learn_time")}}
    alg = runner.alg
    upd = alg.update
    prof = {}

    def profiled_update():
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        out = upd()
        pr.disable()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        prof["host_s"] = t1 - t0
        prof["wall_s"] = time.perf_counter() - t0
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(45)
        prof["text"] = s.getvalue()
        return out

    alg.update = profiled_update
    runner.learn(1)
    res["update_host_s"], res["update_wall_s"] = prof["host_s"], prof["wall_s"]
    res["iteration"] = {k: runner.last_log[k] for k in ("fps", "collection_time", "learn_time")}
    print(json.dumps(res, indent=1))
    print(prof["text"])
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
            f.write("\n")
        with open(a.out.replace(".json", "_cprofile.txt"), "w") as f:
            f.write(prof["text"])
    env.close()


if __name__ == "__main__":
    main()
