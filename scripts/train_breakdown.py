"""Perf/total_fps of one training configuration, split into collection and learning time, plus the top
device kernels of one iteration (torch.profiler).  N, FUSED (1 = bf16, fp32), BF16, GRAPH, SINK env vars select the options."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg  # noqa: E402

n = int(os.environ.get("N", "65536"))
dev = "cuda:0"
venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=dev))))
cfg = QuadcopterPPORunnerCfg(device=dev)
cfg.algorithm.fused_rollout_inference = os.environ.get("FUSED", "0") in ("1", "fp32")
cfg.algorithm.fused_rollout_precision = "fp32" if os.environ.get("FUSED") == "fp32" else "bf16"
cfg.algorithm.storage_obs_dtype = "bfloat16" if os.environ.get("BF16", "0") == "1" else "float32"
cfg.algorithm.graph_update = os.environ.get("GRAPH", "0") == "1"
cfg.algorithm.obs_sink = os.environ.get("SINK", "1") == "1"
runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=dev)
runner.learn(1, init_at_random_ep_len=True)
for _ in range(3):
    runner.learn(1)
    lg = runner.last_log
    print(f"fps {lg['fps']} collection {lg['collection_time']:.4f} s learn {lg['learn_time']:.4f} s", flush=True)
if os.environ.get("PROF", "1") == "1":
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        runner.learn(1)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25, max_name_column_width=70), flush=True)
