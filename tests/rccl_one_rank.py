"""Helper of tests/test_gpu_rccl_one_rank.py (run as its own process): the data-parallel PPO training path on a
process group of ONE rank, with the world-size > 1 code forced on (distributed.is_dist), so every exchange the N-GPU
run makes goes through the backend given: the rank-0 parameter broadcast, the global advantage statistics, the
segmented graph-captured update with the flat gradient + KL all-reduce issued eagerly between its two graphs, and the
env's episode-statistics reduction.  Prints one JSON line: the parameters' SHA-256 after the run, the exchanges of the
last update, the backend.

    python tests/rccl_one_rank.py nccl|gloo PORT
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(backend, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=0, world_size=1)
    from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg
    from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper
    from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg
    from generalizableracing_amd.rsl_rl import distributed as gdist

    gdist.is_dist = lambda: True  # the N-rank code paths on a world of one
    dev = "cuda:0"
    venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=4096), sim=SimCfg(device=dev))))
    cfg = QuadcopterPPORunnerCfg(device=dev)
    cfg.algorithm.fused_rollout_inference = True
    cfg.algorithm.fused_rollout_precision = "fp32"
    cfg.algorithm.graph_update = True
    torch.manual_seed(5)
    runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=dev)
    runner.learn(1, init_at_random_ep_len=True)  # (capture)
    gdist.FlatGrads.timings = []
    runner.learn(1)
    torch.cuda.synchronize()
    n_ex = len(gdist.FlatGrads.timings)
    gdist.FlatGrads.timings = None
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).cpu()
    out = {"backend": dist.get_backend(), "param_sha256": hashlib.sha256(flat.numpy().tobytes()).hexdigest(),
           "exchanges": n_ex, "segmented": bool(runner.alg._graphed.segmented) if runner.alg._graphed else None,
           "finite": bool(torch.isfinite(flat).all())}
    venv.close()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
