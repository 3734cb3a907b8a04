"""The vision racing task end to end on one MI355X: depth-camera env step + VisionActorCritic.

Measures, at --envs envs/GPU with the reference recipe (QuadcopterVisionPPORunnerCfg:
VisionActorCritic 72x96 stem, 128x128 heads, PPOL2C2):
  * env step alone (gr_step + gr_camera_render), env-steps/s;
  * rollout step (policy act + critic evaluate + env step) as the runner does it;
  * one full training iteration (24-step rollout + PPOL2C2 update, 5 epochs x 4 minibatches) with
    the runner's own timers -> the reference's Perf/total_fps definition.

  python scripts/bench_vision.py --envs 4096 --iters 2
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv, RslRlVecEnvWrapper  # noqa: E402
from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterVisionPPORunnerCfg  # noqa: E402


def timed(fn, steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--iters", type=int, default=2, help="training iterations (0: skip)")
    ap.add_argument("--storage-bf16", action="store_true", help="rollout storage observations in bf16")
    ap.add_argument("--no-fused-bn", action="store_true", help="the stem's BatchNorm + activation on torch's ops")
    ap.add_argument("--no-fused-conv2-forward", action="store_true",
                    help="conv2's forward as a GEMM (not inside the first block's apply pass)")
    ap.add_argument("--no-fused-conv2", action="store_true",
                    help="conv2's input gradient as a GEMM (not inside the first block's backward passes)")
    ap.add_argument("--no-share", action="store_true", help="PPOL2C2's mixed batch through two stem forwards")
    ap.add_argument("--no-rows", action="store_true", help="the graphed update gathers the mini-batch rows")
    ap.add_argument("--no-fused-conv3", action="store_true", help="block 2 materialised before conv3")
    ap.add_argument("--graph-update", action="store_true",
                    help="the update's mini-batch steps as hipGraph replays (ppo_l2c2._GraphedStepL2C2)")
    print(json.dumps(run(ap.parse_args(argv))))


def run(args):
    """-> the measurements above as a dict (args: envs, steps, iters, storage_bf16, no_fused_bn)."""
    n = args.envs
    dev = "cuda:0"
    torch.manual_seed(0)
    env = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=dev),
                                                    camera=CameraCfg())))
    cfg = QuadcopterVisionPPORunnerCfg(device=dev)
    d = cfg.to_dict()
    if args.storage_bf16:
        d["algorithm"]["storage_obs_dtype"] = torch.bfloat16
    runner = OnPolicyRunner(env, d, log_dir=None, device=dev)
    runner.alg.share_mix_features = not getattr(args, "no_share", False)
    runner.alg.graph_update = bool(getattr(args, "graph_update", False))
    runner.alg.rows_update = not getattr(args, "no_rows", False)
    pol = runner.alg.policy
    pol.fused_bn = not args.no_fused_bn
    pol.fused_conv2 = not getattr(args, "no_fused_conv2", False)
    pol.fused_conv2_forward = not getattr(args, "no_fused_conv2_forward", False)
    pol.fused_conv3 = not getattr(args, "no_fused_conv3", False)
    obs, extras = env.get_observations()
    crit = extras["observations"]["critic"]
    g = torch.Generator(device=dev).manual_seed(1)
    acts = [torch.randn(n, 4, device=dev, generator=g) for _ in range(4)]
    out = {"fused_bn": pol.fused_bn, "fused_conv2": pol.fused_conv2, "fused_conv2_forward": pol.fused_conv2_forward, "share_mix_features": runner.alg.share_mix_features, "graph_update": runner.alg.graph_update, "envs": n, "obs_dim": int(obs.shape[1]), "params": sum(p.numel() for p in pol.parameters())}

    for _ in range(4):
        env.step(acts[0])
    t_env = timed(lambda k: env.step(acts[k % 4]), args.steps)
    out["env_step_ms"] = t_env * 1e3
    out["env_steps_per_s"] = n / t_env

    with torch.inference_mode():
        def act_step(k):
            a = runner.alg.act(obs, crit)
            env.step(a)
            runner.alg.transition.clear()
        for _ in range(3):
            act_step(0)
        t_roll = timed(act_step, args.steps)
        t_act = timed(lambda k: (pol.act(obs), pol.evaluate(crit)), args.steps)
    out["rollout_step_ms"] = t_roll * 1e3
    out["policy_act_evaluate_ms"] = t_act * 1e3
    out["rollout_env_steps_per_s"] = n / t_roll

    if args.iters > 0:
        runner.learn(1)  # warm-up (kernels, allocator)
        t0 = time.perf_counter()
        runner.learn(args.iters)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        out["train_iters"] = args.iters
        out["train_iter_s"] = wall / args.iters
        out["train_total_fps"] = runner.cfg["num_steps_per_env"] * n * args.iters / wall
        out["last_log"] = {k: runner.last_log[k] for k in ("fps", "collection_time", "learn_time")
                           if k in runner.last_log}
        out["max_mem_GB"] = torch.cuda.max_memory_allocated() / 1e9
    env.close()
    return out


if __name__ == "__main__":
    main()
