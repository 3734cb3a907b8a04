"""Train the racing policy with the rsl_rl PPO stack on the HIP env (reference: standalone/rsl_rl/train.py).

Same command line as the reference (train.sh):

    python standalone/rsl_rl/train.py --task DiffLab-Quadcopter-CTBR-Racing-v0 --num_envs 1024 --headless

trains the reference recipe for that id (depth camera + VisionActorCritic + PPOL2C2); the state-only MLP
task of the BASELINE configs is DiffLab-Quadcopter-CTBR-Racing-State-v0.

Multi-GPU (one env shard per GPU, PPO gradients all-reduced over RCCL):

    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        standalone/rsl_rl/train.py --task DiffLab-Quadcopter-CTBR-Racing-State-v0 --num_envs 65536

There is no simulator app to launch: `--headless` and the other AppLauncher
flags are accepted and ignored; `--video` is rejected (no renderer).
"""
from __future__ import annotations

import argparse
import os
import re
import sys
from datetime import datetime

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import cli_args  # noqa: E402  isort: skip


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train an RL agent with RSL-RL.")
    p.add_argument("--video", action="store_true", default=False, help="(unsupported: no renderer)")
    p.add_argument("--video_length", type=int, default=200)
    p.add_argument("--video_interval", type=int, default=2000)
    p.add_argument("--num_envs", type=int, default=None, help="Number of environments per GPU.")
    p.add_argument("--task", type=str, default=None, help="Name of the task.")
    p.add_argument("--seed", type=int, default=42, help="Seed used for the environment")
    p.add_argument("--deterministic", action="store_true", default=False)
    p.add_argument("--max_iterations", type=int, default=None, help="RL Policy training iterations.")
    p.add_argument("--device", type=str, default=None, help="cuda:N (default: cuda:LOCAL_RANK)")
    p.add_argument("--log_root", type=str, default="logs", help="Root of logs/rsl_rl/<experiment>.")
    p.add_argument("--agent", type=str, default="rsl_rl_cfg_entry_point",
                   help="Registry key of the runner cfg (rsl_rl_l2c2_cfg_entry_point: PPOL2C2 recipe).")
    # AppLauncher flags the reference's train.sh passes; accepted for drop-in compatibility
    p.add_argument("--headless", action="store_true", default=False)
    p.add_argument("--enable_cameras", action="store_true", default=False)
    p.add_argument("--livestream", type=int, default=None)
    p.add_argument("--fused_rollout", action="store_true", default=False,
                   help="Rollout inference as one bf16 MFMA launch (algorithm.fused_rollout_inference).")
    p.add_argument("--fused_rollout_fp32", action="store_true", default=False,
                   help="The same launch with fp32 operands on fp32 MFMA, the reference's precision "
                        "(algorithm.fused_rollout_precision=fp32).")
    p.add_argument("--graph_update", action="store_true", default=False,
                   help="PPO mini-batch step replayed from hipGraphs (algorithm.graph_update; at world size > 1 two graphs "
                        "with the gradient all-reduce issued eagerly between them).")
    p.add_argument("--bf16_update", action="store_true", default=False,
                   help="PPO update forward/backward under bf16 autocast (algorithm.update_autocast_bf16).")
    p.add_argument("--bf16_storage", action="store_true", default=False,
                   help="bf16 observation buffers in the rollout storage (algorithm.storage_obs_dtype).")
    cli_args.add_rsl_rl_args(p)
    return p


def get_checkpoint_path(log_path: str, run_dir: str = ".*", checkpoint: str = ".*") -> str:
    """Latest run folder matching `run_dir`, latest checkpoint in it matching `checkpoint` (IL semantics)."""
    runs = sorted(e.name for e in os.scandir(log_path) if e.is_dir() and re.match(run_dir, e.name))
    if not runs:
        raise ValueError(f"no runs in {log_path!r} match {run_dir!r}")
    run = os.path.join(log_path, runs[-1])
    ckpts = [f for f in os.listdir(run) if re.match(checkpoint, f)]
    if not ckpts:
        raise ValueError(f"no checkpoints in {run!r} match {checkpoint!r}")
    ckpts.sort(key=lambda m: f"{m:0>15}")
    return os.path.join(run, ckpts[-1])


def main(argv=None):
    args, _unknown = build_parser().parse_known_args(argv)
    if args.video:
        raise SystemExit("--video is not supported: this build has no renderer")
    import torch
    import yaml

    import importlib

    registry = importlib.import_module("generalizableracing_amd.registry")
    from generalizableracing_amd.envs.racing_env import RslRlVecEnvWrapper
    from generalizableracing_amd.rsl_rl import OnPolicyRunner
    from generalizableracing_amd.rsl_rl import distributed as gdist

    task = args.task or "DiffLab-Quadcopter-CTBR-Racing-v0"
    rank, local_rank, world = gdist.init_from_env()
    env_cfg = registry.load_cfg_from_registry(task, "env_cfg_entry_point")
    agent_cfg = registry.load_cfg_from_registry(task, args.agent)
    agent_cfg = cli_args.update_rsl_rl_cfg(agent_cfg, args)
    if args.num_envs is not None:
        env_cfg.scene.num_envs = args.num_envs
    if args.max_iterations is not None:
        agent_cfg.max_iterations = args.max_iterations
    if args.fused_rollout or args.fused_rollout_fp32:
        agent_cfg.algorithm.fused_rollout_inference = True
    if args.fused_rollout_fp32:
        agent_cfg.algorithm.fused_rollout_precision = "fp32"
    if args.bf16_storage:
        agent_cfg.algorithm.storage_obs_dtype = "bfloat16"
    if args.graph_update:
        agent_cfg.algorithm.graph_update = True
    if args.bf16_update:
        agent_cfg.algorithm.update_autocast_bf16 = True
    device = args.device or (f"cuda:{local_rank}" if torch.cuda.is_available() else "cpu")
    agent_cfg.device = device
    env_cfg.sim.device = device
    # per-shard env ids (independent RNG streams) and per-shard randomized track layouts
    env_cfg.seed = agent_cfg.seed
    env_cfg.env_id_offset = rank * env_cfg.scene.num_envs
    env_cfg.track_seed_offset = rank

    log_root_path = os.path.abspath(os.path.join(args.log_root, "rsl_rl", agent_cfg.experiment_name))
    log_dir = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    if agent_cfg.run_name:
        log_dir += f"_{agent_cfg.run_name}"
    log_dir = os.path.join(log_root_path, log_dir)
    torch.manual_seed(args.seed + rank)
    if args.deterministic:
        torch.use_deterministic_algorithms(True)

    env = RslRlVecEnvWrapper(registry.make(task, cfg=env_cfg))
    runner = OnPolicyRunner(env, agent_cfg.to_dict(), log_dir=log_dir if rank == 0 else None, device=device)
    if agent_cfg.resume:
        resume_path = get_checkpoint_path(log_root_path, agent_cfg.load_run, agent_cfg.load_checkpoint)
        print(f"[INFO]: Loading model checkpoint from: {resume_path}")
        runner.load(resume_path)
    if rank == 0:
        os.makedirs(os.path.join(log_dir, "params"), exist_ok=True)
        from dataclasses import asdict

        with open(os.path.join(log_dir, "params", "env.yaml"), "w") as f:
            yaml.safe_dump(asdict(env_cfg), f)
        with open(os.path.join(log_dir, "params", "agent.yaml"), "w") as f:
            yaml.safe_dump(agent_cfg.to_dict(), f)
    runner.learn(num_learning_iterations=agent_cfg.max_iterations, init_at_random_ep_len=True)
    env.close()
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    return runner


if __name__ == "__main__":
    main()
