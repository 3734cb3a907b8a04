"""RSL-RL command-line arguments (same flags as the reference's standalone/rsl_rl/cli_args.py:10-33)."""
from __future__ import annotations

import argparse


def add_rsl_rl_args(parser: argparse.ArgumentParser):
    g = parser.add_argument_group("rsl_rl", description="Arguments for RSL-RL agent.")
    g.add_argument("--experiment_name", type=str, default=None, help="Name of the experiment folder for logs.")
    g.add_argument("--run_name", type=str, default=None, help="Run name suffix to the log directory.")
    g.add_argument("--resume", type=bool, default=None, help="Whether to resume from a checkpoint.")
    g.add_argument("--load_run", type=str, default=None, help="Name of the run folder to resume from.")
    g.add_argument("--checkpoint", type=str, default=None, help="Checkpoint file to resume from.")
    g.add_argument("--logger", type=str, default=None, choices={"wandb", "tensorboard", "neptune"},
                   help="Logger module to use (tensorboard if importable, else CSV scalars).")
    g.add_argument("--log_project_name", type=str, default=None, help="Logging project (wandb/neptune).")


def update_rsl_rl_cfg(agent_cfg, args_cli: argparse.Namespace):
    """Override runner cfg fields from the CLI (reference cli_args.py:54-80)."""
    if getattr(args_cli, "seed", None) is not None:
        agent_cfg.seed = args_cli.seed
    if args_cli.resume is not None:
        agent_cfg.resume = args_cli.resume
    if args_cli.load_run is not None:
        agent_cfg.load_run = args_cli.load_run
    if args_cli.checkpoint is not None:
        agent_cfg.load_checkpoint = args_cli.checkpoint
    if args_cli.run_name is not None:
        agent_cfg.run_name = args_cli.run_name
    if args_cli.logger is not None:
        agent_cfg.logger = args_cli.logger
    if args_cli.experiment_name is not None:
        agent_cfg.experiment_name = args_cli.experiment_name
    return agent_cfg
