"""MI355X-native drone-racing env step + rsl_rl PPO rollout.

Re-implements the hot path of yufengsjtu/GeneralizableRacing's
`DiffLab-Quadcopter-CTBR-Racing-v0`: the per-env step (CTBR controller,
rigid-body integration, gate progress, collision, reward, termination, reset,
observation) as hand-written HIP for gfx950 behind a C ABI (include/gr.h),
driven by a PyTorch-ROCm re-implementation of the rsl_rl runner / PPO /
rollout storage, sharded one env shard per GPU with RCCL gradient all-reduce.
"""
from .registry import make, register, registry  # noqa: F401

__version__ = "0.1.0"
