"""Gym-free task registry.

Keeps the reference's task id resolving (extensions/diff.lab_tasks/.../quadcopter_diff/__init__.py:77-90):
`DiffLab-Quadcopter-CTBR-Racing-v0` -> (env class, env cfg, rsl_rl runner cfg).
The reference registers the vision PPO-L2C2 runner cfg for this id; the
state-only MLP runner cfg (QuadcopterPPORunnerCfg, rsl_rl_ppo_cfg.py:15-41,
hidden dims 256x256 per BASELINE.json) is what this build trains.
"""
from __future__ import annotations

_REGISTRY: dict = {}


def register(id: str, entry_point, env_cfg_entry_point, rsl_rl_cfg_entry_point, **extra_entry_points):
    _REGISTRY[id] = {
        "entry_point": entry_point,
        "env_cfg_entry_point": env_cfg_entry_point,
        "rsl_rl_cfg_entry_point": rsl_rl_cfg_entry_point,
        **extra_entry_points,
    }


def registry() -> dict:
    return dict(_REGISTRY)


def _resolve(x):
    if isinstance(x, str):
        mod, _, attr = x.partition(":")
        import importlib

        return getattr(importlib.import_module(mod), attr)
    return x


def load_cfg_from_registry(task: str, key: str):
    if task not in _REGISTRY:
        raise KeyError(f"unknown task {task!r}; registered: {sorted(_REGISTRY)}")
    return _resolve(_REGISTRY[task][key])()


def make(task: str, cfg=None, render_mode=None, **kwargs):
    spec = _REGISTRY[task]
    cls = _resolve(spec["entry_point"])
    if cfg is None:
        cfg = load_cfg_from_registry(task, "env_cfg_entry_point")
    return cls(cfg, render_mode=render_mode, **kwargs)


register(
    "DiffLab-Quadcopter-CTBR-Racing-v0",
    entry_point="generalizableracing_amd.envs.racing_env:RacingEnv",
    env_cfg_entry_point="generalizableracing_amd.envs.racing_cfg:RacingEnvCfg",
    rsl_rl_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterPPORunnerCfg",
    rsl_rl_l2c2_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterL2C2PPORunnerCfg",
    env_cfg_vision_entry_point="generalizableracing_amd.envs.racing_cfg:RacingVisionEnvCfg",
    rsl_rl_vision_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterVisionPPORunnerCfg",
)

# the reference's registration of the id above, with the front depth camera and the
# VisionActorCritic + PPOL2C2 recipe (quadcopter_diff/__init__.py:50-62)
register(
    "DiffLab-Quadcopter-CTBR-Racing-Vision-v0",
    entry_point="generalizableracing_amd.envs.racing_env:RacingEnv",
    env_cfg_entry_point="generalizableracing_amd.envs.racing_cfg:RacingVisionEnvCfg",
    rsl_rl_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterVisionPPORunnerCfg",
)
