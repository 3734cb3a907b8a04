"""Gym-free task registry.

Keeps the reference's task id resolving (extensions/diff.lab_tasks/.../quadcopter_diff/__init__.py:50-63) to
the same pairing: `DiffLab-Quadcopter-CTBR-Racing-v0` -> (env class, the camera env cfg, the vision PPO-L2C2 runner
cfg), so the reference's train.sh trains the reference's recipe.  The state-only MLP task of the BASELINE
configs is `DiffLab-Quadcopter-CTBR-Racing-State-v0`.
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


# the reference's registration (quadcopter_diff/__init__.py:50-63): the racing env WITH the front depth camera
# (QuadcopterRacingCTBREnvCfg, racing_ctbr_env.py:77-95) and QuadcopterVisionPPORunnerCfg, i.e. VisionActorCritic +
# PPOL2C2 (rsl_rl_ppo_cfg.py:87-101) -- what the reference's train.sh trains
_VISION = dict(
    entry_point="generalizableracing_amd.envs.racing_env:RacingEnv",
    env_cfg_entry_point="generalizableracing_amd.envs.racing_cfg:RacingVisionEnvCfg",
    rsl_rl_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterVisionPPORunnerCfg",
)
register("DiffLab-Quadcopter-CTBR-Racing-v0", **_VISION)
# (round-3/4 name of the same pairing, kept as an alias)
register("DiffLab-Quadcopter-CTBR-Racing-Vision-v0", **_VISION)

# the state-only task: the same env without the camera (16-dim policy / critic observations) and rsl_rl PPO over
# MLP(256, 256) (QuadcopterPPORunnerCfg, rsl_rl_ppo_cfg.py:15-41 with BASELINE.json's hidden sizes); the BASELINE
# configs C2-C5, bench.py and smoke() measure this one.  The L2C2 recipe over the same MLP is a second agent key.
register(
    "DiffLab-Quadcopter-CTBR-Racing-State-v0",
    entry_point="generalizableracing_amd.envs.racing_env:RacingEnv",
    env_cfg_entry_point="generalizableracing_amd.envs.racing_cfg:RacingEnvCfg",
    rsl_rl_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterPPORunnerCfg",
    rsl_rl_l2c2_cfg_entry_point="generalizableracing_amd.rsl_rl.config:QuadcopterL2C2PPORunnerCfg",
)
