"""Task configuration for DiffLab-Quadcopter-CTBR-Racing-v0.

Mirrors the fields of `QuadcopterRacingCTBREnvCfg`
(extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/racing_ctbr_env.py:97-398)
that the env step consumes, including the TRAINING_STAGE switch read from the
environment (racing_ctbr_env.py:39) that selects rewards / terminations /
curricula.  `to_gr_config()` lowers it to the C struct of include/gr.h.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

from .. import _abi

STAGE_ENV = "TRAINING_STAGE"


def training_stage() -> int:
    return int(os.environ.get(STAGE_ENV, 1))  # 0: pre-training, 1: training, 2: testing


@dataclass
class SceneCfg:
    num_envs: int = 2048          # racing_ctbr_env.py:357
    env_spacing: float = 2.5


@dataclass
class TerrainCfg:
    """RacingComplexTerrainCfg essentials (quadcopter_diff/terrains/racing_terrains.py:137-210)."""

    seed: int = 42
    num_rows: int = 10            # levels
    num_cols: int = 20            # types
    num_gates: int = 8
    max_init_terrain_level: int = 5
    # walls / orbits / ground obstacles (add_obs / add_ground_obs of every sub-terrain cfg)
    obstacles: bool = True
    obstacle_cell: float = 2.0    # xy grid cell of the obstacle lists (m)
    # EventCfg.reset_terrain (racing_ctbr_env.py:221-225): regenerate the terrain every
    # 0.03 * 24 * 5000 s of simulated time (None: never)
    regen_interval_s: float | None = 0.03 * 24 * 5000


@dataclass
class SimCfg:
    dt: float = 0.01
    device: str = "cuda:0"


@dataclass
class CameraCfg:
    """`front_camera` RayCasterCameraCfg (racing_ctbr_env.py:77-95, update_period :390-391)
    and the `depth_image` observation term (mdp/observation.py:65-94)."""

    width: int = 96
    height: int = 72
    # from_intrinsic_matrix([fx, 0, cx, 0, fy, cy, 0, 0, 1]) of the reference (python doubles)
    intrinsic_matrix: tuple = (388.963 / (640 / 96), 0.0, 317.04 / (640 / 96),
                               0.0, 388.963 / (480 / 72), 241.99 / (480 / 72), 0.0, 0.0, 1.0)
    offset_pos: tuple = (0.01, 0.0, 0.0)
    offset_rot: tuple = (0.991, 0.0, -0.131, 0.0)  # w x y z, convention "world" (normalised)
    max_distance: float = 10.0
    update_period: float = 0.04
    noise_std: float = 0.02      # policy group add_noise=True
    add_noise: bool = True
    obs_scale: float = 10.0      # depth_image normalize: > 10 -> 10, / 10

    @property
    def num_pixels(self) -> int:
        return self.width * self.height

    def to_gr(self) -> _abi.GrCameraConfig:
        k = _abi.GrCameraConfig()
        k.width, k.height = int(self.width), int(self.height)
        m = self.intrinsic_matrix
        k.fx, k.cx, k.fy, k.cy = float(m[0]), float(m[2]), float(m[4]), float(m[5])
        for j in range(3):
            k.offset_pos[j] = float(self.offset_pos[j])
        for j in range(4):
            k.offset_rot[j] = float(self.offset_rot[j])
        k.max_distance = float(self.max_distance)
        k.update_period = float(self.update_period)
        k.noise_std = float(self.noise_std)
        k.add_noise = int(bool(self.add_noise))
        k.obs_scale = float(self.obs_scale)
        return k


@dataclass
class RacingEnvCfg:
    scene: SceneCfg = field(default_factory=SceneCfg)
    terrain: TerrainCfg = field(default_factory=TerrainCfg)
    sim: SimCfg = field(default_factory=SimCfg)
    decimation: int = 3
    episode_length_s: float | None = None   # 6.0 (8.0 in stage 2)
    seed: int | None = None
    stage: int | None = None                # None: read TRAINING_STAGE
    integrator: str = "dd_explicit"         # or "semi_implicit"
    mass: float = 0.6                       # ASSUMPTION: USD mass not in the reference
    is_finite_horizon: bool = False
    # front depth camera: None = the state-only task (obs 16); CameraCfg() = the reference's
    # vision task (obs 16 + 96*72, racing_ctbr_env.py:141-160)
    camera: CameraCfg | None = None
    # shard description for multi-GPU runs (env ids offset for the RNG, track seed offset)
    env_id_offset: int = 0
    track_seed_offset: int = 0
    # any gr_config field by name, applied last
    overrides: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.stage is None:
            self.stage = training_stage()
        if self.episode_length_s is None:
            self.episode_length_s = 8.0 if self.stage == 2 else 6.0

    @property
    def step_dt(self) -> float:
        return self.sim.dt * self.decimation

    @property
    def max_episode_length(self) -> int:
        return math.ceil(self.episode_length_s / self.step_dt)

    def to_gr_config(self) -> _abi.GrConfig:
        c = _abi.default_config()
        c.num_envs = int(self.scene.num_envs)
        c.env_id_offset = int(self.env_id_offset)
        seed = 42 if self.seed is None else int(self.seed)
        c.seed_lo = seed & 0xFFFFFFFF
        c.seed_hi = (seed >> 32) & 0xFFFFFFFF
        c.num_types = self.terrain.num_cols
        c.num_levels = self.terrain.num_rows
        c.max_gates = self.terrain.num_gates
        c.max_init_level = min(self.terrain.max_init_terrain_level, self.terrain.num_rows - 1)
        c.stage = int(self.stage)
        c.integrator = {"dd_explicit": _abi.GR_INTEGRATOR_DD_EXPLICIT,
                        "semi_implicit": _abi.GR_INTEGRATOR_SEMI_IMPLICIT}[self.integrator]
        c.decimation = int(self.decimation)
        c.sim_dt = float(self.sim.dt)
        c.step_dt = float(self.sim.dt * self.decimation)
        c.episode_length_s = float(self.episode_length_s)
        c.max_episode_length = self.max_episode_length
        c.mass = float(self.mass)
        s = self.stage
        # commands (racing_ctbr_env.py:98-121)
        half = 0.1 if s in (0, 1) else 0.5
        for k in range(3):
            c.gate_noise_pos[k] = half
        c.add_gate_noise = int(s != 0)
        # curriculum (racing_ctbr_env.py:263-278)
        c.noise_curriculum = int(s == 1)
        # terminations (racing_ctbr_env.py:248-260)
        c.term_contact = 1
        c.term_bad_pose = int(s != 0)
        # rewards (racing_ctbr_env.py:281-328)
        c.w_progress = 1.0
        c.w_body_rate = -0.02 if s == 0 else -0.1
        c.w_action_rate = -0.01 if s == 0 else -0.05
        c.w_collision = -50.0 if s == 0 else -100.0
        c.collision_count_threshold = 2 if s == 0 else 0
        c.w_perception = 0.1
        c.w_success = 10.0 if s == 0 else 20.0
        c.w_bad_pose = -30.0 if s == 1 else 0.0
        for k, v in self.overrides.items():
            if not hasattr(c, k):
                raise KeyError(f"unknown gr_config field {k!r}")
            cur = getattr(c, k)
            if hasattr(cur, "__len__"):
                for j, x in enumerate(v):
                    cur[j] = x
            else:
                setattr(c, k, v)
        return c

    # names of the reward / termination terms in declaration order (log keys)
    def reward_term_names(self) -> list[str]:
        names = ["progress_rewards", "command_bodyrate_penalty", "action_rate", "collision_penalty",
                 "perception_reward", "success_cross"]
        if self.stage == 1:
            names.append("bad_pose_penalty")
        return names

    def termination_term_names(self) -> list[str]:
        return ["time_out", "outofbound"] if self.stage == 0 else ["time_out", "base_contact", "bad_pose"]

    def curriculum_term_names(self) -> list[str]:
        return ["terrain_levels", "command_noise_level"] if self.stage == 1 else ["terrain_levels"]


QuadcopterRacingCTBREnvCfg = RacingEnvCfg


@dataclass
class RacingVisionEnvCfg(RacingEnvCfg):
    """The reference task as registered (policy/critic obs carry the depth image)."""

    camera: CameraCfg | None = field(default_factory=CameraCfg)
