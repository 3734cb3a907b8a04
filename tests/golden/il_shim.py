"""Stand-ins for the Isaac Lab modules the reference's pure-torch code imports — TEST INFRASTRUCTURE.

Isaac Lab (omni-isaac-lab >= 0.27.15, pyproject.toml:33 of the reference) is not installed and cannot be:
the fixture generators (make_golden.py, make_golden_env.py) load the reference's own files with these
modules registered in sys.modules instead.

* `omni.isaac.lab.utils.math`: the IL formulas the reference calls (quat_mul, quat_rotate(_inverse),
  quat_conjugate / quat_inv, quat_from_euler_xyz, matrix_from_quat, euler_xyz_from_quat, wrap_to_pi,
  quat_unique, compute_pose_error's position error), restated from the Isaac Lab 1.x source text.
  They are restatements: the fixtures pin the reference's composition of them, not IL itself
  ("parity unpinned" for IL).
* managers / assets / sensors / markers / terrains: empty base classes and plain config holders, so
  the reference's class and function definitions import; nothing of IL's behaviour is emulated here
  except what the fixture generators restate explicitly (and say so).
"""
from __future__ import annotations

import importlib.util
import math
import os
import sys
import types

import torch

REF = os.environ.get("GR_REFERENCE_ROOT", "/root/reference")


# ------------------------------------------------------------------ IL utils.math (restated)
def quat_mul(q1, q2):
    shape = q1.shape
    q1 = q1.reshape(-1, 4)
    q2 = q2.reshape(-1, 4)
    w1, x1, y1, z1 = q1[:, 0], q1[:, 1], q1[:, 2], q1[:, 3]
    w2, x2, y2, z2 = q2[:, 0], q2[:, 1], q2[:, 2], q2[:, 3]
    ww = (z1 + x1) * (x2 + y2)
    yy = (w1 - y1) * (w2 + z2)
    zz = (w1 + y1) * (w2 - z2)
    xx = ww + yy + zz
    qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
    w = qq - ww + (z1 - y1) * (y2 - z2)
    x = qq - xx + (x1 + w1) * (x2 + w2)
    y = qq - yy + (w1 - x1) * (y2 + z2)
    z = qq - zz + (z1 + y1) * (w2 - x2)
    return torch.stack([w, x, y, z], dim=-1).view(shape)


def quat_rotate(q, v):
    q_w = q[..., 0]
    q_vec = q[..., 1:]
    a = v * (2.0 * q_w**2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * (q_vec * v).sum(-1, keepdim=True) * 2.0
    return a + b + c


def quat_rotate_inverse(q, v):
    q_w = q[..., 0]
    q_vec = q[..., 1:]
    a = v * (2.0 * q_w**2 - 1.0).unsqueeze(-1)
    b = torch.cross(q_vec, v, dim=-1) * q_w.unsqueeze(-1) * 2.0
    c = q_vec * (q_vec * v).sum(-1, keepdim=True) * 2.0
    return a - b + c


def normalize(x, eps: float = 1e-9):
    return x / x.norm(p=2, dim=-1).clamp(min=eps).unsqueeze(-1)


def quat_conjugate(q):
    shape = q.shape
    q = q.reshape(-1, 4)
    return torch.cat((q[:, 0:1], -q[:, 1:]), dim=-1).view(shape)


def quat_inv(q):
    return normalize(quat_conjugate(q))


def quat_from_euler_xyz(roll, pitch, yaw):
    cy = torch.cos(yaw * 0.5)
    sy = torch.sin(yaw * 0.5)
    cr = torch.cos(roll * 0.5)
    sr = torch.sin(roll * 0.5)
    cp = torch.cos(pitch * 0.5)
    sp = torch.sin(pitch * 0.5)
    qw = cy * cr * cp + sy * sr * sp
    qx = cy * sr * cp - sy * cr * sp
    qy = cy * cr * sp + sy * sr * cp
    qz = sy * cr * cp - cy * sr * sp
    return torch.stack([qw, qx, qy, qz], dim=-1)


def quat_unique(q):
    return torch.where(q[..., 0:1] < 0, -q, q)


def matrix_from_quat(quaternions):
    r, i, j, k = torch.unbind(quaternions, -1)
    two_s = 2.0 / (quaternions * quaternions).sum(-1)
    o = torch.stack((
        1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j),
    ), -1)
    return o.reshape(quaternions.shape[:-1] + (3, 3))


def euler_xyz_from_quat(quat):
    q_w, q_x, q_y, q_z = quat[:, 0], quat[:, 1], quat[:, 2], quat[:, 3]
    sin_roll = 2.0 * (q_w * q_x + q_y * q_z)
    cos_roll = 1 - 2 * (q_x * q_x + q_y * q_y)
    roll = torch.atan2(sin_roll, cos_roll)
    sin_pitch = 2.0 * (q_w * q_y - q_z * q_x)
    pitch = torch.where(torch.abs(sin_pitch) >= 1, torch.copysign(torch.full_like(sin_pitch, math.pi / 2.0), sin_pitch),
                        torch.asin(sin_pitch))
    sin_yaw = 2.0 * (q_w * q_z + q_x * q_y)
    cos_yaw = 1 - 2 * (q_y * q_y + q_z * q_z)
    yaw = torch.atan2(sin_yaw, cos_yaw)
    return roll % (2 * torch.pi), pitch % (2 * torch.pi), yaw % (2 * torch.pi)


def wrap_to_pi(angles):
    wrapped = (angles + torch.pi) % (2 * torch.pi)
    return torch.where((wrapped == 0) & (angles > 0), torch.pi, wrapped - torch.pi)


def compute_pose_error(t01, q01, t02, q02, rot_error_type: str = "axis_angle"):
    """IL compute_pose_error: position error t02 - t01 (the reference only takes its norm); the rotation
    error (quaternion difference as axis-angle) is restated for completeness."""
    source_quat_inv = quat_inv(q01)
    quat_error = quat_mul(source_quat_inv, q02)
    pos_error = t02 - t01
    mag = 2.0 * torch.atan2(quat_error[..., 1:].norm(dim=-1), quat_error[..., 0])
    half = 0.5 * mag
    scale = torch.where(half.abs() > 1e-6, half / torch.sin(half).clamp(min=1e-12), 0.5 - half * half / 48)
    return pos_error, quat_error[..., 1:] / scale.unsqueeze(-1)


def yaw_quat(quat):
    qw, qz = quat[..., 0], quat[..., 3]
    yaw = torch.atan2(2 * (qw * qz + quat[..., 1] * quat[..., 2]), 1 - 2 * (quat[..., 2] ** 2 + qz ** 2))
    out = torch.zeros_like(quat)
    out[..., 0] = torch.cos(yaw / 2)
    out[..., 3] = torch.sin(yaw / 2)
    return normalize(out)


# IL sample_uniform: torch.rand(size) * (upper - lower) + lower.  SAMPLE_HOOK (a callable(size) -> tensor of U(0, 1), or
# None) lets a fixture generator feed the draws (make_golden_noise.py injects the build's Philox values).
SAMPLE_HOOK = None


def sample_uniform(lower, upper, size, device=None):
    if isinstance(size, int):
        size = (size,)
    u = SAMPLE_HOOK(tuple(size)) if SAMPLE_HOOK is not None else torch.rand(*size, device=device)
    return u * (upper - lower) + lower


def _randomize_prop_by_op(data, distribution_parameters, dim_0_ids, dim_1_ids, operation, distribution):
    """omni.isaac.lab.envs.mdp.events._randomize_prop_by_op (IL 1.x), restated for the uniform distribution."""
    if dim_0_ids is None:
        n_dim_0 = data.shape[0]
        dim_0_ids = slice(None)
    else:
        n_dim_0 = len(dim_0_ids)
        if not isinstance(dim_1_ids, slice):
            dim_0_ids = dim_0_ids[:, None]
    n_dim_1 = data.shape[1] if isinstance(dim_1_ids, slice) else len(dim_1_ids)
    if distribution != "uniform":
        raise NotImplementedError("not restated: not on the fixture path")
    v = sample_uniform(*distribution_parameters, (n_dim_0, n_dim_1), device=data.device)
    if operation == "add":
        data[dim_0_ids, dim_1_ids] += v
    elif operation == "scale":
        data[dim_0_ids, dim_1_ids] *= v
    elif operation == "abs":
        data[dim_0_ids, dim_1_ids] = v
    else:
        raise NotImplementedError(operation)
    return data


# ------------------------------------------------------------------ scripted draws (make_golden_noise.py)
class TorchProxy:
    """A reference module's `torch` with some call sites replaced (injected draws); everything else is torch."""

    def __init__(self, **over):
        self._over = over

    def __getattr__(self, k):
        return self._over[k] if k in self._over else getattr(torch, k)


class Queue:
    """Scripted draws: each call site takes the next tensor, which must have the requested shape."""

    def __init__(self, items=()):
        self.items = [torch.as_tensor(t, dtype=torch.float32) for t in items]

    def push(self, t):
        self.items.append(torch.as_tensor(t, dtype=torch.float32))

    def take(self, shape):
        t = self.items.pop(0)
        assert tuple(t.shape) == tuple(shape), (tuple(t.shape), tuple(shape))
        return t.clone()

    def done(self):
        assert not self.items, f"{len(self.items)} scripted draws unused"


class ScriptedUniform:
    """torch.empty(n) stand-in whose uniform_() yields the next scripted U(0, 1) tensor (commands.py's `r`)."""

    def __init__(self, q, n):
        self.q, self.n = q, n

    def uniform_(self):
        return self.q.take((self.n,))


def size_of(size):
    return tuple(size[0]) if len(size) == 1 and isinstance(size[0], (tuple, list)) else tuple(size)


def push_gate_noise(q, u):
    """The 12 uniform_ draws of one _resample_command / _update_command over envs with gate-noise draws u [m, 6] (gate
    x y z, next gate x y z): gate x y z roll pitch yaw, next gate x y z roll pitch yaw; the orientation draws are 0.5
    (zero angle: gate orientations are not observed)."""
    u = torch.as_tensor(u, dtype=torch.float32)
    half = torch.full((u.shape[0],), 0.5)
    for base in (0, 3):
        for k in range(3):
            q.push(u[:, base + k])
        for _ in range(3):
            q.push(half)


def _unsupported(*a, **k):
    raise NotImplementedError("not restated: not on the fixture path")


# ------------------------------------------------------------------ module tree
class _Base:
    """Empty base for IL classes the reference subclasses (ActionTerm, CommandTerm, ...)."""

    def __init__(self, *a, **k):
        pass


class SceneEntityCfg:
    def __init__(self, name="robot", body_names=None, **kw):
        self.name = name
        self.body_names = body_names
        self.body_ids = [0]


def install():
    mods = {}
    for n in ["omni", "omni.isaac", "omni.isaac.lab", "omni.isaac.lab.utils", "omni.isaac.lab.utils.math",
              "omni.isaac.lab.managers", "omni.isaac.lab.assets", "omni.isaac.lab.sensors", "omni.isaac.lab.markers",
              "omni.isaac.lab.terrains", "omni.isaac.lab.envs", "omni.isaac.lab.envs.mdp",
              "omni.isaac.lab.envs.mdp.events", "diff", "diff.lab", "diff.lab.utils", "diff.lab.controllers",
              "diff.lab.terrains"]:
        mods[n] = sys.modules.get(n) or types.ModuleType(n)
        sys.modules[n] = mods[n]
    m = mods["omni.isaac.lab.utils.math"]
    for f in (quat_mul, quat_rotate, quat_rotate_inverse, quat_conjugate, quat_inv, quat_from_euler_xyz, quat_unique,
              matrix_from_quat, euler_xyz_from_quat, wrap_to_pi, compute_pose_error, yaw_quat, normalize,
              sample_uniform):
        setattr(m, f.__name__, f)
    m.subtract_frame_transforms = _unsupported
    m.orthogonalize_perspective_depth = _unsupported
    mods["omni.isaac.lab.utils"].math = m
    mg = mods["omni.isaac.lab.managers"]
    mg.SceneEntityCfg = SceneEntityCfg
    for cname in ("ActionTerm", "CommandTerm", "ManagerTermBase"):
        setattr(mg, cname, type(cname, (_Base,), {}))
    for cname in ("Articulation", "RigidObject"):
        setattr(mods["omni.isaac.lab.assets"], cname, type(cname, (_Base,), {}))
    mods["omni.isaac.lab.envs.mdp.events"]._randomize_prop_by_op = _randomize_prop_by_op
    mods["diff.lab.terrains"].TerrainImporterCfg = type("TerrainImporterCfg", (_Base,), {})
    for cname in ("ContactSensor", "FrameTransformerData", "TiledCamera", "Camera", "RayCasterCamera",
                  "RayCasterCameraCfg"):
        setattr(mods["omni.isaac.lab.sensors"], cname, type(cname, (_Base,), {}))
    mods["omni.isaac.lab.markers"].VisualizationMarkers = type("VisualizationMarkers", (_Base,), {})
    mods["omni.isaac.lab.terrains"].TerrainImporter = type("TerrainImporter", (_Base,), {})
    # diff.lab.utils: the Warp ray test is not importable (stage 0's collision term is fed the build's count)
    mods["diff.lab.utils"].get_uav_collision_num_ray = _unsupported
    mods["diff.lab.utils"].LATTICE_TENSOR = None
    return mods


def load(name, path, package=None):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    if package:
        mod.__package__ = package
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def synthetic_package(name, path):
    """A package object whose submodules load from `path` without running its __init__.py."""
    pkg = types.ModuleType(name)
    pkg.__path__ = [path]
    sys.modules[name] = pkg
    return pkg


CTRL_DIR = os.path.join(REF, "extensions/diff.lab/diff/lab/controllers")
MDP_DIR = os.path.join(REF, "extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/mdp")


def load_controllers():
    install()
    synthetic_package("grref_ctrl", CTRL_DIR)
    thr = load("grref_ctrl.thrust_controller_diff", os.path.join(CTRL_DIR, "thrust_controller_diff.py"), "grref_ctrl")
    ctl = load("grref_ctrl.controller_diff", os.path.join(CTRL_DIR, "controller_diff.py"), "grref_ctrl")
    c = sys.modules["diff.lab.controllers"]
    c.ThrustController, c.CTBRController = thr.ThrustController, ctl.CTBRController
    c.PSController, c.LVController = ctl.PSController, ctl.LVController
    return thr, ctl


def load_mdp():
    """The reference's mdp modules of the racing task (rewards, observation, termination, curriculums,
    commands, diff_action, dynamics) as `grref_mdp.*`."""
    load_controllers()
    synthetic_package("grref_mdp", MDP_DIR)
    synthetic_package("grref_mdp.dynamics", os.path.join(MDP_DIR, "dynamics"))
    out = {"droneDynamics": load("grref_mdp.dynamics.droneDynamics", os.path.join(MDP_DIR, "dynamics/droneDynamics.py"),
                                 "grref_mdp.dynamics")}
    for name in ("diff_action", "rewards", "observation", "termination", "curriculums", "commands", "events"):
        out[name] = load(f"grref_mdp.{name}", os.path.join(MDP_DIR, f"{name}.py"), "grref_mdp")
    return out
