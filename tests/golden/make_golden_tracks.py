"""Golden vectors for the gate layouts and obstacles, produced by the REFERENCE's own track generators.

Run in the development container (the reference is mounted read-only at /root/reference; it never
travels to the GPU box):

    python tests/golden/make_golden_tracks.py

Calls ZigzagRacingTerrain / SquareRacingTrackTerrain ("circular") / EllipseRacingTerrain
(extensions/diff.lab/diff/lab/terrains/trimesh/racing_terrains.py:167-336,423-832) with the sub-terrain
configs of the task's RacingComplexTerrainCfg (quadcopter_diff/terrains/racing_terrains.py:137-210, over
the class defaults of trimesh/racing_terrains_cfg.py), imported from their source files with stand-ins for
Isaac Lab's `configclass` / `SubTerrainBaseCfg` / `TerrainGeneratorCfg` / `make_border` and for trimesh:
trimesh is not installed, so `trimesh.creation.*` return records of their arguments and the meshes record
the transforms applied to them (make_gate / make_wall / make_orbit / make_ground_* of trimesh/utils.py run
unchanged, drawing their own random numbers).  Each case seeds NumPy's and Python's global generators, as
Isaac Lab's generator leaves them, and records the gate poses (position, Euler angles), the start gate, the
origin, every gate's outer / inner box extents and every obstacle primitive (kind, size, Euler angles,
position), plus the gate quaternion the reference stores (terrain_generator.py:64-73, scipy).
"""
from __future__ import annotations

import os
import random
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)

import il_shim  # noqa: E402

OUT = os.path.join(HERE, "golden_tracks.npz")
TRIMESH_DIR = os.path.join(il_shim.REF, "extensions/diff.lab/diff/lab/terrains/trimesh")
TASK_TERRAINS = os.path.join(il_shim.REF, "extensions/diff.lab_tasks/diff/lab_tasks/tasks/quadcopter_diff/terrains/"
                                          "racing_terrains.py")
KINDS = {"box": 0, "cylinder": 1, "icosphere": 2, "capsule": 3, "cone": 4}


class FakeMesh:
    """What trimesh.creation returns here: the primitive's arguments, then the transforms applied to it."""

    def __init__(self, kind, **params):
        self.kind, self.params = kind, params
        self.euler = np.zeros(3)
        self.pos = np.zeros(3)

    def difference(self, other):
        m = FakeMesh("gate", outer=np.asarray(self.params["extents"], np.float64),
                     inner=np.asarray(other.params["extents"], np.float64))
        return m

    def apply_transform(self, M):
        self.euler = np.asarray(M, np.float64)  # the recorded (ai, aj, ak) of euler_matrix, radians

    def apply_translation(self, t):
        self.pos = np.array(t, np.float64)


def install_trimesh():
    tm = types.ModuleType("trimesh")
    cr = types.ModuleType("trimesh.creation")
    tr = types.ModuleType("trimesh.transformations")
    ut = types.ModuleType("trimesh.util")
    cr.box = lambda extents=None, transform=None, **k: FakeMesh("box", extents=extents)  # noqa: E731
    cr.cylinder = lambda radius, height, **k: FakeMesh("cylinder", radius=radius, height=height)  # noqa: E731
    cr.icosphere = lambda radius=1.0, **k: FakeMesh("icosphere", radius=radius)  # noqa: E731
    cr.capsule = lambda radius=1.0, height=1.0, **k: FakeMesh("capsule", radius=radius, height=height)  # noqa: E731
    cr.cone = lambda radius, height, **k: FakeMesh("cone", radius=radius, height=height)  # noqa: E731
    tr.euler_matrix = lambda ai, aj, ak, axes="sxyz": (float(ai), float(aj), float(ak))  # noqa: E731
    tr.translation_matrix = lambda pos: np.asarray(pos)  # noqa: E731
    ut.concatenate = lambda meshes: meshes  # noqa: E731
    tm.creation, tm.transformations, tm.util, tm.Trimesh = cr, tr, ut, FakeMesh
    for name, mod in (("trimesh", tm), ("trimesh.creation", cr), ("trimesh.transformations", tr), ("trimesh.util", ut)):
        sys.modules[name] = mod


def load_reference():
    mods = il_shim.install()
    install_trimesh()

    def configclass(cls):
        def __init__(self, **kw):
            for k, v in kw.items():
                setattr(self, k, v)
        cls.__init__ = __init__
        return cls

    mods["omni.isaac.lab.utils"].configclass = configclass
    terr = mods["omni.isaac.lab.terrains"]
    terr.SubTerrainBaseCfg = type("SubTerrainBaseCfg", (), {"proportion": 1.0, "size": (10.0, 10.0)})
    terr.TerrainGeneratorCfg = type("TerrainGeneratorCfg", (), {"__init__": lambda self, **kw: self.__dict__.update(kw)})
    tmu = types.ModuleType("omni.isaac.lab.terrains.trimesh.utils")
    tmu.make_border = lambda *a, **k: []  # add_border is off in the task's configs
    sys.modules["omni.isaac.lab.terrains.trimesh"] = types.ModuleType("omni.isaac.lab.terrains.trimesh")
    sys.modules["omni.isaac.lab.terrains.trimesh.utils"] = tmu
    il_shim.synthetic_package("diff.lab.terrains", os.path.dirname(TRIMESH_DIR))
    pkg = il_shim.synthetic_package("diff.lab.terrains.trimesh", TRIMESH_DIR)
    il_shim.load("diff.lab.terrains.trimesh.utils", os.path.join(TRIMESH_DIR, "utils.py"), "diff.lab.terrains.trimesh")
    rt = il_shim.load("diff.lab.terrains.trimesh.racing_terrains", os.path.join(TRIMESH_DIR, "racing_terrains.py"),
                      "diff.lab.terrains.trimesh")
    pkg.racing_terrains = rt
    cfgm = il_shim.load("diff.lab.terrains.trimesh.racing_terrains_cfg",
                        os.path.join(TRIMESH_DIR, "racing_terrains_cfg.py"), "diff.lab.terrains.trimesh")
    for k in dir(cfgm):
        if k.endswith("Cfg"):
            setattr(pkg, k, getattr(cfgm, k))
    task = il_shim.load("grref_task_terrains", TASK_TERRAINS)
    return task.RacingComplexTerrainCfg


def gate_quat(gate_pose):
    """terrain_generator.py:64-73: the gate orientation the reference stores next to the position."""
    from scipy.spatial.transform import Rotation as R

    ori = R.from_euler("YXZ", np.stack([gate_pose[:, 3], -gate_pose[:, 4], gate_pose[:, 5]], axis=1), degrees=True)
    q = (ori * R.from_euler("XYZ", [-90, -90, 0], degrees=True)).as_quat()
    return np.concatenate([q[:, 3:], q[:, :3]], axis=1)  # w x y z


def main():
    gen = load_reference()
    out = {}
    cases = []
    for fam in ("zigzag", "circular", "ellipse"):
        for d in (0.05, 0.35, 0.65, 0.95):
            for obs in (False, True):
                for seed in (3, 11):
                    cases.append((fam, d, obs, seed))
    for c, (fam, d, obs, seed) in enumerate(cases):
        cfg = gen.sub_terrains[fam]
        cfg.size = gen.size
        cfg.add_obs = cfg.add_ground_obs = obs
        np.random.seed(seed)
        random.seed(seed + 1000)
        meshes, origin, extras = type(cfg).function(d, cfg)
        gates = [m for m in meshes if m.kind == "gate"]
        others = [m for m in meshes if m.kind != "gate"][:-1]  # the last mesh is the ground box
        p = f"c{c}_"
        out[p + "case"] = np.array([("zigzag", "circular", "ellipse").index(fam), d, int(obs), seed], np.float64)
        out[p + "gate_pose"] = extras["gate_pose"]
        out[p + "gate_quat"] = gate_quat(extras["gate_pose"])
        out[p + "next_gate_id"] = np.array([extras["next_gate_id"]])
        out[p + "origin"] = np.asarray(origin, np.float64)
        out[p + "gate_outer"] = np.stack([m.params["outer"] for m in gates])
        out[p + "gate_inner"] = np.stack([m.params["inner"] for m in gates])
        out[p + "gate_euler_rad"] = np.stack([m.euler for m in gates])
        out[p + "gate_pos"] = np.stack([m.pos for m in gates])
        rows = []
        for m in others:
            pr = m.params
            if m.kind == "box":
                size = np.asarray(pr["extents"], np.float64)
            elif m.kind in ("cylinder", "capsule", "cone"):
                size = np.array([pr["radius"], pr["radius"], pr["height"]])
            else:
                size = np.array([pr["radius"]] * 3)
            rows.append(np.concatenate([[KINDS[m.kind]], size, m.euler, m.pos]))
        out[p + "obstacles"] = np.array(rows, np.float64).reshape(-1, 10)
    out["num_cases"] = np.array([len(cases)])
    np.savez_compressed(OUT, **out)
    n_obs = sum(out[f"c{c}_obstacles"].shape[0] for c in range(len(cases)))
    print(f"wrote {OUT}: {len(cases)} cases, {n_obs} obstacles, "
          f"{sum(v.nbytes for v in out.values()) / 1e3:.1f} kB raw")


if __name__ == "__main__":
    main()
