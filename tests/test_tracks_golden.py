"""The build's track generator (generalizableracing_amd/envs/tracks.py) against the REFERENCE's own
generators (tests/golden/make_golden_tracks.py: ZigzagRacingTerrain / SquareRacingTrackTerrain /
EllipseRacingTerrain of trimesh/racing_terrains.py with the task's RacingComplexTerrainCfg).

The reference draws from NumPy's and Python's global generators; the build takes one stream of each as
arguments (gates and obstacles on separate streams in production).  Handed the same two streams for both
(the reference's draw order), every family must reproduce the reference's gate positions and Euler angles,
gate frame sizes, start gate, origin and — with add_obs / add_ground_obs on — every obstacle primitive
(kind, size, orientation, position) in order: 3 families x 4 difficulties x obstacles off/on x 2 seeds.
Positions, angles and the origin are bit-exact (the build follows the reference's fp32 / fp64 arithmetic);
sizes to 1e-12 (trimesh receives w + 2e where the build stores w and e)."""
import math
import os
import random

import numpy as np
import pytest

from generalizableracing_amd.envs import tracks

FAMILIES = {0: tracks.zigzag_track, 1: tracks.square_track, 2: tracks.ellipse_track}


@pytest.fixture(scope="module")
def gt():
    return dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_tracks.npz")))


def cases(gt):
    return range(int(gt["num_cases"][0]))


def run_case(gt, c):
    fam, d, obs, seed = gt[f"c{c}_case"]
    fam, obs, seed = int(fam), bool(obs), int(seed)
    gen = tracks.TrackGenCfg()
    cfg = [f for f in gen.families if f.kind == ("zigzag", "circular", "ellipse")[fam]][0]
    cfg.add_obs = cfg.add_ground_obs = obs
    rng, prng = np.random.RandomState(seed), random.Random(seed + 1000)
    return FAMILIES[fam](float(d), cfg, gen.size, rng, prng, rng, prng)


def test_gate_layouts_match_reference(gt):
    for c in cases(gt):
        tr = run_case(gt, c)
        p = f"c{c}_"
        pose = gt[p + "gate_pose"]
        # bit-exact: the same draws in the same order and the same fp32 / fp64 arithmetic as the reference
        np.testing.assert_array_equal(tr.gate_pts, gt[p + "gate_pos"], err_msg=f"case {c} gate positions")
        np.testing.assert_array_equal(tr.gate_pts.astype(np.float32), pose[:, :3], err_msg=f"case {c} gate_pose")
        np.testing.assert_array_equal(tr.gate_euler, pose[:, 3:6], err_msg=f"case {c} gate euler")
        assert tr.next_gate_id == int(gt[p + "next_gate_id"][0]), c
        np.testing.assert_array_equal(tr.origin, gt[p + "origin"], err_msg=f"case {c} origin")
        # make_gate(outer=(w + 2e, h + 2e, t), inner=(w, h, t), position, euler) per gate (trimesh/utils.py:10-33)
        outer = np.stack([tr.gate_w + 2 * tr.gate_e, tr.gate_h + 2 * tr.gate_e, tr.gate_t], 1)
        inner = np.stack([tr.gate_w, tr.gate_h, tr.gate_t], 1)
        np.testing.assert_allclose(outer, gt[p + "gate_outer"], rtol=1e-12, atol=1e-12, err_msg=f"case {c} outer")
        np.testing.assert_allclose(inner, gt[p + "gate_inner"], rtol=1e-12, atol=1e-12, err_msg=f"case {c} inner")
        np.testing.assert_allclose(np.radians(tr.gate_euler.astype(np.float64)), gt[p + "gate_euler_rad"],
                                   rtol=0, atol=1e-6, err_msg=f"case {c} gate mesh rotation")


def test_obstacles_match_reference(gt):
    total = 0
    for c in cases(gt):
        tr = run_case(gt, c)
        want = gt[f"c{c}_obstacles"]
        assert len(tr.obstacles) == want.shape[0], (c, len(tr.obstacles), want.shape[0])
        for k, (o, row) in enumerate(zip(tr.obstacles, want)):
            kind = int(row[0])
            assert o.kind == kind, (c, k)
            if kind == tracks.OBST_BOX:
                size = 2 * o.half
            elif kind == tracks.OBST_SPHERE:
                size = o.half
            else:  # cylinder / capsule: (radius, radius, height)
                size = np.array([o.half[0], o.half[1], 2 * o.half[2]])
            np.testing.assert_allclose(size, row[1:4], rtol=1e-12, atol=1e-12, err_msg=f"case {c} obstacle {k} size")
            np.testing.assert_array_equal(np.radians(o.euler), row[4:7], err_msg=f"case {c} obstacle {k} rotation")
            np.testing.assert_array_equal(o.pos, row[7:10], err_msg=f"case {c} obstacle {k} position")
        total += want.shape[0]
    assert total > 500


def test_gate_quaternion_and_frame_agree(gt):
    """The orientation the reference stores with each gate (terrain_generator.py:64-73:
    R.from_euler('YXZ', [e0, -e1, e2]) * R.from_euler('XYZ', [-90, -90, 0])) and the frame the build packs
    (make_gate's 'rxyz' rotation, tracks.euler_matrix_rxyz) describe the same gate: the stored frame's
    through-axis (z of make_gate's box, the frame's thickness direction) is the quaternion's body x (the
    direction a drone flies through the gate)."""
    for c in cases(gt):
        pose, q = gt[f"c{c}_gate_pose"], gt[f"c{c}_gate_quat"]
        for g in range(pose.shape[0]):
            R = tracks.euler_matrix_rxyz(pose[g, 3:6].astype(np.float64))
            w, x, y, z = q[g]
            qx = np.array([1 - 2 * (y * y + z * z), 2 * (x * y + w * z), 2 * (x * z - w * y)])
            assert abs(abs(float(np.dot(R[:, 2], qx))) - 1.0) < 1e-6, (c, g)
            assert math.isclose(np.linalg.norm(q[g]), 1.0, rel_tol=1e-9)
