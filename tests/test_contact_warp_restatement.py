"""The build's collision count against a float64 restatement of the reference's Warp lattice ray test, and the
lattice against an exact box collider — quantifying the contact reformulation.

Reference test (extensions/diff.lab/diff/lab/utils/mesh_tools.py:128-233, called from mdp/rewards.py:226-242
with arm_length 0.09, height 0.05): for each of the 17 lattice points (utils/__init__.py:19-37) scaled by
(0.707 arm, 0.707 arm, 0.5 height) and rotated by the drone's attitude, cast the six world-axis rays
(+-x, +-y, +-z) into the terrain mesh in that order; the point counts once as soon as a ray's FIRST hit is a back
face (Warp's `sign <= 0`), a front-face hit moves on to the next direction.  The terrain mesh here is restated from
trimesh/utils.py:10-33 (`make_gate`: outer box (w + 2e, h + 2e, t) minus the through-hole (w, h, t), Euler 'rxyz',
translated) as each frame's four bars, every bar a 12-triangle box with outward winding (as
trimesh.creation.box), and racing_terrains.py:144-150's ground box (40 x 40 x 1 m, top at the sub-terrain's
z = 0).  Möller–Trumbore in float64; the gate geometry comes from the track generator (Track objects), not from the
packed table the kernel and oracle read.

Build test (oracle/gr_oracle.c gro_collision_count, the kernel's arithmetic): a lattice point counts if it is inside
a frame (point in the outer box, not in the hole) or below the ground plane.  For closed meshes "first hit is a
back face" is point-in-solid, so the two must agree except where a point lies within round-off of a face.

Neither Warp nor trimesh is installed: this is a restatement, so the comparison quantifies the reformulation
(point-in-solid for the ray query) and is not reference parity.
"""
import math

import numpy as np
import pytest

import oracle
from generalizableracing_amd.envs import tracks as T
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg

LATTICE = np.array([[0, 0, 0], [1, 1, 1], [1, -1, 1], [-1, 1, 1], [-1, -1, 1], [1, 1, -1], [1, -1, -1], [-1, 1, -1],
                    [-1, -1, -1], [.5, .5, .5], [.5, -.5, .5], [-.5, .5, .5], [-.5, -.5, .5], [.5, .5, -.5],
                    [.5, -.5, -.5], [-.5, .5, -.5], [-.5, -.5, -.5]], np.float64)
ARM, HEIGHT = 0.09, 0.05
SCALE = np.array([0.707 * ARM, 0.707 * ARM, 0.5 * HEIGHT])
DIRS = np.array([[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]], np.float64)
MAX_DIST = 1e3
# trimesh.creation.box: 8 corners (+-1 per axis), 12 outward triangles
_CORNERS = np.array([[-1, -1, -1], [-1, -1, 1], [-1, 1, -1], [-1, 1, 1], [1, -1, -1], [1, -1, 1], [1, 1, -1],
                     [1, 1, 1]], np.float64)
_FACES = np.array([[1, 3, 0], [4, 1, 0], [0, 3, 2], [2, 4, 0], [1, 7, 3], [5, 1, 4], [5, 7, 1], [3, 7, 2],
                   [6, 4, 2], [2, 7, 6], [6, 5, 4], [7, 5, 6]])


def box_tris(lo, hi, R=np.eye(3), t=np.zeros(3)):
    """[12, 3, 3] triangles of the box [lo, hi] (local), rotated by R and translated by t, outward winding."""
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    v = (lo + hi) / 2 + _CORNERS * (hi - lo) / 2
    v = v @ R.T + t
    return v[_FACES]


def test_box_winding_is_outward():
    tri = box_tris([-1, -2, -3], [1, 2, 3])
    n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    c = tri.mean(1)
    assert (np.einsum("ij,ij->i", n, c) > 0).all()


def track_mesh(tr: T.Track, near_gate: int | None = None, reach: float = 3.0):
    """The track's gate frames (4 bars each) and ground box as triangles in the env-local frame.  near_gate: only
    the frames within `reach` m of that gate's centre (a drone sampled around it cannot be inside another frame, and
    for a point outside every solid any first hit is a front face whatever the rest of the mesh holds, so the
    count is the same as over the whole terrain mesh)."""
    tris = []
    c0 = None if near_gate is None else tr.gate_pts[near_gate].astype(np.float64)
    for g in range(len(tr.gate_pts)):
        if c0 is not None and np.linalg.norm(tr.gate_pts[g] - c0) > reach:
            continue
        c = tr.gate_pts[g].astype(np.float64) - tr.origin
        R = T.euler_matrix_rxyz(tr.gate_euler[g])
        hw, hh, ht, e = tr.gate_w[g] / 2, tr.gate_h[g] / 2, tr.gate_t[g] / 2, tr.gate_e[g]
        how, hoh = hw + e, hh + e
        for lo, hi in (((-how, hh, -ht), (how, hoh, ht)), ((-how, -hoh, -ht), (how, -hh, ht)),
                       ((-how, -hh, -ht), (-hw, hh, ht)), ((hw, -hh, -ht), (how, hh, ht))):
            tris.append(box_tris(lo, hi, R, c))
    # ground box: x, y in [0, 40] m of the sub-terrain, z in [-1, 0]
    tris.append(box_tris((0.0, 0.0, -1.0), (40.0, 40.0, 0.0), np.eye(3), -tr.origin))
    return np.concatenate(tris)


def warp_count64(tris, pts):
    """mesh_tools.py:186-233 over `pts` [P, 3] (the lattice points of one drone): the number of points one of whose
    six axis rays first hits a back face (the kernel's loop stops at the first such direction, so a point counts
    once; evaluated here for every (point, direction) ray at once)."""
    v0, e1, e2 = tris[:, 0], tris[:, 1] - tris[:, 0], tris[:, 2] - tris[:, 0]
    n = np.cross(e1, e2)
    o = np.repeat(np.asarray(pts, np.float64), len(DIRS), axis=0)[:, None, :]  # [R, 1, 3], R = P * 6
    d = np.tile(DIRS, (len(pts), 1))[:, None, :]
    pv = np.cross(d, e2[None])  # [R, T, 3]
    det = np.einsum("tk,rtk->rt", e1, pv)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / det
        s = o - v0[None]
        u = np.einsum("rtk,rtk->rt", s, pv) * inv
        qv = np.cross(s, e1[None])
        v = np.einsum("rtk,rk->rt", qv, d[:, 0]) * inv
        t = np.einsum("tk,rtk->rt", e2, qv) * inv
        ok = (np.abs(det) > 1e-18) & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 0) & (t < MAX_DIST)
    tt = np.where(ok, t, np.inf)
    first = tt.argmin(1)
    hit = np.isfinite(tt[np.arange(len(tt)), first])
    back = hit & (np.einsum("rk,rk->r", n[first], d[:, 0]) >= 0.0)  # back face (Warp: sign <= 0)
    return int(back.reshape(len(pts), len(DIRS)).any(1).sum())


def quat_matrix64(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def lattice_points(p, q):
    return p + (LATTICE * SCALE) @ quat_matrix64(q).T


def box_overlaps_frame(p, q, tr: T.Track, near_gate: int, reach: float = 3.0):
    """Exact test: does the drone's box collider (half extents 0.707 arm, 0.707 arm, 0.5 height — the box the
    lattice samples) intersect a bar of any frame or the ground box?  Separating-axis test in float64."""
    Rd = quat_matrix64(q)
    hd = SCALE
    boxes = []
    c0 = tr.gate_pts[near_gate].astype(np.float64)
    for g in range(len(tr.gate_pts)):
        if np.linalg.norm(tr.gate_pts[g] - c0) > reach:
            continue
        c = tr.gate_pts[g].astype(np.float64) - tr.origin
        R = T.euler_matrix_rxyz(tr.gate_euler[g])
        hw, hh, ht, e = tr.gate_w[g] / 2, tr.gate_h[g] / 2, tr.gate_t[g] / 2, tr.gate_e[g]
        how, hoh = hw + e, hh + e
        for lo, hi in (((-how, hh, -ht), (how, hoh, ht)), ((-how, -hoh, -ht), (how, -hh, ht)),
                       ((-how, -hh, -ht), (-hw, hh, ht)), ((hw, -hh, -ht), (how, hh, ht))):
            lo, hi = np.array(lo), np.array(hi)
            boxes.append((c + R @ ((lo + hi) / 2), R, (hi - lo) / 2))
    boxes.append((np.array([20.0, 20.0, -0.5]) - tr.origin, np.eye(3), np.array([20.0, 20.0, 0.5])))
    for cb, Rb, hb in boxes:
        axes = [Rd[:, i] for i in range(3)] + [Rb[:, i] for i in range(3)]
        axes += [np.cross(Rd[:, i], Rb[:, j]) for i in range(3) for j in range(3)]
        d = cb - p
        sep = False
        for a in axes:
            na = np.linalg.norm(a)
            if na < 1e-12:
                continue
            a = a / na
            ra = np.abs(Rd.T @ a) @ hd
            rb = np.abs(Rb.T @ a) @ hb
            if abs(d @ a) > ra + rb:
                sep = True
                break
        if not sep:
            return True
    return False


def sample_poses(tracks, rng, n):
    """Poses near gate frames: a random gate of a random track, a position uniform in the frame's outer box grown
    by 0.15 m per side (bars, hole and surroundings), a uniformly random attitude; one in ten near the ground."""
    out = []
    ks = list(range(len(tracks)))
    for _ in range(n):
        k = int(rng.choice(ks))
        tr = tracks[k]
        g = int(rng.integers(len(tr.gate_pts)))
        c = tr.gate_pts[g].astype(np.float64) - tr.origin
        R = T.euler_matrix_rxyz(tr.gate_euler[g])
        hw, hh, ht, e = tr.gate_w[g] / 2, tr.gate_h[g] / 2, tr.gate_t[g] / 2, tr.gate_e[g]
        m = 0.15
        loc = rng.uniform(-1, 1, 3) * np.array([hw + e + m, hh + e + m, ht + m])
        p = c + R @ loc
        if rng.random() < 0.1:
            p[2] = -tr.origin[2] + rng.uniform(-0.06, 0.06)
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        out.append((k, g, p.astype(np.float32), q.astype(np.float32)))
    return out


@pytest.fixture(scope="module")
def setup():
    cfg = T.TrackGenCfg(seed=42, num_rows=10, num_cols=20).with_gates(8)
    cfg.with_obstacles(False)
    tracks_2d = T.generate_tracks(cfg)
    gates, recs = T.pack_tracks(tracks_2d, 8, 0.1)
    flat = [tracks_2d[t][lv] for t in range(len(tracks_2d)) for lv in range(len(tracks_2d[0]))]
    gcfg = RacingEnvCfg(scene=SceneCfg(num_envs=16), sim=SimCfg(device="cpu"), stage=1).to_gr_config()
    assert np.allclose(list(gcfg.collider_half), SCALE, rtol=1e-6)  # the build's lattice box is the reference's
    return flat, oracle.Oracle(gcfg, gates, recs)


def test_warp_restatement_known_answers(setup):
    flat, _ = setup
    tr = flat[0]
    tris = track_mesh(tr)
    c = tr.gate_pts[0].astype(np.float64) - tr.origin
    R = T.euler_matrix_rxyz(tr.gate_euler[0])
    hh, e = tr.gate_h[0] / 2, tr.gate_e[0]
    # single points: the centre of the top bar is inside, the centre of the hole is not; a level drone centred in
    # the hole touches nothing
    q0 = np.array([1.0, 0, 0, 0])
    top = c + R @ np.array([0, hh + e / 2, 0])
    assert warp_count64(tris, top[None]) == 1
    assert warp_count64(tris, c[None]) == 0
    assert warp_count64(tris, lattice_points(c, q0)) == 0
    # under the ground: every point; 1 m above it, away from the gates: none
    far = np.array([20.0, 20.0, 0.0]) - tr.origin
    assert warp_count64(tris, lattice_points(far + [0, 0, -0.3], q0)) == 17
    assert warp_count64(tris, lattice_points(far + [0, 0, 1.0], q0)) == 0


def test_build_count_matches_warp_restatement(setup):
    """>= 10^4 poses near gates: the build's count equals the Warp restatement's except within round-off of a face
    (none expected at this sample size); both contact predicates (count >= 1: stage 1 / 2, count > 2: stage 0)."""
    flat, orc = setup
    rng = np.random.default_rng(2025)
    poses = sample_poses(flat, rng, 10000)
    meshes = {}
    diff_count = diff_contact = diff_stage0 = contacts = 0
    for k, g, p, q in poses:
        if (k, g) not in meshes:
            meshes[(k, g)] = track_mesh(flat[k], near_gate=g)
        want = warp_count64(meshes[(k, g)], lattice_points(p.astype(np.float64), q.astype(np.float64)))
        got = orc.collision_count(k, p, q)
        diff_count += got != want
        diff_contact += (got >= 1) != (want >= 1)
        diff_stage0 += (got > 2) != (want > 2)
        contacts += want >= 1
    n = len(poses)
    print(f"poses {n}, contact {contacts / n:.3f}; count differs {diff_count}, contact predicate {diff_contact}, "
          f"stage-0 predicate {diff_stage0}")
    assert contacts > 0.2 * n  # the sample exercises the frames
    assert diff_count <= 1e-3 * n and diff_contact <= 1e-3 * n and diff_stage0 <= 1e-3 * n


def test_lattice_against_exact_box_collider(setup):
    """The 17-point lattice (both the reference's ray test and the build sample the drone's box with it) against
    an exact box-vs-bar / box-vs-ground overlap: the lattice misses shallow corner and edge contacts, never reports
    a contact the box does not have.  The rate is what the reformulation shares with the reference's stage-0 test;
    PhysX contact (stages 1 / 2) is closer to the exact overlap."""
    flat, orc = setup
    rng = np.random.default_rng(7)
    poses = sample_poses(flat, rng, 3000)
    box_only = lattice_only = both = 0
    for k, g, p, q in poses:
        lat = orc.collision_count(k, p, q) >= 1
        box = box_overlaps_frame(p.astype(np.float64), q.astype(np.float64), flat[k], g)
        both += lat and box
        box_only += box and not lat
        lattice_only += lat and not box
    n = len(poses)
    print(f"poses {n}: both {both}, exact box only {box_only} ({box_only / n:.3%}), lattice only {lattice_only}")
    assert lattice_only == 0
    assert box_only < 0.1 * n
