"""Track obstacles (walls, orbits, ground obstacles): generator, grid, collision and camera.

Reference: the sub-terrain generators' obstacle loops (extensions/diff.lab/diff/lab/terrains/trimesh/
racing_terrains.py:87-150 circular, :254-319 square, :510-610 zigzag, :750-815 ellipse) and the
primitives make_wall / make_orbit / make_ground_high_obs / make_ground_little_obj
(trimesh/utils.py:35-131), enabled by RacingComplexTerrainCfg (quadcopter_diff/terrains/
racing_terrains.py:137-210).  trimesh, PhysX and Warp are not installed, so parity against the
reference's own mesh / contact / ray results is unpinned: the oracle (shared fp32 functions of
gr_obstacles.h) is held here to an independent float64 restatement of the primitives, and the
HIP kernels are held to the oracle bit for bit by the -m gpu tests."""
from __future__ import annotations

import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402

from generalizableracing_amd import _abi  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs import tracks as T  # noqa: E402

LATTICE = np.array([[0, 0, 0], [1, 1, 1], [1, -1, 1], [-1, 1, 1], [-1, -1, 1], [1, 1, -1], [1, -1, -1],
                    [-1, 1, -1], [-1, -1, -1]] + [[sx * .5, sy * .5, sz * .5] for sz in (1, -1) for sx in (1, -1)
                                                   for sy in (1, -1)], dtype=np.float64)


@pytest.fixture(scope="module")
def gen():
    cfg = T.TrackGenCfg()
    tracks = T.generate_tracks(cfg)
    return cfg, tracks, T.pack_obstacles(tracks, 0.1)


def gr_cfg(n=16):
    return RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=1).to_gr_config()


def isolated_oracle(ot, n=16):
    """Oracle whose gates sit far above and ground far below: counts / depths come from obstacles only."""
    ntr = ot.records.shape[0]
    gates = np.zeros((ntr, 8, 20), np.float32)
    gates[:, :, 2] = 1000.0
    gates[:, :, 3] = 1.0
    gates[:, :, 4] = gates[:, :, 9] = gates[:, :, 14] = 1.0  # identity frames
    gates[:, :, 7] = gates[:, :, 11] = gates[:, :, 15] = gates[:, :, 16] = gates[:, :, 17] = 0.1
    recs = np.zeros((ntr, 4), np.float32)
    recs[:, 0] = -1000.0
    recs[:, 3] = 8
    return oracle.Oracle(gr_cfg(n), gates, recs, ot.records, ot.counts)


# ------------------------------------------------------------------ float64 restatement
def quat_matrix(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def inside64(o: T.Obstacle, origin, x):
    """point x (env-local, float64) inside primitive o (generator record, sub-terrain frame)"""
    R = T.euler_matrix_rxyz(np.asarray(o.euler))
    l = R.T @ (np.asarray(x) - (o.pos - origin))
    h = o.half
    if o.kind == T.OBST_BOX:
        return bool(np.all(np.abs(l) <= h))
    rad = l[0] ** 2 + l[1] ** 2
    if o.kind == T.OBST_CYLINDER:
        return rad <= h[0] ** 2 and abs(l[2]) <= h[2]
    if o.kind == T.OBST_SPHERE:
        return rad + l[2] ** 2 <= h[0] ** 2
    dz = max(abs(l[2]) - h[2], 0.0)
    return rad + dz * dz <= h[0] ** 2


def sdf_margin(o: T.Obstacle, origin, x):
    """rough distance of x to the primitive's surface (for excusing boundary cases)"""
    R = T.euler_matrix_rxyz(np.asarray(o.euler))
    l = np.abs(R.T @ (np.asarray(x) - (o.pos - origin)))
    h = o.half
    if o.kind == T.OBST_BOX:
        return float(np.min(np.abs(l - h)))
    rad = math.hypot(l[0], l[1])
    if o.kind == T.OBST_CYLINDER:
        return min(abs(rad - h[0]), abs(l[2] - h[2]))
    if o.kind == T.OBST_SPHERE:
        return abs(np.linalg.norm(l) - h[0])
    dz = max(l[2] - h[2], 0.0)
    return abs(math.hypot(rad, dz) - h[0])


# ------------------------------------------------------------------ generator
def test_generator_counts_follow_the_reference_loops(gen):
    cfg, tracks, ot = gen
    fams = T.column_families(cfg)
    for col, colv in enumerate(tracks):
        f = cfg.families[fams[col]]
        for row, tr in enumerate(colv):
            G = len(tr.gate_pts)
            n = len(tr.obstacles)
            walls = sum(1 for o in tr.obstacles if o.kind == T.OBST_BOX and o.half[2] <= f.wall_thickness[1] / 2 + 1e-9
                        and np.any(o.euler != 0))
            if f.kind == "zigzag":
                segs = G - 1  # no wrap-around segment (:518)
                lo = segs * (f.num_wall_seg[0] + f.num_orbit_seg[0] + f.num_ground_obs[0])
                hi = segs * (f.num_wall_seg[1] + f.num_orbit_seg[1] + f.num_ground_obs[1] + 4)
            elif f.kind == "circular":
                segs = G - 1  # the start segment carries none (:247-249)
                lo, hi = 0, segs * (f.num_wall_seg[1] + f.num_orbit_seg[1] + f.num_ground_obs[1] + 4)
            else:
                segs = G - 1
                lo = segs * (f.num_wall_seg[0] + f.num_orbit_seg[0] + f.num_ground_obs[0] + 1)
                hi = segs * (f.num_wall_seg[1] + f.num_orbit_seg[1] + f.num_ground_obs[1] + 2)
            assert lo <= n <= hi, (f.kind, row, n, lo, hi)
            assert walls <= n
            assert ot.counts[col * len(colv) + row] == n
    kinds = np.concatenate([ot.records[k, :ot.counts[k], 16] for k in range(len(ot.counts))])
    assert set(np.unique(kinds).astype(int)) == {T.OBST_BOX, T.OBST_CYLINDER, T.OBST_SPHERE, T.OBST_CAPSULE}


def test_primitive_sizes_and_placement(gen):
    _, tracks, _ = gen
    for colv in tracks:
        for tr in colv:
            for o in tr.obstacles:
                assert np.all(o.half > 0)
                if np.all(o.euler == 0) and o.kind in (T.OBST_BOX, T.OBST_CYLINDER):
                    # ground obstacles stand on (or sink into) the ground plane z = 0
                    assert o.pos[2] - o.half[2] <= 0.5 + 1e-9
                if o.kind == T.OBST_CAPSULE:
                    assert 0.1 <= o.half[0] <= 0.3 and 0.1 <= o.half[2] <= 0.3


def test_obstacles_off_and_gate_stream_independent():
    a = T.generate_tracks(T.TrackGenCfg().with_obstacles(False))
    b = T.generate_tracks(T.TrackGenCfg())
    for ca, cb in zip(a, b):
        for ta, tb in zip(ca, cb):
            assert not ta.obstacles
            np.testing.assert_array_equal(ta.gate_pts, tb.gate_pts)
            np.testing.assert_array_equal(ta.origin, tb.origin)


def test_grid_cells_are_conservative(gen):
    """The list the step kernel reads (the pre-step cell's, grown by the per-step margin, when the drone
    stayed within it; else the post-step cell's) holds every obstacle whose cull sphere holds the post-step
    point; points outside the grid have no obstacle in reach.  fp32 arithmetic as in the kernel."""
    _, _, ot = gen
    rng = np.random.default_rng(3)
    f32 = np.float32
    n_pre = n_post = 0
    for k in range(0, ot.records.shape[0], 5):
        n = ot.counts[k]
        recs = ot.records[k, :n]
        gf, gi = ot.grid_f[k], ot.grid_i[k]
        centres = recs[rng.integers(0, n, 400), :3].astype(np.float64)
        p0s = (centres + rng.uniform(-2.5, 2.5, (400, 3))).astype(np.float32)
        moves = rng.uniform(-0.7, 0.7, (400, 3)).astype(np.float32)
        for p0, mv in zip(p0s, moves):
            p = (p0 + mv).astype(np.float32)
            d2 = ((p[None, :] - recs[:, :3]) ** 2).astype(np.float32)
            near = set(np.nonzero((d2[:, 0] + d2[:, 1]) + d2[:, 2] <= recs[:, 3])[0].tolist())

            def cell(x):
                fx, fy = f32(f32(x[0] - gf[0]) * gf[2]), f32(f32(x[1] - gf[1]) * gf[2])
                return fx, fy, (fx >= 0 and fy >= 0 and fx < gi[0] and fy < gi[1])

            fx0, fy0, in0 = cell(p0)
            fx, fy, inp = cell(p)
            m = gf[3]
            cx0, cy0 = f32(int(fx0)), f32(int(fy0))
            if in0 and cx0 - m <= fx <= cx0 + 1 + m and cy0 - m <= fy <= cy0 + 1 + m:
                c = gi[2] + int(cy0) * gi[0] + int(cx0)
                n_pre += 1
            elif inp:
                c = gi[2] + int(fy) * gi[0] + int(fx)
                n_post += 1
            else:
                assert not near
                continue
            first, cnt = ot.cells[c]
            listed = ot.items[first:first + cnt]
            for j in near:
                assert any(np.array_equal(recs[j], it) for it in listed), (k, p, j)
    assert n_pre > 10 * n_post > 0


# ------------------------------------------------------------------ collision
def test_collision_known_answers():
    """Axis-aligned unit box / sphere / cylinder / capsule at the origin: a level drone at the centre has all
    17 lattice points inside; just beyond the surface (by more than the drone's half extents) none."""
    hx, hz = 0.707 * 0.09, 0.025
    cases = [(T.OBST_BOX, (0.5, 0.5, 0.5)), (T.OBST_SPHERE, (0.5, 0.5, 0.5)), (T.OBST_CYLINDER, (0.5, 0.5, 0.5)),
             (T.OBST_CAPSULE, (0.3, 0.3, 0.3))]
    for kind, half in cases:
        tr = T.Track(np.zeros((2, 3)), np.zeros((2, 3)), np.ones(2), np.ones(2), np.ones(2), np.ones(2),
                     np.zeros(3), 0, [T.Obstacle(kind, np.zeros(3), np.zeros(3), np.array(half, float))])
        ot = T.pack_obstacles([[tr]], 0.1)
        orc = isolated_oracle(ot)
        q = np.array([1, 0, 0, 0], np.float32)
        assert orc.collision_count(0, np.zeros(3, np.float32), q) == 17, kind
        top = half[2] + (half[2] if kind == T.OBST_CAPSULE else 0.0)
        assert orc.collision_count(0, np.array([0, 0, top + hz + 1e-3], np.float32), q) == 0, kind
        # half the drone below the top surface: the 4 + 1 lower corners / half-corners... at least the z<0 layer
        c = orc.collision_count(0, np.array([0, 0, top - 1e-3], np.float32), q)
        assert 8 <= c < 17, (kind, c)
        side = half[0] + hx * 1.5 + 1e-3
        assert orc.collision_count(0, np.array([side, 0, 0], np.float32), q) == 0, kind


def test_collision_matches_float64_restatement(gen):
    """Random drone poses around random obstacles: the oracle's lattice count (fp32, gr_obstacles.h) equals
    a float64 count over the generator's primitives, except for lattice points within 1e-5 m of a surface."""
    _, tracks, ot = gen
    orc = isolated_oracle(ot)
    h = np.array([0.707 * 0.09, 0.707 * 0.09, 0.025])
    rng = np.random.default_rng(7)
    L = len(tracks[0])
    checked = excused = hits = 0
    for k in range(0, ot.records.shape[0], 3):
        tr = tracks[k // L][k % L]
        obs = tr.obstacles
        for _ in range(40):
            o = obs[rng.integers(len(obs))]
            c = o.pos - tr.origin
            p = c + rng.uniform(-1, 1, 3) * (T.obstacle_radius(o) + 0.05)
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            p32, q32 = p.astype(np.float32), q.astype(np.float32)
            got = orc.collision_count(k, p32, q32)
            R = quat_matrix(q32.astype(np.float64))
            pts = [p32.astype(np.float64) + R @ (l * h) for l in LATTICE]
            cand = [ob for ob in obs if np.linalg.norm(ob.pos - tr.origin - p) < T.obstacle_radius(ob) + 0.1]
            want = sum(any(inside64(ob, tr.origin, x) for ob in cand) for x in pts)
            checked += 1
            hits += got > 0
            if got != want:
                margin = min(sdf_margin(ob, tr.origin, x) for ob in cand for x in pts)
                assert margin < 1e-5, (k, p, q, got, want, margin)
                excused += 1
    assert hits > checked // 5
    assert excused <= max(2, checked // 200)


# ------------------------------------------------------------------ camera
def ray_first64(o: T.Obstacle, origin, ro, rd):
    """first surface crossing s > 0 of ro + s rd with primitive o, float64 (np.inf if none)"""
    R = T.euler_matrix_rxyz(np.asarray(o.euler))
    lo = R.T @ (ro - (o.pos - origin))
    ld = R.T @ rd
    h = o.half

    def first(tin, tout):
        if not (tin <= tout) or not (tout > 0):
            return np.inf
        return tin if tin > 0 else tout

    def sphere(zc, r):
        oc = lo - np.array([0, 0, zc])
        a, b, c = ld @ ld, oc @ ld, oc @ oc - r * r
        disc = b * b - a * c
        if disc < 0:
            return np.inf
        s = math.sqrt(disc)
        return first((-b - s) / a, (-b + s) / a)

    def slab(o_, d_, hh):
        if abs(d_) < 1e-20:
            return (-np.inf, np.inf) if abs(o_) <= hh else (1.0, -1.0)
        t0, t1 = (-hh - o_) / d_, (hh - o_) / d_
        return min(t0, t1), max(t0, t1)

    if o.kind == T.OBST_BOX:
        iv = [slab(lo[j], ld[j], h[j]) for j in range(3)]
        return first(max(v[0] for v in iv), min(v[1] for v in iv))
    if o.kind == T.OBST_SPHERE:
        return sphere(0.0, h[0])
    zlo, zhi = slab(lo[2], ld[2], h[2])
    a = ld[0] ** 2 + ld[1] ** 2
    b = lo[0] * ld[0] + lo[1] * ld[1]
    c = lo[0] ** 2 + lo[1] ** 2 - h[0] ** 2
    disc = b * b - a * c
    if a < 1e-12 or disc < 0:
        cyl = np.inf if (a >= 1e-12 or c > 0) else first(zlo, zhi)
    else:
        s = math.sqrt(disc)
        cyl = first(max(zlo, (-b - s) / a), min(zhi, (-b + s) / a))
    if o.kind == T.OBST_CYLINDER:
        return cyl
    return min(cyl, sphere(h[2], h[0]), sphere(-h[2], h[0]))


def test_camera_obstacle_depth_matches_float64_caster(gen):
    _, tracks, ot = gen
    orc = isolated_oracle(ot)
    cam = CameraCfg()
    orc.enable_camera(cam.to_gr())
    rng = np.random.default_rng(11)
    L = len(tracks[0])
    total = bad = hit = 0
    for k in range(0, ot.records.shape[0], 23):
        tr = tracks[k // L][k % L]
        for _ in range(3):
            o = tr.obstacles[rng.integers(len(tr.obstacles))]
            target = o.pos - tr.origin
            p = target + rng.uniform(-1, 1, 3) * 3.0
            yaw = math.atan2(target[1] - p[1], target[0] - p[0]) + rng.uniform(-0.3, 0.3)
            q = np.array([math.cos(yaw / 2), 0, 0, math.sin(yaw / 2)], np.float32)
            p32 = p.astype(np.float32)
            oo, c0, c1, c2, ra, rb = orc.camera_frame(p32, q)
            near = [ob for ob in tr.obstacles
                    if np.linalg.norm(ob.pos - tr.origin - oo) < cam.max_distance + T.obstacle_radius(ob)]
            for _ in range(60):
                u, v = int(rng.integers(cam.width)), int(rng.integers(cam.height))
                got = orc.camera_ray(k, p32, q, u, v)
                rd = c0.astype(np.float64) + float(ra[u]) * c1.astype(np.float64) + float(rb[v]) * c2.astype(np.float64)
                want = min(ray_first64(ob, tr.origin, oo.astype(np.float64), rd) for ob in near)
                want = min(want, cam.max_distance)
                total += 1
                hit += want < cam.max_distance
                if not abs(got - want) <= 1e-4 * max(1.0, want):
                    bad += 1
    assert hit > total // 20, (hit, total)
    assert bad <= max(2, total // 300), (bad, total)


def test_camera_obstacle_known_answers():
    """A unit box / sphere straight ahead at 3 m: the centre pixel reads the near face distance."""
    cam = CameraCfg(offset_rot=(1.0, 0.0, 0.0, 0.0), offset_pos=(0.0, 0.0, 0.0))
    for kind, half, near in ((T.OBST_BOX, (0.5, 0.5, 0.5), 2.5), (T.OBST_SPHERE, (0.5, 0.5, 0.5), 2.5),
                             (T.OBST_CYLINDER, (0.5, 0.5, 0.5), 2.5), (T.OBST_CAPSULE, (0.4, 0.4, 0.3), 2.6)):
        tr = T.Track(np.zeros((2, 3)), np.zeros((2, 3)), np.ones(2), np.ones(2), np.ones(2), np.ones(2),
                     np.zeros(3), 0, [T.Obstacle(kind, np.array([3.0, 0, 0]), np.zeros(3), np.array(half, float))])
        orc = isolated_oracle(T.pack_obstacles([[tr]], 0.1))
        orc.enable_camera(cam.to_gr())
        p = np.zeros(3, np.float32)
        q = np.array([1, 0, 0, 0], np.float32)
        _, _, _, _, ra, rb = orc.camera_frame(p, q)
        u, v = int(np.argmin(np.abs(ra))), int(np.argmin(np.abs(rb)))
        d = orc.camera_ray(0, p, q, u, v)
        assert abs(d - near) < 0.02, (kind, d)
        # looking away: nothing within range
        qb = np.array([0, 0, 0, 1], np.float32)
        assert orc.camera_ray(0, p, qb, u, v) == pytest.approx(cam.max_distance)


def test_camera_tile_cull_is_conservative():
    """camera_kernel's per-tile cull (gr_cam_gate_outside / gr_cam_obst_outside: the bounding box beyond a side
    plane of the 8x32 tile's frustum; kernel-only, the oracle tests every window pixel) never removes a (tile,
    gate or obstacle) pair with a pixel the per-pixel test hits, at poses all around the obstacles and through the
    gates (close, grazing, the window-is-the-whole-screen case of a box reaching behind the camera) — and it
    removes many pairs."""
    gates, recs, ot = T.build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42)
    orc = oracle.Oracle(gr_cfg(16), gates, recs, ot.records, ot.counts)
    orc.enable_camera(CameraCfg().to_gr())
    rng = np.random.default_rng(5)
    tot = np.zeros((2, 4), np.int64)
    for k in range(0, ot.records.shape[0], 7):
        for j in range(8):
            if j % 2:  # near an obstacle
                centre = ot.records[k, rng.integers(ot.counts[k]), 0:3]
            else:  # in or near a gate's frame
                centre = gates[k, rng.integers(gates.shape[1]), 0:3]
            p = (centre + rng.uniform(-1, 1, 3) * rng.choice([0.3, 1.5, 4.0])).astype(np.float32)
            roll, pitch, yaw = rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(-math.pi, math.pi)
            R = T.euler_matrix_rxyz(np.array([roll, pitch, yaw]))
            w = math.sqrt(max(1e-12, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
            q = np.array([w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w)],
                         np.float32)
            q /= np.linalg.norm(q)
            r = orc.camera_cull_check(k, p, q)
            assert r[0, 2] == 0 and r[1, 2] == 0, (k, p, q, r)
            tot += r
    print("[gates, obstacles] x [pairs, culled, culled with a hit, culled window pixels]:", tot.tolist())
    assert tot[0, 1] > tot[0, 0] // 10 and tot[1, 1] > tot[1, 0] // 4, tot
