"""Procedural racing tracks -> the device track table.

Restates the three gate-layout families the task uses
(`RacingComplexTerrainCfg`, extensions/diff.lab_tasks/.../quadcopter_diff/terrains/racing_terrains.py:137-210):

  columns 0-5   "zigzag"   ZigzagRacingTerrain        (extensions/diff.lab/diff/lab/terrains/trimesh/racing_terrains.py:423-620)
  columns 6-11  "circular" SquareRacingTrackTerrain   (same file :167-336)
  columns 12-19 "ellipse"  EllipseRacingTerrain       (same file :625-832)

laid out as Isaac Lab's curriculum generator does: one family per column by
proportion (0.3 / 0.3 / 0.4), difficulty (row + U(0,1)) / num_rows per row,
table indexed [col=type][row=level] (terrain_importer.py:150-153).

Only what the env step consumes is produced: gate centres relative to the
env origin (terrain_generator.py:66-67), the frame geometry (make_gate,
trimesh/utils.py:10-33) for the collision test, the ground height below the
origin, the start gate, and the obstacles of `add_obs` / `add_ground_obs`
(walls, "orbits", ground-high obstacles and small ground objects,
trimesh/utils.py:35-131) as analytic primitives (box, cylinder, sphere,
capsule) for the collision test and the depth camera.  Mesh building / PhysX
import are not: there is no mesh anywhere in this build.
Exact layouts are not reproducible (the reference draws from Python's and
NumPy's global RNGs inside Isaac Lab's generator): same families, same
parameter ranges, our own seeded streams (gates and obstacles on separate
streams, so the gate layouts do not depend on whether obstacles are drawn).
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field

import numpy as np

from .._abi import GATE_FLOATS, OBST_FLOATS, TRACK_FLOATS


@dataclass
class FamilyCfg:
    kind: str
    proportion: float
    num_gate: int = 8
    gate_size: tuple = (0.8, 1.2)
    gate_thickness: tuple = (0.03, 0.06)
    pos_noise_scale: tuple = (0.2, 1.0)
    pos_z_noise_scale: tuple = (0.1, 1.0)
    rot_noise_scale: tuple = (0.0, 30.0)
    only_yaw: bool = True
    radius: tuple = (5.0, 8.0)
    track_length: float = 35.0
    gate_distance: float = 5.0
    short_axis_prop: tuple = (1.414, 0.8)
    long_axis_prop: tuple = (3.1414, 4.8)
    edge: tuple = (0.15, 0.25)
    # obstacles (trimesh/racing_terrains_cfg.py; values of RacingComplexTerrainCfg)
    add_obs: bool = True
    add_ground_obs: bool = True
    num_wall_seg: tuple = (1, 4)
    wall_size: tuple = (0.4, 1.0)
    wall_thickness: tuple = (0.04, 0.08)
    num_orbit_seg: tuple = (1, 4)
    num_ground_obs: tuple = (1, 4)
    adj_dir_shift_prop: tuple = (0.6, 0.6)
    radius_dir_shift_prop: tuple = (0.5, 0.5)
    no_obs_range: float = 1.5


@dataclass
class TrackGenCfg:
    """RacingComplexTerrainCfg (racing_terrains.py:137-210)."""

    seed: int = 42
    size: tuple = (40.0, 40.0)
    num_rows: int = 10
    num_cols: int = 20
    difficulty_range: tuple = (0.0, 1.0)
    families: list = field(default_factory=lambda: [
        FamilyCfg("zigzag", 0.3, pos_noise_scale=(1.0, 4.0), pos_z_noise_scale=(0.1, 1.0),
                  num_wall_seg=(2, 6), num_orbit_seg=(2, 6), num_ground_obs=(1, 4), radius_dir_shift_prop=(6, 6)),
        FamilyCfg("circular", 0.3, radius=(5.0, 8.0)),
        FamilyCfg("ellipse", 0.4, edge=(0.15, 0.22), num_ground_obs=(1, 2)),
    ])

    def with_gates(self, n: int) -> "TrackGenCfg":
        for f in self.families:
            f.num_gate = n
        return self

    def with_obstacles(self, on: bool) -> "TrackGenCfg":
        for f in self.families:
            f.add_obs = f.add_ground_obs = bool(on)
        return self


@dataclass
class Track:
    gate_pts: np.ndarray   # [G,3] sub-terrain frame
    gate_euler: np.ndarray  # [G,3] degrees, trimesh 'rxyz'
    gate_w: np.ndarray
    gate_h: np.ndarray
    gate_t: np.ndarray
    gate_e: np.ndarray
    origin: np.ndarray     # [3] sub-terrain frame
    next_gate_id: int
    obstacles: list = field(default_factory=list)  # [Obstacle]


# obstacle primitive kinds (the GR_OBST_* codes of include/gr.h)
OBST_BOX, OBST_CYLINDER, OBST_SPHERE, OBST_CAPSULE = 0, 1, 2, 3


@dataclass
class Obstacle:
    """One obstacle primitive in the sub-terrain frame.  `half`: box half extents |
    cylinder (r, r, half height) | sphere (r, r, r) | capsule (r, r, half segment), all
    along / about the local z axis as trimesh.creation builds them; `euler` in degrees,
    trimesh 'rxyz' (make_wall / make_orbit, trimesh/utils.py:35-83)."""

    kind: int
    pos: np.ndarray
    euler: np.ndarray
    half: np.ndarray


def _shape_noise(rng, n, gate_size, gate_thickness, edge):
    w = gate_size + rng.uniform(-0.05, 0.05, n)
    h = gate_size + rng.uniform(-0.05, 0.05, n)
    t = gate_thickness + rng.uniform(-1, 1, n) / 5 * gate_thickness
    e = rng.uniform(edge[0], edge[1], n)
    return w, h, t, e


def _lerp(rng_pair, d):
    return d * (rng_pair[1] - rng_pair[0]) + rng_pair[0]


# ---------------------------------------------------------------- obstacles
# trimesh/utils.py:35-131 as primitives; the draws follow the reference's argument order.
def make_wall(size, pos, euler) -> Obstacle:
    """make_wall (trimesh/utils.py:35-54): box of extents (w, h, t), rotated 'rxyz'."""
    return Obstacle(OBST_BOX, np.asarray(pos, np.float64), np.asarray(euler, np.float64),
                    np.asarray(size, np.float64) / 2)


def make_orbit(pos, euler, orng: np.random.RandomState, oprng: random.Random) -> Obstacle:
    """make_orbit (trimesh/utils.py:56-83): box 20 % / cylinder 20 % / icosphere 20 % / capsule 40 %
    (the cone branch `0.8 <= prob < 0.8` is unreachable)."""
    prob = oprng.random()
    if prob < 0.2:
        kind, half = OBST_BOX, orng.uniform(0.1, 0.5, 3) / 2
    elif prob < 0.4:
        r, h = orng.uniform(0.1, 0.3), orng.uniform(0.2, 0.6)
        kind, half = OBST_CYLINDER, np.array([r, r, h / 2])
    elif prob < 0.6:
        r = orng.uniform(0.1, 0.3)
        kind, half = OBST_SPHERE, np.array([r, r, r])
    else:
        r, h = orng.uniform(0.1, 0.3), orng.uniform(0.2, 0.6)
        kind, half = OBST_CAPSULE, np.array([r, r, h / 2])  # trimesh capsule: height = centre-to-centre
    return Obstacle(kind, np.asarray(pos, np.float64), np.asarray(euler, np.float64), half)


def make_ground_high_obs(pos, orng: np.random.RandomState, oprng: random.Random) -> Obstacle:
    """make_ground_high_obs (trimesh/utils.py:85-104): standing box or cylinder of height 1-3 m on
    the ground, not rotated."""
    height = 1.0 + oprng.uniform(0.0, 2.0)
    pos = np.array(pos, np.float64)
    pos[2] = height / 2
    if oprng.random() < 0.5:
        sxy = orng.uniform(0.05, 1.0, 2)
        return Obstacle(OBST_BOX, pos, np.zeros(3), np.array([sxy[0] / 2, sxy[1] / 2, height / 2]))
    r = orng.uniform(0.025, 0.5)
    return Obstacle(OBST_CYLINDER, pos, np.zeros(3), np.array([r, r, height / 2]))


def make_ground_little_obj(pos, orng: np.random.RandomState, oprng: random.Random) -> Obstacle:
    """make_ground_little_obj (trimesh/utils.py:106-131): small box / cylinder / sphere near the
    ground, not rotated."""
    pos = np.array(pos, np.float64)
    prob = oprng.random()
    if prob < 0.33:
        size = orng.uniform(0.1, 1.5, 3)
        pos[2] = size[2] / 2 + oprng.uniform(-0.2, 0.5)
        return Obstacle(OBST_BOX, pos, np.zeros(3), size / 2)
    if prob < 0.66:
        r, h = oprng.uniform(0.025, 0.5), oprng.uniform(0.1, 1.0)
        pos[2] = h / 2 + oprng.uniform(-0.2, 0.5)
        return Obstacle(OBST_CYLINDER, pos, np.zeros(3), np.array([r, r, h / 2]))
    r = oprng.uniform(0.05, 0.5)
    pos[2] = oprng.uniform(-r, r) + oprng.uniform(-0.2, 0.5)
    return Obstacle(OBST_SPHERE, pos, np.zeros(3), np.array([r, r, r]))


def _seg_point(mid, vec, adj, rad, scale, rrange, orng):
    """mid + a shift along the segment (offset_1) + a shift along a random direction normal to it
    (offset_2), as every family's obstacle loop draws it."""
    off1 = vec / 2 * orng.uniform(-adj, adj)
    while True:
        r = orng.uniform(-rrange, rrange, 3)
        cr = np.cross(vec, r)
        if not np.allclose(cr, np.zeros(3)):
            break
    off2 = cr / np.linalg.norm(cr) * orng.uniform(-rad, rad) * scale
    return mid + off1 + off2


def segment_obstacles(cfg: FamilyCfg, d: float, pts: np.ndarray, segs, scale: float, rrange: float,
                      counts: tuple, little: tuple, little_adj, no_obs: bool,
                      orng: np.random.RandomState, oprng: random.Random) -> list:
    """Walls, orbits, ground-high obstacles and small ground objects along the gate segments
    `segs` (square :254-319, zigzag :510-610, ellipse :750-815 of trimesh/racing_terrains.py).
    counts = (walls, orbits, ground) per segment; little = randint range of small objects;
    no_obs: zigzag's rejection of points within no_obs_range of the segment's gates."""
    out = []
    if not cfg.add_obs:
        return out
    G = len(pts)
    adj = _lerp(cfg.adj_dir_shift_prop, d)
    rad = _lerp(cfg.radius_dir_shift_prop, d)
    n_wall, n_orbit, n_ground = counts

    def near(pt, i, j, xy=False):
        if not no_obs:
            return False
        k = 2 if xy else 3
        return (np.linalg.norm(pt[:k] - pts[i][:k]) < cfg.no_obs_range
                or np.linalg.norm(pt[:k] - pts[j][:k]) < cfg.no_obs_range)

    for i in segs:
        j = (i + 1) % G
        p0, p1 = pts[i], pts[j]  # fp32, as the reference's gate_pts: mid and the along-segment shift round there
        mid, vec = (p0 + p1) / 2, p1 - p0
        cnt = 0
        while cnt < n_wall:
            pt = _seg_point(mid, vec, adj, rad, scale, rrange, orng)
            pt[2] = oprng.uniform(0.5, 3.0)
            if near(pt, i, j):
                continue
            eul = orng.uniform(-180, 180, 3)
            ws = orng.uniform(cfg.wall_size[0], cfg.wall_size[1], 2)
            wt = orng.uniform(cfg.wall_thickness[0], cfg.wall_thickness[1])
            out.append(make_wall((ws[0], ws[1], wt), pt, eul))
            cnt += 1
        cnt = 0
        while cnt < n_orbit:
            pt = _seg_point(mid, vec, adj, rad, scale, rrange, orng)
            pt[2] = oprng.uniform(0.5, 3.0)
            if near(pt, i, j):
                continue
            out.append(make_orbit(pt, orng.uniform(-180, 180, 3), orng, oprng))
            cnt += 1
        if cfg.add_ground_obs:
            cnt = 0
            while cnt < n_ground:
                pt = _seg_point(mid, vec, adj, rad, scale, rrange, orng)
                if near(pt, i, j, xy=True):
                    continue
                orng.uniform(-180, 180, 3)  # the (unused) orientation draw
                out.append(make_ground_high_obs(pt, orng, oprng))
                cnt += 1
            for _ in range(oprng.randint(*little)):
                pt = _seg_point(mid, vec, little_adj if little_adj is not None else adj, rad, scale, rrange, orng)
                if near(pt, i, j, xy=True):
                    continue
                orng.uniform(-180, 180, 3)
                out.append(make_ground_little_obj(pt, orng, oprng))
    return out


def _counts(cfg: FamilyCfg, d: float, scale: float = 1.0):
    return (int(_lerp(cfg.num_wall_seg, d) * scale), int(_lerp(cfg.num_orbit_seg, d) * scale),
            int(_lerp(cfg.num_ground_obs, d) * scale))


def square_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random,
                 orng: np.random.RandomState, oprng: random.Random) -> Track:
    """SquareRacingTrackTerrain (trimesh/racing_terrains.py:167-336)."""
    radius = prng.uniform(cfg.radius[0], cfg.radius[1])
    G = cfg.num_gate
    gate_size = cfg.gate_size[1] - (cfg.gate_size[1] - cfg.gate_size[0]) * d
    gate_thickness = cfg.gate_thickness[0] + (cfg.gate_thickness[1] - cfg.gate_thickness[0]) * d
    pos_noise = _lerp(cfg.pos_noise_scale, d)
    rot_noise = _lerp(cfg.rot_noise_scale, d)
    theta = np.linspace(0, 2 * np.pi, G, endpoint=False)
    pts = np.zeros((G, 3), dtype=np.float32)  # fp32 stores in the reference's order (:190-197)
    pts[:, 0] = np.cos(theta) * radius
    pts[:, 1] = np.sin(theta) * radius
    pts[:, 2] = 1.0
    pts[:, 0] += size[0] / 2
    pts[:, 1] += size[1] / 2
    eul = np.zeros((G, 3), dtype=np.float32)
    eul[:, 0] = 90.0
    eul[:, 1] = theta / np.pi * 180.0
    pn = rng.uniform(-1, 1, (G, 3)) * pos_noise
    rn = rng.uniform(-1, 1, (G, 3)) * rot_noise
    if cfg.only_yaw:
        rn[:, 0] = 0.0
        rn[:, 2] = 0.0
    pts += pn
    pts[:, 2] = pts[:, 2].clip(0.8, 2.0)
    eul += rn
    w, h, t, e = _shape_noise(rng, G, gate_size, gate_thickness, cfg.edge)
    reverse = 1
    if prng.random() < 0.5:
        pts = pts[::-1].copy()
        eul = eul[::-1].copy()
        reverse = -1
    start_seg = prng.randint(0, G - 1)
    k = (start_seg + 1) % G
    ang = eul[k][1] / 180 * np.pi + np.pi / 2
    origin = pts[k] - reverse * prng.uniform(2, 4) * np.array([np.cos(ang), np.sin(ang), 0.0])
    origin[2] = prng.uniform(0.7, 1.5)
    # no obstacles on the start segment (:247-249); counts scale with radius / radius_max (:244-245, :297)
    obs = segment_obstacles(cfg, d, pts, [i for i in range(G) if i != start_seg], radius, 10.0,
                            _counts(cfg, d, radius / cfg.radius[1]), (1, 4), None, False, orng, oprng)
    return Track(pts, eul, w, h, t, e, origin.astype(np.float64), (start_seg + 1) % G, obs)


def zigzag_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random,
                 orng: np.random.RandomState, oprng: random.Random) -> Track:
    """ZigzagRacingTerrain (trimesh/racing_terrains.py:423-620)."""
    G = cfg.num_gate
    gate_size = cfg.gate_size[1] - (cfg.gate_size[1] - cfg.gate_size[0]) * d
    gate_thickness = cfg.gate_thickness[0] + (cfg.gate_thickness[1] - cfg.gate_thickness[0]) * d
    pos_noise = _lerp(cfg.pos_noise_scale, d)
    z_noise_scale = _lerp(cfg.pos_z_noise_scale, d)
    rot_noise = _lerp(cfg.rot_noise_scale, d)
    theta = rng.uniform(0, 2 * np.pi)
    direction = np.array([np.cos(theta), np.sin(theta), 0.0])
    start, end = -0.5 * cfg.track_length * direction, 0.5 * cfg.track_length * direction
    t_values = np.linspace(0, 1, G)
    points = start + np.outer(t_values, end - start)
    for i in range(1, G - 1):
        f = t_values[i]
        ndir = np.array([-direction[1], direction[0], 0.0])
        points[i] += 2.0 * (rng.rand() - 0.5) * pos_noise * f * ndir
        _ = 2.0 * (rng.rand() - 0.5)  # longitudinal draw: computed but never applied in the reference (:465-467)
        points[i] += 2.0 * (rng.rand() - 0.5) * z_noise_scale * f * np.array([0.0, 0.0, 1.0])
    eul = np.zeros((G, 3), dtype=np.float32)
    eul[:, 0] = 90.0
    eul[:, 1] = theta / np.pi * 180.0 + 90
    pts = points  # fp64 here: the reference rebinds gate_pts to these points (:470)
    pts[:, 0] += size[0] / 2
    pts[:, 1] += size[1] / 2
    pts[:, 2] += 1.0
    pts[:, 2] = pts[:, 2].clip(0.8, 2.0)
    rn = rng.uniform(-1, 1, (G, 3)) * rot_noise
    if cfg.only_yaw:
        rn[:, 0] = 0.0
        rn[:, 2] = 0.0
    eul += rn
    w, h, t, e = _shape_noise(rng, G, gate_size, gate_thickness, cfg.edge)
    fdir = pts[1] - pts[0]
    fdir = fdir / np.linalg.norm(fdir)
    origin = pts[0].astype(np.float64) - fdir * prng.uniform(2, 3)
    origin[2] = prng.uniform(0.7, 1.5)
    # between consecutive gates (no wrap-around), offsets scaled by the largest gate size, points
    # within no_obs_range of the segment's gates rejected (:517-610)
    obs = segment_obstacles(cfg, d, pts, range(G - 1), cfg.gate_size[1] / 2, 1.0, _counts(cfg, d), (1, 4), 0.5,
                            True, orng, oprng)
    return Track(pts, eul, w, h, t, e, origin, 0, obs)


def ellipse_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random,
                  orng: np.random.RandomState, oprng: random.Random) -> Track:
    """EllipseRacingTerrain (trimesh/racing_terrains.py:625-832).
    The reference hard-codes 8 gates; other gate counts (config C5: 32) place
    G gates on the same ellipse, facing along the tangent (our extension)."""
    G = cfg.num_gate
    a_coef = cfg.long_axis_prop[0] + d * (cfg.long_axis_prop[1] - cfg.long_axis_prop[0])
    b_coef = cfg.short_axis_prop[0] + d * (cfg.short_axis_prop[1] - cfg.short_axis_prop[0])
    a_e, b_e = a_coef * cfg.gate_distance, b_coef * cfg.gate_distance
    gate_size = cfg.gate_size[1] - (cfg.gate_size[1] - cfg.gate_size[0]) * d
    gate_thickness = cfg.gate_thickness[0] + (cfg.gate_thickness[1] - cfg.gate_thickness[0]) * d
    pos_noise = _lerp(cfg.pos_noise_scale, d)
    rot_noise = _lerp(cfg.rot_noise_scale, d)
    eul = np.zeros((G, 3), dtype=np.float32)
    eul[:, 0] = 90.0
    theta = rng.uniform(0, 2 * np.pi)
    te = theta / np.pi * 180.0
    L = np.array([np.cos(theta), np.sin(theta), 0.0])
    S = np.array([-np.sin(theta), np.cos(theta), 0.0])
    pts = np.zeros((G, 3), dtype=np.float32 if G == 8 else np.float64)  # fp32 like the reference's points (:673)
    if G == 8:
        pts[0], pts[4] = -0.5 * a_e * L, 0.5 * a_e * L
        pts[2], pts[6] = 0.5 * b_e * S, -0.5 * b_e * S
        pts[1] = pts[2] - cfg.gate_distance * L
        pts[3] = pts[2] + cfg.gate_distance * L
        pts[5] = pts[6] + cfg.gate_distance * L
        pts[7] = pts[6] - cfg.gate_distance * L
        eul[0, 1], eul[4, 1] = te, 180 + te
        eul[2, 1], eul[6, 1] = te + 90, te + 270
        eul[1, 1] = eul[3, 1] = te + 90
        eul[5, 1] = eul[7, 1] = te + 270
    else:
        phi = np.linspace(np.pi, 3 * np.pi, G, endpoint=False)  # start at -a/2 on the long axis like gate 0
        for i, f in enumerate(phi):
            pts[i] = 0.5 * a_e * np.cos(f) * L - 0.5 * b_e * np.sin(f) * S
            tangent = -0.5 * a_e * np.sin(f) * L - 0.5 * b_e * np.cos(f) * S
            eul[i, 1] = math.degrees(math.atan2(tangent[1], tangent[0])) - 90.0
    pts = pts.astype(np.float32)
    pts[:, 0] += size[0] / 2
    pts[:, 1] += size[1] / 2
    pts[:, 2] += 1.0
    pn = rng.uniform(-1, 1, (G, 3)) * pos_noise
    rn = rng.uniform(-1, 1, (G, 3)) * rot_noise
    if cfg.only_yaw:
        rn[:, 0] = 0.0
        rn[:, 2] = 0.0
    pts += pn
    pts[:, 2] = pts[:, 2].clip(0.8, 2.0)
    eul += rn
    w, h, t, e = _shape_noise(rng, G, gate_size, gate_thickness, cfg.edge)
    if prng.random() < 0.5:
        pts = pts[::-1].copy()
        eul = eul[::-1].copy()
    start_seg = prng.randint(0, G - 1)
    nxt = (start_seg + 1) % G
    seg = pts[nxt] - pts[start_seg]
    seg = seg / np.linalg.norm(seg)
    origin = pts[start_seg] + seg * prng.uniform(2, 3)  # fp32, as the reference's (:746)
    origin[2] = prng.uniform(0.7, 1.5)
    # all segments but the start one, offsets scaled by gate_distance (:750-815)
    obs = segment_obstacles(cfg, d, pts, [i for i in range(G) if i != start_seg], cfg.gate_distance, 10.0,
                            _counts(cfg, d), (1, 2), None, False, orng, oprng)
    return Track(pts, eul, w, h, t, e, origin, nxt, obs)


GENERATORS = {"zigzag": zigzag_track, "circular": square_track, "ellipse": ellipse_track}


def euler_matrix_rxyz(deg: np.ndarray) -> np.ndarray:
    """trimesh.transformations.euler_matrix(ai, aj, ak, 'rxyz') rotation part = Rx(ai) Ry(aj) Rz(ak)."""
    a, b, c = np.radians(deg.astype(np.float64))
    ca, sa, cb, sb, cc, sc = np.cos(a), np.sin(a), np.cos(b), np.sin(b), np.cos(c), np.sin(c)
    Rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    Ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    Rz = np.array([[cc, -sc, 0], [sc, cc, 0], [0, 0, 1]])
    return Rx @ Ry @ Rz


def column_families(cfg: TrackGenCfg) -> list[int]:
    """IL TerrainGenerator._generate_curriculum_terrains: family of each column by proportion."""
    props = np.array([f.proportion for f in cfg.families], dtype=np.float64)
    props /= props.sum()
    cs = np.cumsum(props)
    return [int(np.min(np.where(c / cfg.num_cols + 0.001 < cs)[0])) for c in range(cfg.num_cols)]


def generate_tracks(cfg: TrackGenCfg) -> list[list[Track]]:
    """tracks[col][row]"""
    np_rng = np.random.RandomState(cfg.seed)       # IL's difficulty stream
    rng = np.random.RandomState(cfg.seed + 1)      # the generators' np.random stream
    prng = random.Random(cfg.seed + 2)             # the generators' `random` stream
    orng = np.random.RandomState(cfg.seed + 3)     # obstacle streams (np.random / random of the reference)
    oprng = random.Random(cfg.seed + 4)
    fams = column_families(cfg)
    out = []
    for col in range(cfg.num_cols):
        f = cfg.families[fams[col]]
        colv = []
        for row in range(cfg.num_rows):
            lo, hi = cfg.difficulty_range
            d = lo + (hi - lo) * (row + np_rng.uniform()) / cfg.num_rows
            colv.append(GENERATORS[f.kind](d, f, cfg.size, rng, prng, orng, oprng))
        out.append(colv)
    return out


def pack_tracks(tracks: list[list[Track]], max_gates: int, lattice_reach: float):
    """-> (gates [T*L][max_gates][20] f32, records [T*L][4] f32) in the GR_GATE_FLOATS layout:
       0-2 centre (env-local), 3 cull radius^2, 4-6 / 8-10 / 12-14 rows of R^T,
       7 inner half-width, 11 inner half-height, 15 half-thickness, 16-17 outer half w/h, 18 edge."""
    T, L = len(tracks), len(tracks[0])
    gates = np.zeros((T * L, max_gates, GATE_FLOATS), dtype=np.float32)
    recs = np.zeros((T * L, TRACK_FLOATS), dtype=np.float32)
    for t in range(T):
        for lv in range(L):
            tr = tracks[t][lv]
            k = t * L + lv
            G = len(tr.gate_pts)
            if G > max_gates:
                raise ValueError(f"track ({t},{lv}) has {G} gates > max_gates {max_gates}")
            for g in range(G):
                c = tr.gate_pts[g].astype(np.float64) - tr.origin
                R = euler_matrix_rxyz(tr.gate_euler[g])
                hw, hh, ht, e = tr.gate_w[g] / 2, tr.gate_h[g] / 2, tr.gate_t[g] / 2, tr.gate_e[g]
                how, hoh = hw + e, hh + e
                bound = (math.sqrt(how * how + hoh * hoh + ht * ht) + lattice_reach) * 1.01 + 1e-3
                rec = gates[k, g]
                rec[0:3] = c
                rec[3] = bound * bound
                M = R.T
                rec[4:7], rec[7] = M[0], hw
                rec[8:11], rec[11] = M[1], hh
                rec[12:15], rec[15] = M[2], ht
                rec[16], rec[17], rec[18] = how, hoh, e
            recs[k] = (-tr.origin[2], tr.origin[2], tr.next_gate_id, G)
    return gates, recs


def obstacle_radius(o: Obstacle) -> float:
    """bounding radius of a primitive about its centre"""
    h = o.half
    if o.kind == OBST_BOX:
        return float(np.linalg.norm(h))
    if o.kind == OBST_CYLINDER:
        return float(math.hypot(h[0], h[2]))
    if o.kind == OBST_SPHERE:
        return float(h[0])
    return float(h[0] + h[2])  # capsule


@dataclass
class ObstacleTable:
    """Device layout of the obstacles (include/gr.h gr_obstacles):
    records [T*L][max_obstacles][OBST_FLOATS]: 0-2 centre (env-local), 3 cull radius^2 (bound +
    lattice reach), 4-6 / 8-10 / 12-14 rows of R^T, 7 / 11 / 15 half sizes (box) | r, r, half height
    (cylinder) | r (sphere) | r, r, half segment (capsule), 16 kind, 17 bounding radius;
    counts [T*L]; per track a uniform xy grid (grid_f: x0, y0, 1/cell, margin/cell; grid_i: nx, ny,
    first cell, 0) whose cells [C][2] (first item, count) list copies of the records (items [I][20])
    whose cull sphere reaches into the cell's rectangle grown by `margin` on every side.  So a drone
    that moved at most `margin` (per axis) out of a cell still finds every obstacle it can touch in
    that cell's list: the step kernel fetches the list of the pre-step cell while it integrates."""

    records: np.ndarray
    counts: np.ndarray
    grid_f: np.ndarray
    grid_i: np.ndarray
    cells: np.ndarray
    items: np.ndarray

    @property
    def max_obstacles(self) -> int:
        return int(self.records.shape[1])


def pack_obstacles(tracks: list[list[Track]], lattice_reach: float, cell: float = 2.0,
                   margin: float = 0.5) -> ObstacleTable:
    T, L = len(tracks), len(tracks[0])
    M = max(1, max(len(tr.obstacles) for col in tracks for tr in col))
    records = np.zeros((T * L, M, OBST_FLOATS), dtype=np.float32)
    counts = np.zeros(T * L, dtype=np.int32)
    grid_f = np.zeros((T * L, 4), dtype=np.float32)
    grid_i = np.zeros((T * L, 4), dtype=np.int32)
    cells, items = [], []
    for t in range(T):
        for lv in range(L):
            tr = tracks[t][lv]
            k = t * L + lv
            n = len(tr.obstacles)
            counts[k] = n
            for j, o in enumerate(tr.obstacles):
                rec = records[k, j]
                rec[0:3] = o.pos - tr.origin
                R = obstacle_radius(o)
                bound = (R + lattice_reach) * 1.01 + 1e-3
                rec[3] = bound * bound
                M_ = euler_matrix_rxyz(o.euler).T
                rec[4:7], rec[7] = M_[0], o.half[0]
                rec[8:11], rec[11] = M_[1], o.half[1]
                rec[12:15], rec[15] = M_[2], o.half[2]
                rec[16], rec[17] = float(o.kind), R
            if n == 0:
                grid_f[k] = (0.0, 0.0, 1.0 / cell, margin / cell)
                grid_i[k] = (0, 0, len(cells), 0)
                continue
            c = records[k, :n, 0:2].astype(np.float64)
            rc = np.sqrt(records[k, :n, 3].astype(np.float64)) + 0.01  # + fp32 rounding slack
            grow = margin + 0.01
            x0 = math.floor(float((c[:, 0] - rc).min()) / cell) * cell
            y0 = math.floor(float((c[:, 1] - rc).min()) / cell) * cell
            nx = max(1, math.ceil((float((c[:, 0] + rc).max()) - x0) / cell))
            ny = max(1, math.ceil((float((c[:, 1] + rc).max()) - y0) / cell))
            grid_f[k] = (x0, y0, 1.0 / cell, margin / cell)
            grid_i[k] = (nx, ny, len(cells), 0)
            for iy in range(ny):
                for ix in range(nx):
                    lo = np.array([x0 + ix * cell, y0 + iy * cell]) - grow
                    q = np.clip(c, lo, lo + cell + 2 * grow)  # closest point of the grown cell to each centre
                    hit = np.nonzero(np.sum((q - c) ** 2, axis=1) <= rc * rc)[0]
                    cells.append((len(items), len(hit)))
                    items.extend(records[k, j] for j in hit)
    cells_a = np.array(cells, dtype=np.int32).reshape(-1, 2) if cells else np.zeros((1, 2), np.int32)
    items_a = np.array(items, dtype=np.float32).reshape(-1, OBST_FLOATS) if items else np.zeros((1, OBST_FLOATS),
                                                                                               np.float32)
    return ObstacleTable(records, counts, grid_f, grid_i, cells_a, items_a)


def build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42, lattice_reach=0.1, obstacles=True,
                 cell=2.0, margin=0.5):
    """-> (gates, records, ObstacleTable or None)"""
    cfg = TrackGenCfg(seed=seed, num_rows=num_levels, num_cols=num_types).with_gates(num_gates)
    cfg.with_obstacles(obstacles)
    tracks = generate_tracks(cfg)
    gates, recs = pack_tracks(tracks, num_gates, lattice_reach)
    return gates, recs, (pack_obstacles(tracks, lattice_reach, cell, margin) if obstacles else None)


def build_track_table(num_types=20, num_levels=10, num_gates=8, seed=42, lattice_reach=0.1):
    """gates and track records only (obstacle-free tables)"""
    cfg = TrackGenCfg(seed=seed, num_rows=num_levels, num_cols=num_types).with_gates(num_gates).with_obstacles(False)
    return pack_tracks(generate_tracks(cfg), num_gates, lattice_reach)
