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
origin, and the start gate.  Mesh building / PhysX import and the
wall/orbit/ground obstacles are out of scope this round.
Exact layouts are not reproducible (the reference draws from Python's and
NumPy's global RNGs inside Isaac Lab's generator): same families, same
parameter ranges, our own seeded stream.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass, field

import numpy as np

from .._abi import GATE_FLOATS, TRACK_FLOATS


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


@dataclass
class TrackGenCfg:
    """RacingComplexTerrainCfg (racing_terrains.py:137-210)."""

    seed: int = 42
    size: tuple = (40.0, 40.0)
    num_rows: int = 10
    num_cols: int = 20
    difficulty_range: tuple = (0.0, 1.0)
    families: list = field(default_factory=lambda: [
        FamilyCfg("zigzag", 0.3, pos_noise_scale=(1.0, 4.0), pos_z_noise_scale=(0.1, 1.0)),
        FamilyCfg("circular", 0.3, radius=(5.0, 8.0)),
        FamilyCfg("ellipse", 0.4, edge=(0.15, 0.22)),
    ])

    def with_gates(self, n: int) -> "TrackGenCfg":
        for f in self.families:
            f.num_gate = n
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


def _shape_noise(rng, n, gate_size, gate_thickness, edge):
    w = gate_size + rng.uniform(-0.05, 0.05, n)
    h = gate_size + rng.uniform(-0.05, 0.05, n)
    t = gate_thickness + rng.uniform(-1, 1, n) / 5 * gate_thickness
    e = rng.uniform(edge[0], edge[1], n)
    return w, h, t, e


def _lerp(rng_pair, d):
    return d * (rng_pair[1] - rng_pair[0]) + rng_pair[0]


def square_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random) -> Track:
    """SquareRacingTrackTerrain (trimesh/racing_terrains.py:167-336), gates + origin only."""
    radius = prng.uniform(cfg.radius[0], cfg.radius[1])
    G = cfg.num_gate
    gate_size = cfg.gate_size[1] - (cfg.gate_size[1] - cfg.gate_size[0]) * d
    gate_thickness = cfg.gate_thickness[0] + (cfg.gate_thickness[1] - cfg.gate_thickness[0]) * d
    pos_noise = _lerp(cfg.pos_noise_scale, d)
    rot_noise = _lerp(cfg.rot_noise_scale, d)
    theta = np.linspace(0, 2 * np.pi, G, endpoint=False)
    pts = np.zeros((G, 3), dtype=np.float32)
    pts[:, 0] = np.cos(theta) * radius + size[0] / 2
    pts[:, 1] = np.sin(theta) * radius + size[1] / 2
    pts[:, 2] = 1.0
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
    return Track(pts, eul, w, h, t, e, origin.astype(np.float64), (start_seg + 1) % G)


def zigzag_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random) -> Track:
    """ZigzagRacingTerrain (trimesh/racing_terrains.py:423-620), gates + origin only."""
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
    pts = points.astype(np.float32)
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
    return Track(pts, eul, w, h, t, e, origin, 0)


def ellipse_track(d: float, cfg: FamilyCfg, size, rng: np.random.RandomState, prng: random.Random) -> Track:
    """EllipseRacingTerrain (trimesh/racing_terrains.py:625-832), gates + origin only.
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
    pts = np.zeros((G, 3))
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
    origin = pts[start_seg].astype(np.float64) + seg * prng.uniform(2, 3)
    origin[2] = prng.uniform(0.7, 1.5)
    return Track(pts, eul, w, h, t, e, origin, nxt)


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
    fams = column_families(cfg)
    out = []
    for col in range(cfg.num_cols):
        f = cfg.families[fams[col]]
        colv = []
        for row in range(cfg.num_rows):
            lo, hi = cfg.difficulty_range
            d = lo + (hi - lo) * (row + np_rng.uniform()) / cfg.num_rows
            colv.append(GENERATORS[f.kind](d, f, cfg.size, rng, prng))
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


def build_track_table(num_types=20, num_levels=10, num_gates=8, seed=42, lattice_reach=0.1):
    cfg = TrackGenCfg(seed=seed, num_rows=num_levels, num_cols=num_types).with_gates(num_gates)
    return pack_tracks(generate_tracks(cfg), num_gates, lattice_reach)
