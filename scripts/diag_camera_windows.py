"""Diagnostic (CPU, oracle): how much per-pixel obstacle work does a re-render of the depth camera carry?

For envs at their post-reset pose (oracle), restates gr_cam_frame_setup's screen window per obstacle (numpy fp32,
statistics only) and reports, per env: obstacles in view, (8x32 tile, slot) pairs the kernel's tile masks select,
and the pixels of those pairs that lie inside the slot's window (the per-pixel test the kernel and oracle apply).

    python scripts/diag_camera_windows.py [--envs 512]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg  # noqa: E402
from generalizableracing_amd.envs.tracks import build_tracks  # noqa: E402


frames = []


def outside_tile(fr, a_lo, a_hi, b_lo, b_hi):
    """The box lies wholly outside one of the tile frustum's four side planes (y = a x, z = b x)."""
    c, ax, l = fr
    for nrm in ((-a_hi, 1.0, 0.0), (a_lo, -1.0, 0.0), (-b_hi, 0.0, 1.0), (b_lo, 0.0, -1.0)):
        nrm = np.array(nrm)
        if c @ nrm - (l * np.abs(ax @ nrm)).sum() > 0:
            return True
    return False


def windows(recs, o, c0, c1, c2, maxd=10.0):
    """[n, 5]: valid, amin, amax, bmin, bmax (gr_cam_frame_setup, gr_obst_local_box)."""
    out = np.zeros((len(recs), 5), np.float32)
    frames.clear()
    for k, r in enumerate(recs):
        kind = int(r[16])
        l = np.array([r[7], r[11], r[15] + (r[7] if kind == 3 else 0.0)], np.float32)
        rel = r[0:3] - o
        M = np.stack([r[4:7], r[8:11], r[12:15]])
        D0, D1, D2 = M @ c0, M @ c1, M @ c2
        x0, y0, z0 = c0 @ rel, c1 @ rel, c2 @ rel
        ex = np.abs(l * D0).sum()
        valid = (x0 + ex > 0) and (x0 - ex <= maxd)
        amin, amax, bmin, bmax = -3e38, 3e38, -3e38, 3e38
        if x0 - ex > 1e-3:
            pts = []
            for c in range(8):
                s = np.array([l[0] if c & 1 else -l[0], l[1] if c & 2 else -l[1], l[2] if c & 4 else -l[2]])
                pts.append((x0 + s @ D0, y0 + s @ D1, z0 + s @ D2))
            pts = np.array(pts)
            a, b = pts[:, 1] / pts[:, 0], pts[:, 2] / pts[:, 0]
            amin, amax, bmin, bmax = a.min(), a.max(), b.min(), b.max()
        out[k] = (valid, amin, amax, bmin, bmax)
        frames.append((np.array([x0, y0, z0]), np.stack([D0, D1, D2], 1), l))  # centre, axes (rows j), half sizes
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=256)
    a = ap.parse_args()
    n = a.envs
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=1)
    gates, recs, ot = build_tracks(num_types=20, num_levels=10, num_gates=8, seed=42)
    orc = oracle.Oracle(cfg.to_gr_config(), gates, recs, ot.records, ot.counts)
    orc.init()
    cam = CameraCfg()
    orc.enable_camera(cam.to_gr())
    orc.reset(None)
    W, H = cam.width, cam.height
    stats = []
    for i in range(n):
        e = orc.envs[i]
        track = int(e["type"]) * 10 + int(e["level"])
        o, c0, c1, c2, ra, rb = orc.camera_frame(e["p"], e["q"])
        wins = windows(ot.records[track, :ot.counts[track]], o, c0, c1, c2)
        frs = [f for f, w in zip(frames, wins) if w[0] > 0]
        wins = wins[wins[:, 0] > 0]
        pairs = pix = full = culled = culled_pix = 0
        for v0 in range(0, H, 8):
            for u0 in range(0, W, 32):
                a_t, b_t = ra[u0:u0 + 32], rb[v0:v0 + 8]
                for w, fr in zip(wins[:64], frs[:64]):
                    if w[2] < a_t.min() or w[1] > a_t.max() or w[4] < b_t.min() or w[3] > b_t.max():
                        continue
                    pairs += 1
                    cols = ((a_t >= w[1]) & (a_t <= w[2])).sum()
                    rows = ((b_t >= w[3]) & (b_t <= w[4])).sum()
                    pix += cols * rows
                    full += cols * rows == 256
                    if outside_tile(fr, a_t.min(), a_t.max(), b_t.min(), b_t.max()):
                        culled += 1
                        culled_pix += cols * rows
        stats.append((len(wins), pairs, pix, full, culled, culled_pix))
    s = np.array(stats, np.float64)
    print(f"{n} envs at their post-reset pose, obstacle tracks")
    print(f"  obstacles in view per env: mean {s[:, 0].mean():.1f}, max {s[:, 0].max():.0f}")
    print(f"  in view: p90 {np.percentile(s[:, 0], 90):.0f}, p99 {np.percentile(s[:, 0], 99):.0f}; envs over 48 / 56 / 64: "
          f"{(s[:, 0] > 48).mean():.4f} / {(s[:, 0] > 56).mean():.4f} / {(s[:, 0] > 64).mean():.4f}")
    print(f"  (tile, slot) pairs per env: mean {s[:, 1].mean():.1f} (27 tiles)")
    print(f"  window pixels of those pairs per env: mean {s[:, 2].mean():.0f} (image 6912); "
          f"per pair {s[:, 2].sum() / max(s[:, 1].sum(), 1):.0f} of 256; whole-tile pairs {s[:, 3].sum() / max(s[:, 1].sum(), 1):.2f}")
    print(f"  pairs a box-vs-tile-frustum plane test culls: {s[:, 4].sum() / max(s[:, 1].sum(), 1):.2f} "
          f"(window pixels {s[:, 5].sum() / max(s[:, 2].sum(), 1):.2f})")
    print(f"  quad-path hit evaluations per env (4 per lane per pair, x64 lanes): {s[:, 1].mean() * 256:.0f}; "
          f"packed path: {np.ceil(s[:, 2] / 64).mean() * 64:.0f} lane-hits lower bound")


if __name__ == "__main__":
    main()
