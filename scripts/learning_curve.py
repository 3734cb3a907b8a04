"""Summarise a training run's scalars (the runner's CSV logger: `step,key,value` lines) into a learning-curve
record: per key, the mean over windows of iterations, plus the first / last window.

    python scripts/learning_curve.py gpurun_out/lc profiles/round02_learning_curve.json [--window 100]
"""
import argparse
import collections
import glob
import json
import os

KEYS = ("Train/mean_reward", "Train/mean_episode_length", "Episode_Termination/time_out", "Episode_Termination/contact",
        "Episode_Termination/bad_pose", "Metrics/gates_passed", "Curriculum/terrain_levels", "Loss/value_function",
        "Loss/surrogate", "Policy/mean_noise_std", "Perf/total_fps")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log_root")
    ap.add_argument("out")
    ap.add_argument("--window", type=int, default=100)
    a = ap.parse_args()
    paths = sorted(glob.glob(os.path.join(a.log_root, "**", "scalars.csv"), recursive=True))
    if not paths:
        raise SystemExit(f"no scalars.csv under {a.log_root}")
    rows = collections.defaultdict(dict)
    for line in open(paths[-1]):
        step, key, value = line.rstrip("\n").split(",", 2)
        rows[key][int(step)] = float(value)
    keys = [k for k in KEYS if k in rows] + sorted(k for k in rows if k.startswith(("Episode_Reward/", "Metrics/"))
                                                    and k not in KEYS)
    last = max(max(v) for v in rows.values())
    curve = {}
    for k in keys:
        series = rows[k]
        wins = []
        for w0 in range(0, last + 1, a.window):
            vals = [v for s, v in series.items() if w0 <= s < w0 + a.window and v == v]  # skip NaN (no resets)
            wins.append(sum(vals) / len(vals) if vals else None)
        curve[k] = wins
    out = {"source": os.path.relpath(paths[-1]), "iterations": last + 1, "window": a.window,
           "windows": [f"{w0}-{min(w0 + a.window, last + 1) - 1}" for w0 in range(0, last + 1, a.window)],
           "curve": curve}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    for k in keys[:8]:
        w = curve[k]
        first = next((x for x in w if x is not None), None)
        final = next((x for x in reversed(w) if x is not None), None)
        print(f"{k:40s} {first!s:>24} -> {final!s:>24}")


if __name__ == "__main__":
    main()
