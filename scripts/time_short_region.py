"""How much of a short timed region (the driver's K = 20) is launch / completion latency: the same 20-step graph
replay timed with torch.cuda.synchronize() alone, and with a spin on an event query before it (the GPU work is
the same; only the host's wake-up differs).  Prints one JSON line.

    python scripts/time_short_region.py [--steps 20] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    n = 65536
    env = bench.make_env(n, 0, "cuda:0", 8, "dd_explicit", False)
    g = torch.Generator(device="cuda:0").manual_seed(1234)
    actions = torch.randn(bench.ACTION_RING, n, 4, device="cuda:0", generator=g)
    graph = bench.capture_graph(env, actions, a.steps)
    ev = torch.cuda.Event()
    modes = ["sync", "spin_then_sync", "eager_env", "eager_raw"]
    res = {m: [] for m in modes}
    stream = env._stream()
    ptrs = [actions[k].data_ptr() for k in range(bench.ACTION_RING)]
    lib, ctx = env._lib, env._ctx
    for r in range(len(modes) * a.reps):
        mode = modes[r % len(modes)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode in ("sync", "spin_then_sync"):
            graph.replay()
        elif mode == "eager_env":
            for k in range(a.steps):
                env.step(actions[k % bench.ACTION_RING])
        else:  # the binding rotation and the launch only (what a C-level launcher would do)
            for k in range(a.steps):
                env._advance()
                lib.gr_step(ctx, ptrs[k % bench.ACTION_RING], stream)
        if mode == "spin_then_sync":
            ev.record()
            while not ev.query():
                pass
        torch.cuda.synchronize()
        res[mode].append((time.perf_counter() - t0) * 1e6 / a.steps)
    # GPU-side duration of the same replay (events on the stream around it) vs the wall clock
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    gpu = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        e0.record()
        graph.replay()
        e1.record()
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1) * 1e3 / a.steps)
    res["gpu_events_per_step"] = gpu
    out = {k: {"median_us_per_step": float(np.median(v)), "min": float(np.min(v))} for k, v in res.items()}
    out["steps"] = a.steps
    print(json.dumps(out))


if __name__ == "__main__":
    main()
