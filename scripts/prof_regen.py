"""Where the terrain-regenerating step's wall time goes (obstacle tracks, mdp/events.py:180-204 semantics): every
C-ABI call and the Python pieces of RacingEnv._regenerate_in_step timed with a device synchronisation after each,
against a plain eager step and a step followed by a full reset + observation pass (what the reference's
reset_terrain_period adds besides the new terrain).

    python scripts/prof_regen.py [--envs 65536] [--out gpurun_out/regen.json]
"""
import argparse
import collections
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--interval", type=int, default=256)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = "cuda:0"
    n = a.envs
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=dev), stage=1,
                       terrain=TerrainCfg(num_gates=8, obstacles=True, regen_interval_s=0.03 * a.interval))
    env = RacingEnv(cfg)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(5)
    acts = torch.randn(8, n, 4, device=dev, generator=g)
    for k in range(a.interval - 1 - 15 - 16):  # (then 15 timed plain steps, 16 warm-up steps: phase R - 1)
        env.step(acts[k % 8])
    while env._next_terrain is not None and not env._next_terrain.done():
        time.sleep(0.01)
    torch.cuda.synchronize()

    def wall(fn, reps=16):
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    res = {"envs": n}
    res["plain_step_us"] = wall(lambda: env.step(acts[1]), reps=15)

    # instrument: every C call and the Python pieces, synchronised
    timing = collections.defaultdict(float)
    counts = collections.Counter()
    call0 = env._call

    def timed_call(name, *args):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        r = call0(name, *args)
        t1 = time.perf_counter()
        e1.record()
        torch.cuda.synchronize()
        timing["c:" + name] += time.perf_counter() - t0
        timing["c_host:" + name] += t1 - t0
        timing["c_stream:" + name] += e0.elapsed_time(e1) * 1e-3
        counts["c:" + name] += 1
        return r

    def wrap(obj, attr):
        f = getattr(obj, attr)

        def w(*args, **kw):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f(*args, **kw)
            torch.cuda.synchronize()
            timing["py:" + attr] += time.perf_counter() - t0
            counts["py:" + attr] += 1
            return r
        setattr(obj, attr, w)

    res["full_reset_before_swap_us"] = wall(lambda: env.reset(), reps=4)
    while env.common_step_counter % env._regen_steps != env._regen_steps - 17:
        env.step(acts[3])
    while env._next_terrain is not None and not env._next_terrain.done():
        time.sleep(0.01)
    torch.cuda.synchronize()
    for _ in range(16):  # (the GPU idled while the host waited: warm it up again)
        env.step(acts[3])
    torch.cuda.synchronize()
    from generalizableracing_amd.envs import racing_env as _re
    _re.REGEN_STAMPS = []
    # an uninstrumented interval step first, with stamps inside regenerate_terrain only (host time between them)
    t0 = time.perf_counter()
    env.step(acts[0])
    torch.cuda.synchronize()
    res["regenerating_step_stamped_us"] = (time.perf_counter() - t0) * 1e6
    st = _re.REGEN_STAMPS
    res["regenerate_terrain_host_us"] = {f"{a}->{b}": (tb - ta) * 1e6 for (a, ta), (b, tb) in zip(st, st[1:])}
    _re.REGEN_STAMPS = None
    while env.common_step_counter % env._regen_steps != env._regen_steps - 17:
        env.step(acts[3])
    while env._next_terrain is not None and not env._next_terrain.done():
        time.sleep(0.01)
    torch.cuda.synchronize()
    for _ in range(16):
        env.step(acts[3])
    torch.cuda.synchronize()
    env._call = timed_call
    for attr in ("_regenerate_in_step", "regenerate_terrain", "reset", "observe", "_advance"):
        wrap(env, attr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, _, _, extras = env.step(acts[0])
    torch.cuda.synchronize()
    res["regenerating_step_instrumented_us"] = (time.perf_counter() - t0) * 1e6
    assert extras.get("terrain_regenerated")
    res["pieces_us"] = {k: v * 1e6 for k, v in sorted(timing.items(), key=lambda kv: -kv[1])}
    res["counts"] = dict(counts)
    env._call = call0
    for attr in ("_regenerate_in_step", "regenerate_terrain", "reset", "observe", "_advance"):
        delattr(env, attr)

    def step_reset_observe():
        env.step(acts[2])
        env.reset()
        env.observe()
    res["step_plus_full_reset_and_observe_us"] = wall(step_reset_observe, reps=8)
    # a second interval: the regenerating step again, uninstrumented (the first one may carry one-time costs)
    while env.common_step_counter % env._regen_steps != env._regen_steps - 17:
        env.step(acts[4])
    while env._next_terrain is not None and not env._next_terrain.done():
        time.sleep(0.01)
    torch.cuda.synchronize()
    for _ in range(16):
        env.step(acts[4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, _, _, _, extras = env.step(acts[0])
    torch.cuda.synchronize()
    res["second_regenerating_step_us"] = (time.perf_counter() - t0) * 1e6
    assert extras.get("terrain_regenerated") and env.terrain_generation == 3
    res["plain_step_after_us"] = wall(lambda: env.step(acts[5]), reps=8)
    env.close()
    print(json.dumps(res, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
