"""Diagnostic (GPU box): wall time of each part of the regenerating step (RacingEnv._regenerate_in_step)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs import racing_env as re_mod  # noqa: E402

n = 65536
env = re_mod.RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cuda:0"), stage=1,
                                    terrain=TerrainCfg(num_gates=8, obstacles=True, regen_interval_s=0.03 * 64)))
env.reset()
a = torch.randn(n, 4, device="cuda:0")
for k in range(63):
    env.step(a)
while not env._next_terrain.done():
    time.sleep(0.01)
torch.cuda.synchronize()


def timed(name, f, *args):
    t0 = time.perf_counter()
    r = f(*args)
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) * 1e6:.0f} us", flush=True)
    return r


orig_reset, orig_obs, orig_regen = env.reset, env.observe, env.regenerate_terrain
env.reset = lambda *a, **k: timed("reset", orig_reset, *a, **k)
env.observe = lambda *a, **k: timed("observe", orig_obs, *a, **k)
env.regenerate_terrain = lambda: timed("regenerate_terrain (incl. reset)", orig_regen)
timed("whole regenerating step", env.step, a)
for k in range(3):
    timed("plain step", env.step, a)
env._next_terrain = None
timed("regenerate_terrain again (build inline)", orig_regen)
timed("reset alone", orig_reset)
timed("reset alone", orig_reset)
