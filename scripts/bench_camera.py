"""Depth-camera throughput on one MI355X: gr_camera_render after gr_step.

Times the camera kernel alone with HIP events on the stream it is launched on (torch's current
stream), separately for the calls that re-render every sensor (every 2nd step: update_period
0.04 s at step_dt 0.03 s) and the calls that reuse the depth buffer, and reports algorithmic
bytes per call (gr_camera_bytes_per_env) / time against the HBM peak.

Phases: "synchronized" (default) starts every sensor on the same call, as right after one global reset, so the
calls alternate between all-render and all-reuse.  "steady" spreads the sensors' ages uniformly over the update
period first, as a long training run leaves them (each env's phase is set by its own last reset, and episodes end at
different steps), so every call renders ~1/period of the envs and reuses the rest.

  python scripts/bench_camera.py --envs 65536 --steps 40
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from generalizableracing_amd import _abi  # noqa: E402
from generalizableracing_amd.envs.racing_cfg import CameraCfg, RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def run(n=65536, steps=40, warmup=6, no_noise=False, period=None, device="cuda:0", obstacles=True,
        phase="synchronized") -> dict:
    args = argparse.Namespace(envs=n, steps=steps, warmup=warmup, no_noise=no_noise, period=period)
    cam = CameraCfg(add_noise=not args.no_noise)
    if args.period is not None:
        cam.update_period = args.period
    env = RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=device), camera=cam,
                                 terrain=TerrainCfg(obstacles=obstacles)))
    env.reset()
    g = torch.Generator(device=device).manual_seed(1234)
    acts = [torch.randn(n, 4, device=device, generator=g) for _ in range(8)]
    rb, ub = C.c_int64(), C.c_int64()
    env._call("gr_camera_bytes_per_env", C.byref(rb), C.byref(ub))
    for k in range(args.warmup):
        env.step(acts[k % 8])
    if phase == "steady":
        k_period = 1  # gr_cam_period_steps: renders every k_period steps
        while k_period * env.cfg.step_dt + 1e-6 < env.cfg.camera.update_period:
            k_period += 1
        ages = torch.randint(0, k_period, (n,), generator=torch.Generator().manual_seed(7), dtype=torch.int32)
        env.camera_age.copy_(ages.to(device))
    elif phase != "synchronized":
        raise ValueError(f"phase {phase!r}")
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    rendered = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        env._advance()
        env._call("gr_step", acts[k % 8].data_ptr(), env._stream())
        ev[k][0].record()
        env._render(_abi.GR_CAM_STEP)
        ev[k][1].record()
        rendered.append(env.camera_age.eq(0).float().mean())  # age 0: rendered by this call
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = [a.elapsed_time(b) for a, b in ev]
    frac = [float(r) for r in rendered]
    rend = [m for m, f in zip(ms, frac) if f > 0.5]
    reuse = [m for m, f in zip(ms, frac) if f <= 0.5]
    avg = lambda xs: sum(xs) / max(len(xs), 1)  # noqa: E731
    mean_frac = sum(frac) / len(frac)
    bytes_call = n * (mean_frac * rb.value + (1 - mean_frac) * ub.value)
    out = {
        "kernel": "gr::camera_kernel",
        "noise": not args.no_noise, "phase": phase,
        "envs": n, "steps": args.steps,
        "image": [env.camera.height, env.camera.width],
        "render_fraction": mean_frac,
        "ms_render_call": avg(rend), "ms_reuse_call": avg(reuse), "ms_avg_call": avg(ms),
        "bytes_per_env_render": rb.value, "bytes_per_env_reuse": ub.value,
        "gbs_render_call": n * rb.value / (avg(rend) * 1e6) if rend else None,
        "gbs_reuse_call": n * ub.value / (avg(reuse) * 1e6) if reuse else None,
        "gbs_avg": bytes_call / (avg(ms) * 1e6),
        "hbm_frac_avg": bytes_call / (avg(ms) * 1e6) / HBM_PEAK_GBS,
        "camera_env_steps_per_s": n / (avg(ms) * 1e-3),
        "wall_env_steps_per_s_step_plus_camera": n * args.steps / wall,
    }
    env.close()
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--no-noise", action="store_true", help="ablation: policy image without noise")
    ap.add_argument("--period", type=float, default=None, help="camera update_period override (0: every step)")
    ap.add_argument("--gates-only", action="store_true", help="obstacle-free tracks")
    ap.add_argument("--phase", choices=["synchronized", "steady"], default="synchronized")
    a = ap.parse_args(argv)
    print(json.dumps(run(a.envs, a.steps, a.warmup, a.no_noise, a.period, obstacles=not a.gates_only,
                         phase=a.phase)))


if __name__ == "__main__":
    main()
