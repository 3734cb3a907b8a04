"""Per-phase wave timelines of the fused step kernel (diagnostic build, -DGR_STAMPS).

  python scripts/stamps.py build     # here: build/stamps/libgr.so
  python scripts/stamps.py run       # GPU box: GR_LIB_PATH=build/stamps/libgr.so, prints a JSON summary

Stamps (lane 0 of each wave, s_memtime shader cycles): 0 entry, 1 obs noise done,
2 gate table staged (barrier), 3 controller+integrator, 4 collision, 5 reward/termination,
6 reset+gate advance, 7 obs+state stores issued, 8 log rows; 9/10 s_memrealtime (100 MHz)
at entry/exit; 11 XCC_ID<<32 | HW_ID; 12 loads issued (before the obs noise).
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "stamps")
CSRC = os.path.join(ROOT, "generalizableracing_amd", "csrc")
PHASES = ["obs_noise", "table_barrier", "ctrl_integrate", "collision", "reward_term", "reset_advance",
          "obs_store_issue", "log"]


def build():
    os.makedirs(OUT, exist_ok=True)
    cmd = (f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "
           f"-fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -DGR_STAMPS -shared -o {OUT}/libgr.so "
           f"{CSRC}/gr_kernels.hip -x hip {CSRC}/gr_capi.cpp")
    subprocess.run(cmd, shell=True, check=True)


def run(n=65536, steps=200):
    os.environ["GR_LIB_PATH"] = os.path.join(OUT, "libgr.so")
    import ctypes as C

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    import bench

    env = bench.make_env(n, 0, "cuda:0", 8, "dd_explicit")
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = torch.randn(bench.ACTION_RING, n, 4, device="cuda:0", generator=g)
    res = []
    for rep in range(3):
        for k in range(steps):
            env.step(acts[k % bench.ACTION_RING])
        torch.cuda.synchronize()
        waves = n // 64
        buf = np.zeros(waves * 16, np.uint64)
        assert env._lib.gr_debug_read_stamps(buf.ctypes.data_as(C.c_void_p), buf.size) == 0
        st = buf.reshape(waves, 16).astype(np.int64)
        cyc = st[:, :9]
        d = np.diff(cyc, axis=1)
        life = cyc[:, 8] - cyc[:, 0]
        rt0, rt1 = st[:, 9], st[:, 10]
        xcc = (st[:, 11] >> 32) & 0xF
        span_ns = (rt1.max() - rt0.min()) * 10
        summary = {
            "kernel_span_us(realtime)": span_ns / 1e3,
            "wave_start_spread_us": (rt0.max() - rt0.min()) * 10 / 1e3,
            "wave_end_spread_us": (rt1.max() - rt1.min()) * 10 / 1e3,
            "wave_life_us(realtime) p50/p90/max": [float(np.percentile((rt1 - rt0) * 10 / 1e3, q)) for q in (50, 90, 100)],
            "wave_life_cycles p50/p90/max": [float(np.percentile(life, q)) for q in (50, 90, 100)],
            "clock_ghz(median)": float(np.median(life / ((rt1 - rt0) * 10.0 + 1e-9))),
            "phase_cycles_mean": {PHASES[j]: float(d[:, j].mean()) for j in range(8)},
            "load_issue_cycles_mean": float((st[:, 12] - st[:, 0]).mean()),
            "counter_landed_cycles_mean": float((st[:, 13] - st[:, 0]).mean()),
            "istate_landed_cycles_mean": float((st[:, 14] - st[:, 0]).mean()),
            "phase_cycles_p90": {PHASES[j]: float(np.percentile(d[:, j], 90)) for j in range(8)},
            "xcc_counts": np.bincount(xcc, minlength=8).tolist(),
            "start_us_hist": np.histogram((rt0 - rt0.min()) * 10 / 1e3, bins=8)[0].tolist(),
            "end_us_pcts": [float(np.percentile((rt1 - rt0.min()) * 10 / 1e3, q)) for q in (10, 50, 90, 99, 100)],
        }
        res.append(summary)
    print(json.dumps(res[-1], indent=1))
    env.close()


if __name__ == "__main__":
    {"build": build, "run": run}[sys.argv[1]]()
