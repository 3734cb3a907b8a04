"""Per-phase wave timelines of the fused step kernel (diagnostic build, -DGR_STAMPS).

  python scripts/stamps.py build     # here: variants/stamps/libgr.so
  python scripts/stamps.py run       # GPU box: GR_LIB_PATH=variants/stamps/libgr.so, prints a JSON summary

Stamps of the step kernel (lane 0 of each wave, s_memtime shader cycles; 9/10 s_memrealtime
(100 MHz) at entry/exit; 11 XCC_ID<<32 | HW_ID):
  physics waves:     0 entry, 3 controller+integrator, 4 table barrier + collision,
                     5 reward + handover written, 8 after barrier 2, stores and log rows
  observation waves: 0 entry, 1 loads + obs noise, 2 table barrier, 6 reset draws,
                     7 barrier 2 + resets + gate progress, 8 observations + log rows
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "variants", "stamps")  # (not under build/: .gpurunignore keeps build/ off the box)
CSRC = os.path.join(ROOT, "generalizableracing_amd", "csrc")
PHASES = ["obs_noise", "table_barrier", "ctrl_integrate", "collision", "reward_term", "reset_advance",
          "obs_store_issue", "log"]


def build():
    os.makedirs(OUT, exist_ok=True)
    cmd = (f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "
           f"-fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -DGR_STAMPS -shared -o {OUT}/libgr.so "
           f"{CSRC}/gr_kernels.hip {CSRC}/gr_camera.hip {CSRC}/gr_policy.hip {CSRC}/gr_policy_f32.hip {CSRC}/gr_bn.hip {CSRC}/gr_update.hip -x hip {CSRC}/gr_capi.cpp")
    subprocess.run(cmd, shell=True, check=True)


ROLE_PHASES = {
    "physics": [("loads+integrate", 0, 3), ("barrier1", 3, 14), ("gate_collision", 14, 15),
                ("obstacle_wait", 15, 4), ("termination+handover", 4, 5),
                ("barrier2+reward+stores", 5, 12), ("log", 12, 8)],
    "policy": [("loads(+obstacle prefetch)", 0, 1), ("barrier1 / obs_noise", 1, 2), ("obstacle_test", 2, 12),
               ("barrier2_wait", 12, 13),
               ("merge+advance", 13, 7), ("policy_obs+log", 7, 8)],
    "episode": [("loads+reset_draws", 0, 1), ("barrier1", 1, 2), ("reset_apply+xr", 2, 6),
                ("barrier2_wait", 6, 13), ("merge+advance+istate", 13, 14), ("critic_obs", 14, 8)],
}


def run(n=int(os.environ.get("N", "65536")), steps=200):
    os.environ["GR_LIB_PATH"] = os.path.join(OUT, "libgr.so")
    import ctypes as C

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    import bench

    obst = os.environ.get("GR_STAMPS_OBST", "1") == "1"
    env = bench.make_env(n, 0, "cuda:0", 8, "dd_explicit", obst)
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = torch.randn(bench.ACTION_RING, n, 4, device="cuda:0", generator=g)
    for k in range(steps):
        env.step(acts[k % bench.ACTION_RING])
    torch.cuda.synchronize()
    waves = max(1, n // 256) * 12  # step kernel: 12 waves per 256-env workgroup
    buf = np.zeros(waves * 16, np.uint64)
    assert env._lib.gr_debug_read_stamps(buf.ctypes.data_as(C.c_void_p), buf.size) == 0
    st = buf.reshape(waves, 16).astype(np.int64)
    role = (np.arange(waves) % 12) // 4  # waves 0-3 physics, 4-7 policy, 8-11 episode
    rt0, rt1 = st[:, 9], st[:, 10]
    out = {
        "kernel_span_us(realtime)": float((rt1.max() - rt0.min()) * 10 / 1e3),
        "wave_start_spread_us": float((rt0.max() - rt0.min()) * 10 / 1e3),
        "end_us_pcts(10,50,90,99,100)": [float(np.percentile((rt1 - rt0.min()) * 10 / 1e3, q))
                                         for q in (10, 50, 90, 99, 100)],
    }
    # per XCD (stamp 11: XCC_ID << 32 | HW_ID): when its workgroups start and end, relative to the first start
    xcc = (st[:, 11] >> 32) & 0xF
    wg_end = (rt1.reshape(-1, 12).max(axis=1) - rt0.min()) * 10 / 1e3
    wg_start = (rt0.reshape(-1, 12).min(axis=1) - rt0.min()) * 10 / 1e3
    wg_xcc = xcc.reshape(-1, 12)[:, 0]
    out["per_xcd_us"] = {int(x): {"start_p50": float(np.median(wg_start[wg_xcc == x])),
                                  "end_p50": float(np.median(wg_end[wg_xcc == x])),
                                  "end_max": float(wg_end[wg_xcc == x].max()),
                                  "workgroups": int((wg_xcc == x).sum())} for x in np.unique(wg_xcc)}
    wg_dur = wg_end - wg_start
    out["workgroup_duration_us_pcts(10,50,90,100)"] = [float(np.percentile(wg_dur, q)) for q in (10, 50, 90, 100)]
    # what the slowest tenth of the workgroups spend their extra time on: per role and phase, mean cycles of the
    # workgroups above the 90th duration percentile minus those at or below the median
    slow = np.repeat(wg_dur > np.percentile(wg_dur, 90), 12)
    fast = np.repeat(wg_dur <= np.percentile(wg_dur, 50), 12)
    out["slow_minus_fast_phase_cycles"] = {
        name: {ph: float((st[slow & (role == r)][:, b_] - st[slow & (role == r)][:, a_]).mean()
                         - (st[fast & (role == r)][:, b_] - st[fast & (role == r)][:, a_]).mean())
               for ph, a_, b_ in ROLE_PHASES[name]}
        for r, name in enumerate(("physics", "policy", "episode"))}
    out["slow_workgroup_ids"] = [int(b) for b in np.nonzero(wg_dur > np.percentile(wg_dur, 90))[0]]
    for r, name in enumerate(("physics", "policy", "episode")):
        sel = st[role == r]
        life = sel[:, 8] - sel[:, 0]
        out[name] = {
            "life_cycles p50/p90/max": [float(np.percentile(life, q)) for q in (50, 90, 100)],
            "end_us p50/p90/max": [float(np.percentile((sel[:, 10] - rt0.min()) * 10 / 1e3, q)) for q in (50, 90, 100)],
            "phase_cycles_mean": {ph: float((sel[:, b_] - sel[:, a_]).mean()) for ph, a_, b_ in ROLE_PHASES[name]},
            "phase_cycles_p90": {ph: float(np.percentile(sel[:, b_] - sel[:, a_], 90))
                                 for ph, a_, b_ in ROLE_PHASES[name]},
        }
    print(json.dumps(out, indent=1))
    env.close()


def policy(n=65536):
    """Phase timelines of the fused policy kernel (gr_policy_forward) from its stamps."""
    os.environ["GR_LIB_PATH"] = os.path.join(OUT, "libgr.so")
    import ctypes as C

    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl.fused_inference import FusedPolicyInference

    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to("cuda:0")
    fused = FusedPolicyInference(pol, n, "cuda:0")
    obs = torch.randn(n, 16, device="cuda:0")
    for _ in range(8):
        fused.act(obs, obs)
    torch.cuda.synchronize()
    waves = 4096
    buf = np.zeros(waves * 16, np.uint64)
    assert fused._lib.gr_debug_read_policy_stamps(buf.ctypes.data_as(C.c_void_p), buf.size) == 0
    st = buf.reshape(waves, 16).astype(np.int64)
    live = st[:, 0] != 0
    st = st[live]
    rt0, rt1 = st[:, 14], st[:, 15]
    out = {"waves": int(live.sum()), "kernel_span_us(realtime)": float((rt1.max() - rt0.min()) * 10 / 1e3),
           "wave_start_spread_us": float((rt0.max() - rt0.min()) * 10 / 1e3),
           "end_us_pcts(10,50,90,100)": [float(np.percentile((rt1 - rt0.min()) * 10 / 1e3, q)) for q in (10, 50, 90, 100)],
           "life_cycles_p50": float(np.percentile(st[:, 4 + 4 * 1] - st[:, 0], 50)),
           "staging_cycles_mean": float((st[:, 1] - st[:, 0]).mean())}
    prev = st[:, 1]
    for k in range(2):
        l1, l23, ep = st[:, 2 + 4 * k], st[:, 3 + 4 * k], st[:, 4 + 4 * k]
        out[f"tile{k}"] = {"layer1": float((l1 - prev).mean()), "layer2+3": float((l23 - l1).mean()),
                           "epilogue": float((ep - l23).mean())}
        prev = ep
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    {"build": build, "run": run, "policy": policy}[sys.argv[1]]()
