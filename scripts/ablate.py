"""Timing-only ablation of the fused step kernel (results are NOT correct envs).

  python scripts/ablate.py build        # here: compile one libgr variant per flag into build/abl/
  python scripts/ablate.py run          # GPU box: time each variant (HIP events, 65 536 envs)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "abl")
CSRC = os.path.join(ROOT, "generalizableracing_amd", "csrc")
BASE_FLAGS = "-fno-slp-vectorize"  # as the Makefile
EXTRA = {"slp": ""}  # compiler-flag variants (no source ablation): replace BASE_FLAGS
VARIANTS = {
    "slp": [],
    "base": [], "noreset": ["GR_ABL_NORESET"], "nocoll": ["GR_ABL_NOCOLL"], "noobsnoise": ["GR_ABL_NOOBSNOISE"],
    "nogatenoise": ["GR_ABL_NOGATENOISE"], "nolog": ["GR_ABL_NOLOG"], "noobs": ["GR_ABL_NOOBS"],
    "nolds": ["GR_ABL_NOLDS"],
    "noldsattr": ["GR_ABL_NO_LDS_ATTR"],
    "all": ["GR_ABL_NORESET", "GR_ABL_NOCOLL", "GR_ABL_NOOBSNOISE", "GR_ABL_NOGATENOISE", "GR_ABL_NOLOG", "GR_ABL_NOOBS"],
}


def build():
    os.makedirs(OUT, exist_ok=True)
    procs = []
    for name, flags in VARIANTS.items():
        d = " ".join(f"-D{f}" for f in flags)
        d += " " + EXTRA.get(name, BASE_FLAGS)
        cmd = (f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "
               f"-fhip-fp32-correctly-rounded-divide-sqrt {d} -shared -o {OUT}/libgr_{name}.so "
               f"{CSRC}/gr_kernels.hip -x hip {CSRC}/gr_capi.cpp")
        procs.append(subprocess.Popen(cmd, shell=True))
    for p in procs:
        assert p.wait() == 0


def time_one(n=65536, steps=512):
    import torch

    sys.path.insert(0, ROOT)
    import bench

    env = bench.make_env(n, 0, "cuda:0", 8, "dd_explicit")
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = torch.randn(bench.ACTION_RING, n, 4, device="cuda:0", generator=g)
    for k in range(32):
        env.step(acts[k % bench.ACTION_RING])
    graph = bench.capture_graph(env, acts)
    return bench.kernel_timing(env, acts, steps, graph)["kernel_us"]


def modes(n=65536, reps=200):
    """Per-mode kernel times: gr_step, gr_reset(all), gr_reset(none), gr_observe (HIP events)."""
    import numpy as np
    import torch

    sys.path.insert(0, ROOT)
    import bench

    env = bench.make_env(n, 0, "cuda:0", 8, "dd_explicit")
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = torch.randn(bench.ACTION_RING, n, 4, device="cuda:0", generator=g)
    for k in range(32):
        env.step(acts[k % bench.ACTION_RING])
    res = {"step": bench.kernel_timing(env, acts, reps, None)["eager_event_us"]}
    none = np.zeros(0, np.int64)
    for name, fn in (("reset_all", lambda: env.reset()), ("reset_none", lambda: env.reset(env_ids=none)),
                     ("observe", lambda: env.observe())):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        res[name] = s.elapsed_time(e) / reps * 1e3
    print(json.dumps(res))


def run():
    res = {}
    for name in VARIANTS:
        env = dict(os.environ, GR_LIB_PATH=f"{OUT}/libgr_{name}.so")
        out = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=300)
        res[name] = float(out.stdout.strip().splitlines()[-1]) if out.returncode == 0 else out.stderr[-500:]
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    {"build": build, "run": run, "one": lambda: print(time_one()), "modes": modes}[sys.argv[1]]()
