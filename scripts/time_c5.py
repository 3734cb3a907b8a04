"""The C5 step kernel alone (65 536 envs, 32-gate tracks, rotor-constant DR; bench c5_32_gates' env): HIP events around
graph replays.  GR_LIB_PATH picks a variant library.  Usage: python scripts/time_c5.py [--out file]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

env = bench.make_env(65536, 0, "cuda:0", 32, "dd_explicit", False, dr_rotor=1)
g = torch.Generator(device="cuda:0").manual_seed(7)
actions = torch.randn(bench.ACTION_RING, 65536, 4, device="cuda:0", generator=g)
for k in range(64):
    env.step(actions[k % bench.ACTION_RING])
graph = bench.capture_graph(env, actions)
kt = bench.kernel_timing(graph)
res = {"lib": os.environ.get("GR_LIB_PATH", "tree"), "c5_step_us": kt["kernel_us"]}
print(json.dumps(res))
if len(sys.argv) > 2 and sys.argv[1] == "--out":
    with open(sys.argv[2], "a") as f:
        f.write(json.dumps(res) + "\n")
