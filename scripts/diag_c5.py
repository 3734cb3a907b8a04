"""Diagnostic: the bench's C5 leg step by step with progress lines (65 536 envs, 32 gates, rotor DR)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

T0 = time.time()


def say(m):
    print(f"[{time.time() - T0:6.1f}s] {m}", flush=True)


n = int(os.environ.get("N", "65536"))
dev = "cuda:0"
rotor = int(os.environ.get("ROTOR", "1"))
env = bench.make_env(n, 0, dev, 32, "dd_explicit", False, dr_rotor=rotor)
say("made env")
g = torch.Generator(device=dev).manual_seed(1234)
actions = torch.randn(bench.ACTION_RING, n, 4, device=dev, generator=g)
for k in range(8):
    env.step(actions[k])
    torch.cuda.synchronize()
    say(f"eager step {k}")
graph = bench.capture_graph(env, actions)
say("captured")
kt = bench.kernel_timing(graph)
say(f"kernel {kt}")
del graph
rate, us, _ = bench.policy_in_loop_fused(env, 512, dev)
say(f"fused {rate} {us}")
sink = torch.empty(2, n, 16, device=dev, dtype=torch.bfloat16)
env.set_obs_sink(sink[0], sink[1])
env.step(actions[0])
torch.cuda.synchronize()
say("sink step")
graph = bench.capture_graph(env, actions)
say("sink captured")
kt = bench.kernel_timing(graph)
say(f"sink kernel {kt}")
