"""Env shards per GPU as independent chains: S shards of N/S envs (separate contexts, disjoint env ids),
each shard's 64 steps on its own stream, all captured in one hipGraph whose chains only join at the end.
Reports env-steps/s over all N envs against the one-shard graph (bench.py's headline form), with random
actions (the env step alone) and with the fused rollout inference in each chain.

    python scripts/bench_shards.py [--num-envs 65536] [--shards 1 2 4]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import ACTION_RING, make_env  # noqa: E402


def run(n, shards, policy, device="cuda:0", reps=8):
    m = n // shards
    envs = [make_env(m, 0, device, 8, "dd_explicit", False) for _ in range(shards)]
    for k, e in enumerate(envs):  # disjoint env ids (RNG streams) as separate shards of one rank
        e.cfg.env_id_offset = k * m
    fused = None
    if policy:
        from generalizableracing_amd.rsl_rl import ActorCritic
        from generalizableracing_amd.rsl_rl.fused_inference import FusedPolicyInference

        pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(device)
        fused = [FusedPolicyInference(pol, m, device, env_id_offset=k * m) for k in range(shards)]
    g = torch.Generator(device=device).manual_seed(1234)
    acts = [torch.randn(ACTION_RING, m, 4, device=device, generator=g) for _ in range(shards)]
    obs = [e.observe() for e in envs]
    streams = [torch.cuda.Stream() for _ in range(shards)]

    def chain(k, steps):
        o = obs[k]
        for t in range(steps):
            if fused is not None:
                a = fused[k].act(o["policy"], o["critic"])[0]
            else:
                a = acts[k][t % ACTION_RING]
            o = envs[k].step(a)[0]
        obs[k] = o

    cur = torch.cuda.current_stream()
    for k, s in enumerate(streams):  # warm-up outside capture, then align the ping-pong bindings
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            chain(k, 2)
            if fused is not None and (envs[k]._calls - fused[k]._calls) % 2:
                obs[k] = envs[k].observe()
            while envs[k]._calls % ACTION_RING != 0 or (fused is not None and fused[k]._calls % 2 != 0):
                chain(k, 1)
        cur.wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        cap = torch.cuda.current_stream()
        for k, s in enumerate(streams):
            s.wait_stream(cap)
            with torch.cuda.stream(s):
                chain(k, ACTION_RING)
            cap.wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        graph.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for e in envs:
        e.close()
    return {"shards": shards, "envs_per_shard": m, "policy": "fused" if policy else "random actions",
            "env_steps_per_s": n * reps * ACTION_RING / dt, "us_per_step_all_envs": dt * 1e6 / (reps * ACTION_RING)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4])
    a = ap.parse_args()
    for policy in (False, True):
        for s in a.shards:
            print(json.dumps(run(a.num_envs, s, policy)), flush=True)
