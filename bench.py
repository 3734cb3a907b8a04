"""Benchmark: env-steps/s of the fused racing-env step at 65 536 envs per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--num-envs 65536]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

The first form with N > 1 starts the second itself, as a child process (launch_ranks).  Under
torch.distributed.run, --gpus must equal WORLD_SIZE, and with the nccl (RCCL) backend every rank
must own a distinct GPU; anything else exits non-zero rather than print a line for another world.

A "step" is one pass of the hot path (ManagerBasedDiffRLEnv.step equivalent:
action processing, CTBR controller, integrator, collision, gate progress,
reward, termination, in-lane reset, observation, log reduction) over all envs
of a rank, with pre-generated synthetic actions already resident in HBM.
Envs shard one shard per GPU with no data-path collective ("scaling": "weak");
`value` = envs * world_size * K / max-over-ranks wall time.

Also reported (same JSON line): the fused kernel's roofline (HIP events over
graph replays, algorithmic bytes from gr_bytes_per_env_step, PMC traffic from
profiles/pmc_traffic.json) and the CPU oracle timed on the host ("port", rank 0,
N=1 only).  Single-GPU extras: policy-in-the-loop rates (PyTorch actor; fused
MFMA inference in one hipGraph with the step), the step on obstacle tracks, an
env-count sweep, config C5 (32-gate tracks), Perf/total_fps of PPO training at
4 096 envs (C2, eager and graph-captured update) and 65 536 envs, and the depth
camera.  Every run, multi-rank included, also reports `distributed_train`: PPO training at the rank's envs with
the per-mini-batch gradient all-reduce live (BASELINE C4), world-summed Perf/total_fps, per-rank update and
all-reduce time, and a check that the ranks' parameters stay bit-identical.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import subprocess
import sys
import time


def launch_ranks(argv) -> int | None:
    """`python bench.py --gpus N` with N > 1 outside torch.distributed.run: start the N ranks ourselves, one per
    GPU, as `python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py
    <the same arguments>` in a CHILD process, and return its exit status.  Rank 0's JSON line reaches our stdout
    (inherited).  Called before torch or the package is imported, so this process never touches the GPU (no
    exec, the launcher is a child).  Returns None when there is nothing to launch (N == 1, or already a rank)."""
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=None)
    known, _ = p.parse_known_args(argv)
    if known.gpus is None or known.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(known.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    print(f"[bench] launching {known.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


if __name__ == "__main__":
    _rc = launch_ranks(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from generalizableracing_amd.envs.racing_cfg import RacingEnvCfg, SceneCfg, SimCfg, TerrainCfg  # noqa: E402
from generalizableracing_amd.envs.racing_env import RacingEnv  # noqa: E402
from generalizableracing_amd import _abi as _abi_mod  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_MFMA_PEAK_TFS = 157.3  # MI355X dense fp32 matrix peak (v_mfma_f32_16x16x4_f32; MI355X_MICROARCH.md)
# the PPO update's useful flops per sample and epoch, MLP(256, 256) actor (16 -> 4) and critic (16 -> 1): forward
# 140 544 MACs, weight gradients 140 544, input gradients below the first layer 132 352 (2 flops per MAC)
UPDATE_FLOPS_PER_SAMPLE = 2 * (2 * (16 * 256 + 256 * 256 + 256 * 4 + 16 * 256 + 256 * 256 + 256)
                               + (256 * 256 + 256 * 4 + 256 * 256 + 256))
ACTION_RING = 64
STREAM_FLOOR_US = 5.15  # 65 536 envs: the step's own bytes as a pure stream (BASELINE §2)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="number of GPUs = ranks; N > 1 outside torch.distributed.run launches the N ranks itself "
                        "(launch_ranks); under torch.distributed.run it must equal WORLD_SIZE")
    p.add_argument("--steps", type=int, default=1024)
    p.add_argument("--warmup", type=int, default=64)
    p.add_argument("--num-envs", type=int, default=65536)
    p.add_argument("--gates", type=int, default=8)
    p.add_argument("--obstacles", type=int, default=0, help="1: the reference task's walls / orbits / ground "
                   "obstacles (add_obs, add_ground_obs); 0: gates and ground only (BASELINE config C3).  The "
                   "default line also reports the obstacle variant under 'with_obstacles'")
    p.add_argument("--integrator", default="dd_explicit")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--no-extras", action="store_true", help="skip policy/train/cpu legs (profiling runs)")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--legs", default="all",
                   help="comma-separated extra legs to run (policy, obstacles, sweep, c5, regen, dtrain, train4096, "
                        "train65536, camera, vision, cpu) or 'all'; the headline step always runs; at WORLD_SIZE > 1 "
                        "'all' means dtrain (the data-parallel training leg) only")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, one GPU per rank); gloo only to rehearse the multi-rank path with ranks "
                        "sharing one GPU")
    return p.parse_args()


def want(a, leg: str) -> bool:
    """Whether the extra leg `leg` runs (--legs; all by default, none with --no-extras)."""
    return not a.no_extras and (a.legs == "all" or leg in a.legs.split(","))


def barrier():
    if dist.is_initialized():
        dist.barrier()


def max_over_ranks(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    dev = device if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


_T0 = time.time()


def progress(msg):
    """One line per finished leg on stderr (the JSON line alone goes to stdout)."""
    print(f"[bench {time.time() - _T0:6.1f}s] {msg}", file=sys.stderr, flush=True)


def make_env(n, rank, device, gates, integrator, obstacles=True, **overrides):
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=device), stage=1, integrator=integrator,
                       terrain=TerrainCfg(num_gates=gates, obstacles=obstacles), env_id_offset=rank * n,
                       track_seed_offset=rank, overrides=overrides)
    env = RacingEnv(cfg)
    env.reset()
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    env.episode_length_buf = torch.randint(0, env.max_episode_length, (n,), generator=g, dtype=torch.int32).to(device)
    return env


def capture_graph(env, actions, length=ACTION_RING):
    """hipGraph of `length` (<= ACTION_RING) consecutive env steps (buffer bindings and action pointers baked
    in).  The host call counter is realigned to a multiple of the ring first, so every graph starts on the
    same bindings and replays of several graphs chain like consecutive eager calls."""
    assert 1 <= length <= ACTION_RING
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for k in range(2):  # stream warm-up outside capture
            env.step(actions[k % ACTION_RING])
    torch.cuda.current_stream().wait_stream(s)
    while env._calls % ACTION_RING != 0:
        env.step(actions[env._calls % ACTION_RING])
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for k in range(length):
            env.step(actions[k])
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    return graph


def time_env_steps(env, actions, steps, use_graph):
    """Returns (seconds for exactly `steps` env steps, launch mode, the 64-step graph or None).

    Graph mode times steps // 64 replays of a 64-step graph plus one replay of a graph of the remaining
    steps % 64 launches, so any K (the driver's K=20 included) is timed as hipGraph launches."""
    graph = rem_graph = None
    reps, rem = 0, steps
    if use_graph:
        graph = capture_graph(env, actions)
        reps, rem = divmod(steps, ACTION_RING)
        if rem:
            rem_graph = capture_graph(env, actions, rem)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        graph.replay()
    if rem_graph is not None:
        rem_graph.replay()
    elif graph is None:
        for k in range(rem):
            env.step(actions[k % ACTION_RING])
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    del rem_graph
    return t1 - t0, ("hipgraph" if graph is not None else "eager"), graph


def repeat_median(graph, n, reps=3, length=1024):
    """SURVEY §8d's steady-state form: `reps` timed runs of `length` steps (64-step graph replays), median
    env-steps/s of one rank."""
    rates = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(length // ACTION_RING):
            graph.replay()
        torch.cuda.synchronize()
        rates.append(n * (length // ACTION_RING) * ACTION_RING / (time.perf_counter() - t0))
    return float(np.median(rates))


def kernel_timing(graph, replays=16):
    """Average duration of one fused-kernel launch: HIP events on the launch stream around back-to-back
    replays of the 64-launch graph (each replay is exactly 64 env-kernel launches on torch's current stream,
    the stream gr_step launches on), so the per-launch figure includes the graph's inter-kernel gaps — the
    quantity rocprofv3's kernel-trace average approximates from below.  Per-launch event pairs are never
    used: their record overhead exceeds the kernel's own time at this size."""
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    graph.replay()
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(replays):
        graph.replay()
    e1.record(stream)
    e1.synchronize()
    return {"kernel_us": e0.elapsed_time(e1) * 1e3 / (replays * ACTION_RING),
            "timing": f"HIP events around {replays} back-to-back replays of a {ACTION_RING}-launch hipGraph"}


def policy_in_loop(env, steps, device):
    """env step + actor MLP(16->256->256->4) inference per step (rollout without learning)."""
    from generalizableracing_amd.rsl_rl import ActorCritic

    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(device).eval()
    obs = env.observe()["policy"]
    with torch.inference_mode():
        for _ in range(8):
            obs = env.step(pol.act_inference(obs))[0]["policy"]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            obs = env.step(pol.act_inference(obs))[0]["policy"]
        torch.cuda.synchronize()
    return env.num_envs * steps / (time.perf_counter() - t0)


def policy_in_loop_graphed(env, steps, device):
    """SURVEY §8d env-only rate at the reference's precision: per step the fp32 PyTorch actor MLP
    (16-256-256-4, LeakyReLU) computes the mean, a Gaussian sample a = mu + std * eps is drawn (what
    Normal.sample computes; torch.normal itself reads the std back to the host, which a capture forbids),
    and gr_step runs on it; 64 such steps are captured in one hipGraph and replayed."""
    from generalizableracing_amd.rsl_rl import ActorCritic

    n = env.num_envs
    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(device).eval()

    def one_step(obs):
        with torch.no_grad():
            mu = pol.actor(obs)
            a = mu + pol.std * torch.randn_like(mu)
        return env.step(a)[0]["policy"]

    obs = env.observe()["policy"]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            obs = one_step(obs)
    torch.cuda.current_stream().wait_stream(s)
    while env._calls % ACTION_RING != 0:
        obs = one_step(obs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        o = obs
        for _ in range(ACTION_RING):
            o = one_step(o)
    g.replay()
    torch.cuda.synchronize()
    reps = max(1, steps // ACTION_RING)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return n * reps * ACTION_RING / (time.perf_counter() - t0)


def policy_in_loop_fused(env, steps, device, precision="bf16", actor_only=False, sink_ring=None):
    """C5 "hipGraph-captured step + inference": per step, the fused MFMA inference of both MLPs
    (FusedPolicyInference: actor mean + Gaussian sample + log prob, critic value; bf16 operands with fp32
    accumulation, or fp32 operands on fp32 MFMA = the reference's precision) on the step's observations,
    then gr_step on the sampled actions; 64 such steps are captured in one hipGraph and replayed.  actor_only:
    the actor network alone (mean, sample, log prob; no value), the inference an env-only rollout needs.
    sink_ring: [ACTION_RING, 2, n, 16] bf16 rollout rows; step k of the graph writes its observation rows into slot
    k (gr_bind_obs_sink rebound per step, as the runner rebinds it to the storage slot of each transition).
    Returns (env-steps/s, per-launch us of the inference kernel, its useful TFLOP/s)."""
    from generalizableracing_amd.rsl_rl import ActorCritic
    from generalizableracing_amd.rsl_rl.fused_inference import FusedPolicyInference

    n = env.num_envs
    pol = ActorCritic(16, 16, 4, [256, 256], [256, 256], "lrelu").to(device)
    fused = FusedPolicyInference(pol, n, device, env_id_offset=env.cfg.env_id_offset, precision=precision)

    def one_step(obs):
        acts = fused.act(obs["policy"], None if actor_only else obs["critic"])[0]
        if sink_ring is not None:
            slot = sink_ring[env._calls % ACTION_RING]
            env.set_obs_sink(slot[0], slot[1])
        return env.step(acts)[0]

    obs = env.observe()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            obs = one_step(obs)
    torch.cuda.current_stream().wait_stream(s)
    # align the ping-pong bindings (each step advances both call counters by one: fix their parity first)
    if (env._calls - fused._calls) % 2:
        obs = env.observe()
    while env._calls % ACTION_RING != 0 or fused._calls % 2 != 0:
        obs = one_step(obs)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        o = obs
        for _ in range(ACTION_RING):
            o = one_step(o)
    g.replay()
    torch.cuda.synchronize()
    reps = max(1, steps // ACTION_RING)
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    rate = n * reps * ACTION_RING / (time.perf_counter() - t0)
    if sink_ring is not None:
        env.set_obs_sink(None)
    # the inference kernel alone (events on the current stream, 64 back-to-back launches)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    x = obs["policy"].clone()
    xc = None if actor_only else x
    for _ in range(4):
        fused.act(x, xc)
    e0.record()
    for _ in range(64):
        fused.act(x, xc)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 64
    # useful flops: actor (+ critic; its 1-row output counted as 4, the padded rows are free)
    flops = 2 * n * (1 if actor_only else 2) * (16 * 256 + 256 * 256 + 256 * 4)
    return rate, us, flops / (us * 1e-6) / 1e12


def env_count_sweep(rank, device, a, sizes=(16384, 262144, 1048576)):
    """The same step at other env counts per GPU (HBM holds far more than the 65 536 of the headline
    config): per-launch us from HIP events over graph replays, env-steps/s and algorithmic GB/s."""
    out = {}
    for n in sizes:
        env = make_env(n, rank, device, a.gates, a.integrator, False)
        g = torch.Generator(device=device).manual_seed(1234 + rank)
        acts = torch.randn(ACTION_RING, n, 4, device=device, generator=g)
        for k in range(8):
            env.step(acts[k % ACTION_RING])
        torch.cuda.synchronize()
        graph = capture_graph(env, acts)
        kt = kernel_timing(graph)
        del graph
        rd, wr = env.bytes_per_env_step()
        us = kt["kernel_us"]
        out[str(n)] = {"kernel_us": us, "env_steps_per_s": n / (us * 1e-6),
                       "achieved_GBps": (rd + wr) * n / (us * 1e-6) / 1e9,
                       "frac_of_8TBps": (rd + wr) * n / (us * 1e-6) / 8e12,
                       "read_frac_of_8TBps": rd * n / (us * 1e-6) / 8e12}
        env.close()
        del acts
        torch.cuda.empty_cache()
    return out


def train_fps(device, n=4096, iters=3, fused=False, bf16_storage=False, graph_update=False, bf16_update=False,
              obs_sink=True, fused_precision="bf16", fused_mlp=True):
    """The reference's Perf/total_fps (24 steps x N / (collect + learn)) of rsl_rl PPO with MLP(256,256):
    config C2 at 4 096 envs fp32; at 65 536 envs also with the fused bf16 rollout inference and bf16
    rollout obs buffers (C5's training options; the update stays fp32)."""
    from generalizableracing_amd.envs.racing_env import RslRlVecEnvWrapper
    from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg

    venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=device))))
    cfg = QuadcopterPPORunnerCfg(device=device)
    cfg.algorithm.fused_rollout_inference = bool(fused)
    cfg.algorithm.fused_rollout_precision = fused_precision
    cfg.algorithm.storage_obs_dtype = "bfloat16" if bf16_storage else "float32"
    cfg.algorithm.graph_update = bool(graph_update)
    cfg.algorithm.update_autocast_bf16 = bool(bf16_update)
    cfg.algorithm.obs_sink = bool(obs_sink)
    cfg.algorithm.fused_mlp = bool(fused_mlp)
    runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=device)
    upd = runner.alg.update
    upd_s = []

    def timed_update():  # alg.update alone (learn_time also holds compute_returns)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = upd()
        torch.cuda.synchronize()
        upd_s.append(time.perf_counter() - t0)
        return out

    runner.alg.update = timed_update
    runner.learn(1, init_at_random_ep_len=True)  # warm-up iteration
    fps = []
    for _ in range(iters):
        runner.learn(1)
        fps.append(runner.last_log["fps"])
    alg = runner.alg
    samples = alg.num_learning_epochs * n * cfg.num_steps_per_env
    upd_ms = float(np.median(upd_s[1:])) * 1e3
    tfs = UPDATE_FLOPS_PER_SAMPLE * samples / (upd_ms * 1e-3) / 1e12
    progress(f"train_fps n={n} fused={fused}({fused_precision}) bf16_storage={bf16_storage} graph_update={graph_update} "
             f"obs_sink={obs_sink} fused_mlp={fused_mlp}: {np.median(fps):.4g} (update {upd_ms:.1f} ms, "
             f"{tfs:.1f} TFLOP/s)")
    venv.close()
    return {"fps": float(np.median(fps)), "update_ms": upd_ms, "update_TFLOPs": tfs,
            "update_frac_of_fp32_mfma_peak": tfs / FP32_MFMA_PEAK_TFS if not bf16_update else None}


def train_fps_distributed(device, n, rank, ws, iters=3):
    """BASELINE config C4's exchange on the critical path: the reference's Perf/total_fps (on_policy_runner.py:229,
    24 steps x n envs x world_size / iteration time) of PPO with MLP(256,256) at n envs per rank, each rank on its own
    env shard (env ids and track seeds offset by rank), fp32 fused rollout inference, the graph-captured update.  At
    world size > 1 every mini-batch step of the update (ppo.py:174-177) all-reduces the flat gradient + KL mean
    (distributed.FlatGrads, 566 KB) eagerly between the step's two graphs, 20 exchanges per iteration.

    World-summed fps = 24 x n x ws / (max over ranks of the iteration time), median over `iters` iterations after
    one warm-up iteration.  Per rank: update_ms (alg.update alone) and the time the update's stream spends in the
    exchanges (HIP events around each all-reduce, summed per iteration).  After the leg every rank's parameters are
    hashed and compared: a data-parallel update must leave them bit-identical on every rank."""
    import hashlib

    from generalizableracing_amd.envs.racing_env import RslRlVecEnvWrapper
    from generalizableracing_amd.rsl_rl import OnPolicyRunner, QuadcopterPPORunnerCfg
    from generalizableracing_amd.rsl_rl import distributed as gdist

    venv = RslRlVecEnvWrapper(RacingEnv(RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=device),
                                                     env_id_offset=rank * n, track_seed_offset=rank)))
    cfg = QuadcopterPPORunnerCfg(device=device)
    cfg.algorithm.fused_rollout_inference = True
    cfg.algorithm.fused_rollout_precision = "fp32"
    cfg.algorithm.graph_update = True
    torch.manual_seed(1 + rank)  # rank 0's initial parameters are broadcast (PPO.__init__)
    runner = OnPolicyRunner(venv, cfg.to_dict(), log_dir=None, device=device)
    upd = runner.alg.update
    upd_ms, ar_ms, n_ar = [], [], []

    def timed_update():
        gdist.FlatGrads.timings = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = upd()
        torch.cuda.synchronize()
        upd_ms.append((time.perf_counter() - t0) * 1e3)
        ar_ms.append(sum(e0.elapsed_time(e1) for e0, e1 in gdist.FlatGrads.timings))
        n_ar.append(len(gdist.FlatGrads.timings))
        gdist.FlatGrads.timings = None
        return out

    runner.alg.update = timed_update
    iter_s = []
    try:
        runner.learn(1, init_at_random_ep_len=True)  # warm-up iteration (graph capture)
        for _ in range(iters):
            barrier()
            runner.learn(1)
            iter_s.append(runner.last_log["collection_time"] + runner.last_log["learn_time"])
    finally:
        gdist.FlatGrads.timings = None
    worst = [max_over_ranks(t, device) for t in iter_s]
    fps = float(np.median([runner.num_steps_per_env * n * ws / t for t in worst]))
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in runner.alg.policy.parameters()]).cpu()
    digest = hashlib.sha256(flat.numpy().tobytes()).hexdigest()
    me = {"rank": rank, "update_ms": float(np.median(upd_ms[1:])), "allreduce_ms_per_iteration": float(np.median(ar_ms[1:])),
          "allreduces_per_iteration": int(n_ar[-1]), "iteration_s": float(np.median(iter_s)), "param_sha256": digest}
    ranks = [me]
    if dist.is_initialized():
        ranks = [None] * ws
        dist.all_gather_object(ranks, me)
    venv.close()
    progress(f"train_fps_distributed n={n} ws={ws}: {fps:.4g} (update {me['update_ms']:.1f} ms, "
             f"all-reduce {me['allreduce_ms_per_iteration']:.2f} ms / iteration)")
    return {"train_total_fps": fps, "world_size": ws, "num_envs_per_rank": n,
            "params_identical_on_all_ranks": len({r["param_sha256"] for r in ranks}) == 1,
            "ranks": ranks,
            "note": "Perf/total_fps = 24 x envs x world_size / max-over-ranks iteration time (median of "
                    f"{iters}); PPO 5 epochs x 4 mini-batches, fp32 fused rollout inference, graphed update (at "
                    "world size > 1: per mini-batch step two graphs with one eager in-place all-reduce of the "
                    "flat gradient + KL mean between them); allreduce_ms = HIP events on the update's stream "
                    "around each exchange, summed per iteration"}


def regeneration_cost(device, n, interval=256, plain=32, regens=5, replays=20):
    """the interval step that regenerates the terrain (mdp/events.py:180-204) against a plain step,
    both eager from Python with a device synchronisation after each (wall time), over `regens` regenerations.  The
    next generation is built on the background thread from half-way through the interval and staged into the
    context's arrays on a side stream (gr_terrain_stage); the interval step commits it on the stream
    (gr_terrain_commit) and resets every env.  The same interval step captured in a hipGraph and replayed, against
    a captured step + full reset + observation.  The build's own duration (host, in the background) beside it."""
    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device=device), stage=1,
                       terrain=TerrainCfg(num_gates=8, obstacles=True, regen_interval_s=0.03 * interval))
    env = RacingEnv(cfg)
    env.reset()
    g = torch.Generator(device=device).manual_seed(5)
    acts = torch.randn(8, n, 4, device=device, generator=g)

    def to_phase(ph):  # eager steps until the step counter is at phase ph of the interval
        k = 0
        while env.common_step_counter % env._regen_steps != ph:
            env.step(acts[k % 8])
            k += 1

    def wait_build():
        t0 = time.perf_counter()
        if env._next_terrain is not None:
            env._next_terrain.result()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    times, t_regen, build_wait = [], [], 0.0
    for r in range(regens):
        # plain steps between the wait for the build and the interval step (timed): the GPU idled while the host
        # waited, and its first launches after an idle second run at lowered clocks
        to_phase(interval - 1 - plain)
        build_wait += wait_build()
        for k in range(plain):
            t0 = time.perf_counter()
            env.step(acts[k % 8])
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        assert env.common_step_counter % env._regen_steps == env._regen_steps - 1
        t0 = time.perf_counter()
        _, _, _, _, extras = env.step(acts[0])
        torch.cuda.synchronize()
        t_regen.append(time.perf_counter() - t0)
        assert extras.get("terrain_regenerated") and env.terrain_generation == r + 1
    t0 = time.perf_counter()
    env._build_terrain(env._terrain_seed(regens + 1))
    t_build = time.perf_counter() - t0
    # what the event implies besides the new tables (mdp/events.py:180-204 calls env.reset() of every env): a plain
    # step followed by a full reset and an observation pass, the same way (eager, synchronised)
    times_sr = []
    for k in range(8):
        t0 = time.perf_counter()
        env.step(acts[k % 8])
        env.reset()
        env.observe()
        torch.cuda.synchronize()
        times_sr.append(time.perf_counter() - t0)

    # captured: the interval step as one graph, replayed (each replay: step, commit, reset, observe)
    def replay_us(graph):
        graph.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(replays):
            t0 = time.perf_counter()
            graph.replay()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e6

    to_phase(interval - 1 - plain)
    wait_build()
    for k in range(plain):
        env.step(acts[k % 8])
    a_buf = acts[1].clone()
    g_regen = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_regen):
        env.step(a_buf)
    g_regen_us = replay_us(g_regen)
    g_sr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_sr):
        env.step(a_buf)
        env.reset()
        env.observe()
    g_sr_us = replay_us(g_sr)
    g_plain = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g_plain):
        env.step(a_buf)
    g_plain_us = replay_us(g_plain)
    del g_regen, g_sr, g_plain
    env.close()
    plain_us = float(np.median(times)) * 1e6
    sr_us = float(np.median(times_sr)) * 1e6
    regen_us = float(np.median(t_regen)) * 1e6
    return {"plain_step_wall_us": plain_us, "regenerating_step_wall_us": regen_us,
            "regenerating_step_wall_us_each": [t * 1e6 for t in t_regen],
            "ratio": regen_us / plain_us, "step_plus_full_reset_and_observe_wall_us": sr_us,
            "ratio_to_step_plus_full_reset": regen_us / sr_us,
            "graph": {"regenerating_step_us": g_regen_us, "step_plus_full_reset_and_observe_us": g_sr_us,
                      "plain_step_us": g_plain_us, "ratio_to_step_plus_full_reset": g_regen_us / g_sr_us},
            "background_build_s": t_build, "host_wait_for_build_s_before_timing": build_wait,
            "note": f"{n} envs, obstacle tracks; eager: env.step + synchronize per step (median of {regens} "
                    "regenerations); graph: the interval step captured once and replayed (synchronize per replay); "
                    "the build runs on a host thread from half-way through the interval, its upload into the "
                    "context's staging arrays on a side stream; the interval step commits them on the stream "
                    "(gr_terrain_commit) and resets every env (reset + observation launches)"}


def cpu_baseline(seconds: float, n: int = 65536, obstacles: bool = True):
    """The CPU oracle (C restatement of the reference step, OpenMP over envs) on a bounded sample
    of the same workload: n envs stepped for about `seconds`."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    from generalizableracing_amd.envs.tracks import build_tracks

    cfg = RacingEnvCfg(scene=SceneCfg(num_envs=n), sim=SimCfg(device="cpu"), stage=1).to_gr_config()
    gates, recs, ot = build_tracks(obstacles=obstacles)
    orc = oracle.Oracle(cfg, gates, recs, None if ot is None else ot.records, None if ot is None else ot.counts)
    orc.init()
    orc.reset(None)
    rng = np.random.default_rng(0)
    acts = rng.standard_normal((16, n, 4)).astype(np.float32)
    steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.step(acts[steps % 16])
        steps += 1
    dt = time.perf_counter() - t0
    threads = oracle.num_threads()
    return {"value": n * steps / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs x {steps} steps of the C oracle (oracle/gr_oracle.c, gcc -O2, OpenMP "
                      f"{threads} threads = OMP_NUM_THREADS), {dt:.1f} s; the Isaac-Lab/PhysX reference cannot "
                      f"run here (SURVEY §8d)"}


def load_traffic(n, gates, obstacles):
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path)).get("obstacles" if obstacles else "gates_only", {})
        if d.get("num_envs") == n and d.get("gates", 8) == gates:
            return d.get("bytes_per_launch")
    except Exception:
        return None
    return None


# the PPO gradient exchange of one mini-batch step: actor 71 172 + critic 70 401 + std 4 parameters + the KL slot
# (rsl_rl/distributed.py FlatGrads), 566 KB of fp32
GRAD_ALLREDUCE_NUMEL = 71172 + 70401 + 4 + 1


def device_identity(device) -> dict:
    """This rank's device: torch's current device index, the PCI address (so a scaling line shows one distinct GPU
    per rank) and the device name."""
    idx = torch.cuda.current_device()
    p = torch.cuda.get_device_properties(torch.device(device))
    pci = None
    if hasattr(p, "pci_bus_id"):
        pci = f"{getattr(p, 'pci_domain_id', 0):04x}:{p.pci_bus_id:02x}:{getattr(p, 'pci_device_id', 0):02x}"
    return {"current_device": idx, "pci": pci, "name": p.name, "uuid": str(getattr(p, "uuid", "")) or None}


def allreduce_latency_us(device, reps=50, warm=10) -> float:
    """Median wall latency of one in-place all_reduce of the PPO update's flat gradient buffer (566 KB fp32), each
    call synchronised, after `warm` untimed calls: what every mini-batch step of a data-parallel update pays."""
    dev = device if dist.get_backend() == "nccl" else "cpu"
    buf = torch.ones(GRAD_ALLREDUCE_NUMEL, dtype=torch.float32, device=dev)
    lat = []
    for k in range(warm + reps):
        if dev != "cpu":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_reduce(buf)
        if dev != "cpu":
            torch.cuda.synchronize()
        if k >= warm:
            lat.append((time.perf_counter() - t0) * 1e6)
    return float(np.median(lat))


def main():
    a = parse()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # a line must describe what ran: --gpus is the rank count, and with RCCL every rank owns a GPU of its own
    if a.gpus is not None and a.gpus != ws:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws} (run `python bench.py --gpus N` to launch "
                         f"N ranks, or torch.distributed.run --nproc-per-node N ... --gpus N)")
    if a.dist_backend == "nccl":
        if ws > 1 and torch.cuda.device_count() < ws:
            raise SystemExit(f"bench.py: {ws} RCCL ranks need {ws} GPUs, {torch.cuda.device_count()} visible")
    else:  # rehearsal: ranks may share a device
        local = local % max(1, torch.cuda.device_count())
    if ws > 1:
        # the scaling lines report the headline step and the data-parallel training leg (BASELINE C4: every rank
        # trains on its own shard with the gradient all-reduce live); the other extras (policy, camera, sweep, C5,
        # single-GPU training legs) are single-GPU measurements, and a rank-local leg must not hold the others at a
        # collective
        if a.legs == "all":
            a.legs = "dtrain"
        elif not set(a.legs.split(",")) <= {"dtrain", "none"}:
            raise SystemExit(f"bench.py: --legs {a.legs}: at WORLD_SIZE > 1 only the dtrain leg runs")
        torch.cuda.set_device(local)
        dist.init_process_group(a.dist_backend, rank=rank, world_size=ws)
    device = f"cuda:{local}"
    n = a.num_envs
    env = make_env(n, rank, device, a.gates, a.integrator, bool(a.obstacles))
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    actions = torch.randn(ACTION_RING, n, 4, device=device, generator=g)
    for k in range(a.warmup):
        env.step(actions[k % ACTION_RING])
    torch.cuda.synchronize()
    secs, mode, graph = time_env_steps(env, actions, a.steps, not a.no_graph)
    local_secs = secs
    secs = max_over_ranks(secs, device)
    value = n * ws * a.steps / secs
    if graph is None:  # --no-graph: the timed region ran eager, the kernel is still timed from graph replays
        graph = capture_graph(env, actions)
    kt = kernel_timing(graph)
    steady = repeat_median(graph, n)
    del graph
    us = kt["kernel_us"]
    ms_per_step = secs * 1e3 / a.steps
    # a per-launch kernel time cannot exceed the wall time per step of the same graph launches; only checked
    # for a graph-timed region on a device of its own (eager launches under a PMC profiler, or rehearsal ranks
    # sharing one GPU, interleave other work into the event window)
    shared = ws > torch.cuda.device_count()
    if mode == "hipgraph" and not shared and us > ms_per_step * 1e3:
        raise RuntimeError(f"kernel_us {us:.2f} > wall us per step {ms_per_step * 1e3:.2f}: timing is inconsistent")
    rd, wr = env.bytes_per_env_step()
    achieved = (rd + wr) * n / (us * 1e-6) / 1e9
    progress(f"headline: {value:.4g} env-steps/s, kernel {us:.2f} us")
    extra = {"steady_state_env_steps_per_s_per_gpu": steady,
             "steady_state_note": "median of 3 timed runs of 1024 steps (16 replays of the 64-step graph), one rank"}
    if ws > 1:
        # a scaling line that proves what it ran: the backend, one record per rank (its device and PCI address, its
        # own step rate over the timed region) and the latency of the update's one collective on this group
        me = {"rank": rank, **device_identity(device), "env_steps_per_s": n * a.steps / local_secs,
              "timed_region_s": local_secs}
        ranks = [None] * ws
        dist.all_gather_object(ranks, me)
        distinct = len({(r["pci"], r["uuid"], r["current_device"]) for r in ranks})
        if dist.get_backend() == "nccl" and distinct != ws:
            raise SystemExit(f"bench.py: {ws} RCCL ranks ran on {distinct} distinct devices: {ranks}")
        extra["distributed"] = {
            "world_size": ws, "backend": dist.get_backend(), "ranks": ranks,
            "distinct_devices": distinct,
            "grad_allreduce_bytes": GRAD_ALLREDUCE_NUMEL * 4,
            "grad_allreduce_median_us": allreduce_latency_us(device),
            "note": "value = world_size x envs x steps / max over ranks of the timed region; ranks[i].env_steps_per_s "
                    "is rank i's own rate"}
    if want(a, "policy"):
        rate_e, us_e, tfs_e = policy_in_loop_fused(env, 1024, device, precision="fp32", actor_only=True)
        extra["env_only_fp32"] = {
            "env_steps_per_s": rate_e,
            "launch": "hipgraph (64 x [fused fp32 actor inference 16-256-256-4 + Gaussian sample + gr_step])",
            "inference_kernel": "gr::policy_f32_kernel<256> actor only (MFMA 16x16x4 f32), every CU",
            "inference_kernel_us": us_e, "inference_TFLOPs": tfs_e,
            "inference_roofline": {"bound": "mfma", "achieved": tfs_e, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                                   "frac": tfs_e / FP32_MFMA_PEAK_TFS},
            "note": "SURVEY §8d env-only rate: gr_step + policy inference at the reference's fp32 (operands and "
                    "accumulation fp32; mean within 1e-5 of the module)"}
        progress("env_only_fp32")
        extra["env_only_fp32_torch"] = {
            "env_steps_per_s": policy_in_loop_graphed(env, 1024, device),
            "launch": "hipgraph (64 x [PyTorch fp32 actor MLP 16-256-256-4 + Gaussian sample + gr_step])",
            "note": "the same rate with the PyTorch (hipBLASLt) actor"}
        progress("env_only_fp32_torch")
        extra["policy_in_loop_env_steps_per_s"] = policy_in_loop(env, 256, device)
        progress("policy_in_loop")
        rate, us_pol, tfs = policy_in_loop_fused(env, 512, device)
        extra["policy_in_loop_fused"] = {
            "env_steps_per_s": rate, "launch": "hipgraph (64 x [fused inference + gr_step])",
            "inference_kernel": "gr::policy_kernel<256> (MFMA 16x16x32 bf16, fp32 accumulate)",
            "inference_kernel_us": us_pol, "inference_TFLOPs": tfs,
            "note": "actor+critic MLP(16-256-256-out), Gaussian sample + log prob; bf16 operands (C5)"}
        progress("policy_in_loop_fused")
        rate32, us32, tfs32 = policy_in_loop_fused(env, 512, device, precision="fp32")
        extra["policy_in_loop_fused_fp32"] = {
            "env_steps_per_s": rate32, "launch": "hipgraph (64 x [fused fp32 inference + gr_step])",
            "inference_kernel": "gr::policy_f32_kernel<256> (MFMA 16x16x4 f32: fp32 operands, the reference's "
                                "precision)",
            "inference_kernel_us": us32, "inference_TFLOPs": tfs32,
            "roofline": {"bound": "mfma", "achieved": tfs32, "peak": FP32_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": tfs32 / FP32_MFMA_PEAK_TFS},
            "note": "actor+critic MLP(16-256-256-out) in fp32 (mean / value within 1e-5 of the fp32 module), "
                    "Gaussian sample + log prob: SURVEY §8d env-only rate at the reference's precision"}
        progress("policy_in_loop_fused_fp32")
    env.close()
    if want(a, "obstacles") and not a.obstacles:
        # the reference task's terrain also carries walls / orbits / ground obstacles:
        # the same step over obstacle tracks (grid-listed collision, per-env cell hints)
        env_o = make_env(n, rank, device, a.gates, a.integrator, True)
        for k in range(a.warmup):
            env_o.step(actions[k % ACTION_RING])
        torch.cuda.synchronize()
        secs_o, mode_o, graph_o = time_env_steps(env_o, actions, a.steps, not a.no_graph)
        secs_o = max_over_ranks(secs_o, device)
        if graph_o is None:
            graph_o = capture_graph(env_o, actions)
        kt_o = kernel_timing(graph_o)
        del graph_o
        rd_o, wr_o = env_o.bytes_per_env_step()
        extra["with_obstacles"] = {
            "value": n * ws * a.steps / secs_o, "unit": "env-steps/s",
            "kernel": "gr::step_kernel<false, true, 0, 1>",
            "kernel_us": kt_o["kernel_us"], "bytes_per_env_step": {"read": rd_o, "written": wr_o},
            "achieved_GBps": (rd_o + wr_o) * n / (kt_o["kernel_us"] * 1e-6) / 1e9,
            "frac": (rd_o + wr_o) * n / (kt_o["kernel_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "read_frac": rd_o * n / (kt_o["kernel_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
            "traffic": load_traffic(n, a.gates, 1),
            "obstacles_per_track_max": int(env_o.obstacle_table.counts.max()),
            "obstacles_per_track_mean": float(env_o.obstacle_table.counts.mean())}
        progress("with_obstacles")
        env_o.close()
    if want(a, "sweep") and not a.obstacles:
        extra["env_count_sweep"] = env_count_sweep(rank, device, a)
        progress("env_count_sweep")
    if want(a, "c5") and not a.obstacles:
        # BASELINE config C5 on one GPU: 32-gate tracks, startup DR (plant vs controller mass, drag, thrust
        # error, rotor constants), hipGraph of [fused rollout inference + step]
        env_c5 = make_env(n, rank, device, 32, a.integrator, False, dr_rotor=1)
        for k in range(a.warmup):
            env_c5.step(actions[k % ACTION_RING])
        torch.cuda.synchronize()
        graph_c5 = capture_graph(env_c5, actions)
        kt_c5 = kernel_timing(graph_c5)
        del graph_c5
        # the step kernel also writing the bf16 rollout rows (gr_bind_obs_sink: the runner's storage slot)
        sink = torch.empty(2, n, 16, device=device, dtype=torch.bfloat16)
        env_c5.set_obs_sink(sink[0], sink[1])
        graph_c5s = capture_graph(env_c5, actions)
        kt_c5s = kernel_timing(graph_c5s)
        del graph_c5s
        rd_c5s, wr_c5s = env_c5.bytes_per_env_step()
        env_c5.set_obs_sink(None)
        del sink
        # C5 as specified: bf16 BUFFERS (the step writes each transition's bf16 rows into its own storage slot of a
        # 64-slot ring), the policy at the reference's fp32 (actor + critic on fp32 MFMA), hipGraph of 64 x
        # [inference + step]
        ring = torch.empty(ACTION_RING, 2, n, 16, device=device, dtype=torch.bfloat16)
        rate_c5_32, us_c5_32, tfs_c5_32 = policy_in_loop_fused(env_c5, 512, device, precision="fp32", sink_ring=ring)
        # option: the same with the bf16-operand MLP (not the reference's arithmetic)
        rate_c5, us_c5, _ = policy_in_loop_fused(env_c5, 512, device, sink_ring=ring)
        del ring
        extra["c5_32_gates"] = {"dr": "plant/controller mass, inertia, drag, thrust error, rotor constants "
                                      "(thrust map, kappa x U(0.9, 1.1))",
                                "step_kernel_us": kt_c5["kernel_us"], "step_env_steps_per_s": n / (kt_c5["kernel_us"] * 1e-6),
                                "step_plus_fused_fp32_inference_env_steps_per_s": rate_c5_32,
                                "fp32_inference_kernel": "gr::policy_f32_kernel<256>, actor + critic (MFMA 16x16x4 "
                                                         "f32: the reference's precision)",
                                "fp32_inference_kernel_us": us_c5_32, "fp32_inference_TFLOPs": tfs_c5_32,
                                "fp32_inference_frac_of_fp32_mfma_peak": tfs_c5_32 / FP32_MFMA_PEAK_TFS,
                                "option_step_plus_fused_bf16_mlp_inference_env_steps_per_s": rate_c5,
                                "option_bf16_mlp_inference_kernel_us": us_c5,
                                "launch": "hipgraph (64 x [fused inference + gr_step writing its bf16 rows into "
                                          "slot k of a 64-slot rollout ring])",
                                "step_kernel_us_bf16_obs_sink": kt_c5s["kernel_us"],
                                "bytes_per_env_step_bf16_obs_sink": {"read": rd_c5s, "written": wr_c5s},
                                "note": "C5 = bf16 obs / rollout buffers with the policy in fp32 (the headline "
                                        "C5 figure); the bf16-MLP figure is an option, not the reference's "
                                        "arithmetic"}
        env_c5.close()
        progress("c5_32_gates")
    if want(a, "regen"):
        extra["terrain_regeneration"] = regeneration_cost(device, n)
        progress("terrain_regeneration")
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    if want(a, "camera"):
        # (before the training legs: measured in the same clean state as the headline, not after 65 536-env training)
        gc.collect()
        torch.cuda.empty_cache()
        # the depth camera of the vision task (separate kernel, same env shard size)
        import bench_camera

        for key, obst in (("vision_camera", False), ("vision_camera_with_obstacles", True)):
            cam = bench_camera.run(n, steps=24, warmup=4, device=device, obstacles=obst)
            progress(key)
            extra[key] = {
                "kernel": cam["kernel"], "image": cam["image"], "render_fraction": cam["render_fraction"],
                "ms_per_call": cam["ms_avg_call"], "ms_render_call": cam["ms_render_call"],
                "ms_reuse_call": cam["ms_reuse_call"], "achieved_GBps": cam["gbs_avg"], "peak_GBps": HBM_PEAK_GBS,
                "frac": cam["hbm_frac_avg"],
                "bytes_per_env_call": [cam["bytes_per_env_render"], cam["bytes_per_env_reuse"]],
                "env_steps_per_s_step_plus_camera": cam["wall_env_steps_per_s_step_plus_camera"]}
    if want(a, "dtrain"):
        # BASELINE C4 (at world size 1 the same leg without an exchange: the per-N values the scaling run compares)
        gc.collect()
        torch.cuda.empty_cache()
        extra["distributed_train"] = train_fps_distributed(device, n, rank, ws)
    if want(a, "train4096"):
        extra["train_total_fps_4096_envs"] = train_fps(device)
        extra["train_total_fps_4096_envs_graph_update"] = train_fps(device, graph_update=True)
        # C2 with the fp32 fused rollout inference (the reference's precision) and the graphed update
        extra["train_total_fps_4096_envs_fused_fp32_graph_update"] = train_fps(device, fused=True,
                                                                                 fused_precision="fp32",
                                                                                 graph_update=True)
    if want(a, "mlp_ab"):  # the update's MLPs per layer (round 3: fused first layer / head around hipBLASLt)
        extra["train_total_fps_4096_envs_fused_fp32_graph_update_per_layer_mlp"] = train_fps(
            device, fused=True, fused_precision="fp32", graph_update=True, fused_mlp=False)
        extra["train_total_fps_65536_envs_fused_fp32_graph_update_per_layer_mlp"] = train_fps(
            device, n, fused=True, fused_precision="fp32", graph_update=True, fused_mlp=False)
    if want(a, "train65536"):
        extra["train_total_fps_65536_envs"] = {
            "fp32": train_fps(device, n),
            "fp32_fused_fp32_rollout": train_fps(device, n, fused=True, fused_precision="fp32"),
            "fp32_fused_fp32_rollout_graphed_update": train_fps(device, n, fused=True, fused_precision="fp32",
                                                                graph_update=True),
            "fused_rollout_bf16_storage": train_fps(device, n, fused=True, bf16_storage=True),
            "fused_rollout_bf16_storage_no_obs_sink": train_fps(device, n, fused=True, bf16_storage=True,
                                                                obs_sink=False),
            "fused_bf16_storage_graphed_bf16_update": train_fps(device, n, fused=True, bf16_storage=True,
                                                                graph_update=True, bf16_update=True),
            "note": "Perf/total_fps, PPO 5 epochs x 4 mini-batches per 24-step rollout, obstacle tracks; the step "
                    "kernel writes the rollout storage rows (obs sink) unless marked no_obs_sink"}
    if want(a, "vision"):
        # the reference's registered recipe end to end: depth camera + VisionActorCritic + PPOL2C2 (fused BN stem)
        import bench_vision

        vis = bench_vision.run(argparse.Namespace(envs=4096, steps=8, iters=2, storage_bf16=False, no_fused_bn=False,
                                                  graph_update=True))
        progress("vision_train")
        import time_stem12

        stem = time_stem12.roofline(24576)  # one PPO mini-batch of images: the update's stem kernels against bounds
        progress("vision_stem_roofline")
        extra["vision_train_total_fps_4096_envs"] = {
            "value": vis["train_total_fps"], "train_iter_s": vis["train_iter_s"],
            "rollout_env_steps_per_s": vis["rollout_env_steps_per_s"], "max_mem_GB": vis["max_mem_GB"],
            "graph_update": vis["graph_update"], "stem_kernels_24576_images": stem,
            "note": "Perf/total_fps of QuadcopterVisionPPORunnerCfg (VisionActorCritic 72x96 stem: fused HIP first "
                    "block + conv2, BatchNorm + LeakyReLU passes, PPOL2C2 with the update's mini-batch steps as "
                    "hipGraph replays), obstacle tracks, fp32"}
    cpu = None
    if rank == 0 and ws == 1 and want(a, "cpu"):
        cpu = cpu_baseline(a.cpu_seconds, obstacles=bool(a.obstacles))
        progress("cpu_baseline")
    traffic = load_traffic(n, a.gates, a.obstacles)
    if rank == 0:
        line = {
            "metric": "env-steps/sec whole-node @65536 envs/GPU; 1/2/4/8-GPU scaling",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": ws,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: procedural zigzag/circular/ellipse tracks (20 types x 10 levels), "
                    "N(0,1) pre-tanh actions resident in HBM",
            "config": {"workload": f"racing env step, {n} envs/GPU, TRAINING_STAGE=1, {a.gates}-gate tracks"
                                   f"{' with walls/orbits/ground obstacles' if a.obstacles else ', no obstacles'}, "
                                   f"{a.integrator} integrator (BASELINE config C3/C4)",
                       "num_envs_per_gpu": n, "launch": mode, "parallelism": f"env-shard x{ws}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "frac_definition": "(read + written algorithmic bytes) / kernel_us / 8 TB/s",
                         "read_achieved": rd * n / (us * 1e-6) / 1e9,
                         "read_frac": rd * n / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                         "read_frac_definition": "the north star's HBM-read roofline: read bytes only",
                         "kernel": ("gr::step_kernel<false, true, 0, 1>" if a.obstacles else
                                    "gr::step_kernel<true, false, 8, 1>" if a.gates <= 8 and a.integrator == "dd_explicit"
                                    else f"gr::step_kernel<true, false, {8 if a.gates <= 8 else 0}, 0>")
                                   + " (fused step)", **kt,
                         "algorithmic_bytes_per_launch": (rd + wr) * n,
                         # the measured floor: a pure coalesced stream of exactly these bytes in the same launch shape
                         # and hipGraph (tools/streambench.hip, profiles/round01_streambench.json), 65 536 envs
                         "stream_floor_us": STREAM_FLOOR_US if n == 65536 and not a.obstacles else None,
                         "frac_of_stream_floor": STREAM_FLOOR_US / us if n == 65536 and not a.obstacles else None,
                         "bytes_per_env_step": {"read": rd, "written": wr}},
            "cpu_baseline": cpu,
            # which binary ran: the sources libgr.so was built from, against this tree's (a stale build shows false)
            "libgr": {"path": _abi_mod.LIB_PATH if not os.environ.get("GR_LIB_PATH") else os.environ["GR_LIB_PATH"],
                      "source_sha256": _lib_sha(), "matches_tree": _lib_sha() == _abi_mod.tree_source_sha256()},
            **extra,
        }
        print(json.dumps(line))
    if dist.is_initialized():
        dist.destroy_process_group()


def _lib_sha():
    f = getattr(_abi_mod.load(), "gr_source_sha256", None)
    return f().decode() if f is not None else None


if __name__ == "__main__":
    main()
