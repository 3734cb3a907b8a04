"""bench.py's multi-rank path (the driver's N = 2, 4, 8 scaling runs launch it under torch.distributed.run):
two ranks share the one GPU of the test box over gloo, and rank 0 prints one JSON line whose value counts
both shards.  The RCCL path differs only in the backend and one GPU per rank."""
import json
import math
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


BENCH_ARGS = ["--gpus", "2", "--steps", "128", "--warmup", "8", "--num-envs", "8192", "--dist-backend", "gloo"]


@pytest.mark.parametrize("launch", ["torchrun", "plain"])
def test_bench_two_ranks_gloo(launch):
    """torchrun: the driver's form for N > 1.  plain: `python bench.py --gpus 2`, which starts the two ranks itself
    (bench.launch_ranks) and must print the same two-rank line."""
    bench = os.path.join(ROOT, "bench.py")
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), bench, *BENCH_ARGS]
    else:
        cmd = [sys.executable, bench, *BENCH_ARGS]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    assert line["config"]["parallelism"] == "env-shard x2"
    # the value counts both shards: 2 x 8192 envs x steps / max-over-ranks time
    assert abs(line["value"] - 2 * 8192 * 128 / (line["ms_per_step"] * 1e-3 * 128)) < 1e-6 * line["value"]
    assert line["cpu_baseline"] is None and "policy_in_loop_fused" not in line
    # the line proves what ran: backend, per-rank device and rate, the update collective's latency on this group
    d = line["distributed"]
    assert d["world_size"] == 2 and d["backend"] == "gloo"
    assert [r["rank"] for r in d["ranks"]] == [0, 1]
    for r in d["ranks"]:
        assert r["current_device"] == 0 and r["env_steps_per_s"] > 0 and "pci" in r and r["name"]
        assert r["env_steps_per_s"] >= 8192 * 128 / (line["ms_per_step"] * 1e-3 * 128) * (1 - 1e-6)
    assert d["grad_allreduce_bytes"] == 566_312 and d["grad_allreduce_median_us"] > 0
    assert len(d["ranks"]) == 2
    # BASELINE C4: the training leg ran on both ranks with the gradient exchange on the update's critical path
    t = line["distributed_train"]
    assert t["world_size"] == 2 and t["num_envs_per_rank"] == 8192
    assert math.isfinite(t["train_total_fps"]) and t["train_total_fps"] > 0
    assert [r["rank"] for r in t["ranks"]] == [0, 1]
    for r in t["ranks"]:
        # 5 epochs x 4 mini-batches, one in-place all-reduce of the flat gradient + KL mean each
        assert r["allreduces_per_iteration"] == 20
        assert 0 < r["allreduce_ms_per_iteration"] < r["update_ms"]
        assert math.isfinite(r["iteration_s"]) and r["iteration_s"] > 0
    # a data-parallel update leaves every rank's parameters bit-identical
    assert t["params_identical_on_all_ranks"] is True
    assert len({r["param_sha256"] for r in t["ranks"]}) == 1


def test_bench_refuses_a_world_it_cannot_describe():
    """Two RCCL ranks on a one-GPU box: every rank must own a GPU, so the run exits non-zero without a line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    import torch

    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "8",
                        "--num-envs", "8192", "--no-extras"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "need" in r.stderr
