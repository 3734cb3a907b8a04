"""bench.py's rank launcher and its refusals, on the CPU (no GPU is touched: every case exits before a device is).

`python bench.py --gpus N` (N > 1) starts torch.distributed.run with N ranks as a child process; a rank whose world
does not match --gpus, or RCCL ranks without a GPU each, exit non-zero and print no JSON line."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def _run(args, **kw):
    return subprocess.run([sys.executable, BENCH, *args], cwd=ROOT, env=_env(**kw), capture_output=True, text=True,
                          timeout=300)


def test_plain_gpus_2_launches_two_ranks_and_relays_their_failure():
    # no GPU here: the launcher starts torch.distributed.run with two ranks, each refuses RCCL without a GPU of its
    # own, and the parent returns the child's non-zero status
    r = _run(["--gpus", "2", "--steps", "4", "--num-envs", "512", "--no-extras"])
    assert r.returncode != 0
    assert "launching 2 ranks" in r.stderr and "torch.distributed.run" in r.stderr
    assert "2 RCCL ranks need 2 GPUs" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "3", "--steps", "4", "--num-envs", "512", "--no-extras", "--dist-backend", "gloo"],
             WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "--gpus 3 but WORLD_SIZE=2" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_launcher_is_a_no_op_for_one_gpu_and_inside_a_rank():
    sys.path.insert(0, ROOT)
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)  # __name__ != "__main__": nothing launches at import
    assert mod.launch_ranks(["--gpus", "1"]) is None
    assert mod.launch_ranks([]) is None
    os.environ["WORLD_SIZE"] = "2"
    try:
        assert mod.launch_ranks(["--gpus", "2"]) is None
    finally:
        del os.environ["WORLD_SIZE"]
