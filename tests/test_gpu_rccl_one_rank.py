"""The RCCL path of the data-parallel update on hardware.  Two `nccl` ranks cannot share the test box's one GPU (RCCL
refuses a duplicate device), so the N-rank code runs on a process group of one rank with the world-size > 1 paths
forced on (tests/rccl_one_rank.py): every collective an 8-GPU run issues — the parameter broadcast, the global
advantage statistics, the flat gradient + KL all-reduce between the segmented graphs of every mini-batch step, the
env's statistics reduction — goes through RCCL on the update's stream.  The same run over gloo must leave the
parameters bit-identical (a sum over one rank is the identity in both), and the update must have run segmented with
one exchange per mini-batch step (5 epochs x 4 mini-batches)."""
import json
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


def _run(backend):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_one_rank.py"), backend, str(_free_port())],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_rccl_update_on_one_rank_matches_gloo():
    nccl = _run("nccl")
    gloo = _run("gloo")
    assert nccl["backend"] == "nccl" and gloo["backend"] == "gloo"
    for out in (nccl, gloo):
        assert out["segmented"] is True and out["exchanges"] == 20 and out["finite"]
    assert nccl["param_sha256"] == gloo["param_sha256"]
