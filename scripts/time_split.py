"""TallLinear's SPLIT (rows per weight-gradient chunk, rsl_rl/linear.py) against the graph-captured fp32 update with the
fused fp32 rollout (bench train_fps) at 4 096 (C2) and 65 536 envs.  Usage: python scripts/time_split.py SPLIT..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from generalizableracing_amd.rsl_rl import linear  # noqa: E402

out = []
for rep in range(2):
    for split in [int(v) for v in sys.argv[1:]]:
        linear.SPLIT = split
        for n in (4096, 65536):
            r = bench.train_fps("cuda:0", n, iters=3, fused=True, fused_precision="fp32", graph_update=True)
            out.append({"rep": rep, "split": split, "n": n, **r})
            print(json.dumps(out[-1]), flush=True)
