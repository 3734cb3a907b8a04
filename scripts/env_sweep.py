"""bench.py's env_count_sweep alone (per-launch us, env-steps/s, GB/s at 16 384 / 262 144 / 1 048 576 envs).

    python scripts/env_sweep.py [--obstacles 1]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

if __name__ == "__main__":
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    a = bench.parse()
    print(json.dumps(bench.env_count_sweep(0, "cuda:0", a), indent=1))
