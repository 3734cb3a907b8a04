#!/bin/bash
# GPU box: the graphed PPO update's parity test, then Perf/total_fps eager vs graphed (C2 and 65 536 envs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-gu}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_graph_update.py > $OUT/log 2>&1 || exit 3
timeout -k 10 400 python -u - > $OUT/fps.json 2> $OUT/err <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
out = {"c2": bench.train_fps("cuda:0"), "c2_graph": bench.train_fps("cuda:0", graph_update=True),
       "65536": bench.train_fps("cuda:0", 65536), "65536_graph": bench.train_fps("cuda:0", 65536, graph_update=True)}
print(json.dumps(out))
PY
