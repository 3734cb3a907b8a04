#!/bin/bash
# GPU box: Perf/total_fps of PPO training at 65 536 and 4 096 envs under the opt-in training modes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tm}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u - > $OUT/fps.json 2> $OUT/err <<'PY'
import json, sys
sys.path.insert(0, ".")
import bench
out = {}
for n in (65536, 4096):
    out[str(n)] = {
        "fp32": bench.train_fps("cuda:0", n),
        "bf16_update": bench.train_fps("cuda:0", n, bf16_update=True),
        "fused_bf16storage_bf16update": bench.train_fps("cuda:0", n, fused=True, bf16_storage=True, bf16_update=True),
        "all_incl_graph": bench.train_fps("cuda:0", n, fused=True, bf16_storage=True, bf16_update=True, graph_update=True),
    }
    print(json.dumps(out), flush=True)
PY
