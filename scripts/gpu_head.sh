#!/bin/bash
# GPU box: the fused-head tests, the PPO pins that run through it, and the update timings.  Usage: gpu_head.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-head}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_ppo_c2_golden.py tests/test_gpu_graph_update.py tests/test_gpu_graph_update_dp.py tests/test_gpu_parity.py -v -k "leaky_head or mlp_fused or mlp_in or column_sum or fused_ppo or c2 or graph or runner" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -ge 124 ] && exit 10
timeout -k 10 400 python -u -c "
import json, sys
sys.argv = ['bench.py']
import bench
d = 'cuda:0'
out = {'4096_graphed': bench.train_fps(d, graph_update=True), '65536_fp32_fused_graphed': bench.train_fps(d, 65536, fused=True, fused_precision='fp32', graph_update=True), '65536_fp32': bench.train_fps(d, 65536)}
print(json.dumps(out))
" > $OUT/train.json 2> $OUT/train.err || exit 11
echo done > $OUT/done
