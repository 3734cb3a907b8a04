#!/bin/bash
# GPU box: FlatAdam unit tests, the update tests it touches, a kernel trace of one graphed PPO update at 65 536
# envs, and the bench's train legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-adam}
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_graph_update.py tests/test_gpu_graph_update_dp.py \
    tests/test_gpu_ppo_c2_golden.py -v -k "adam or graph or c2 or fused_ppo" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -ge 124 ] && exit 10
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- \
    python3 $R/scripts/prof_update.py --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 17
echo done > $OUT/done
