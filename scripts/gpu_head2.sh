#!/bin/bash
# GPU box: the fused-head unit tests and a kernel trace of one PPO iteration at 65 536 envs (graphed update).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-head2}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_units.py -v -k "leaky_head or mlp_fused or mlp_in or fused_ppo" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -ge 124 ] && exit 10
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- \
    python3 $R/scripts/prof_update.py --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
echo done > $OUT/done
