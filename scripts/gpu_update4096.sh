#!/bin/bash
# GPU box: kernel trace of one training iteration at 4 096 envs (fused fp32 rollout, graphed update).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-u4096}
mkdir -p $OUT
cd $R
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- \
    python3 $R/scripts/prof_update.py --envs 4096 --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
echo done > $OUT/done
