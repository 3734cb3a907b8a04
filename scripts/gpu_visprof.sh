#!/bin/bash
# GPU box: kernel trace of the vision recipe's training (4 096 envs, 2 iterations).  Usage: gpu_visprof.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-visprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/scripts/bench_vision.py --envs 4096 --iters 2 --steps 8 > $OUT/trace.log 2>&1 || exit 11
echo done > $OUT/done
