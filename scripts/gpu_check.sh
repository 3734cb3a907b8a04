#!/bin/bash
# GPU box: parity tests, bench, kernel-trace stats.  Usage: gpu_check.sh TAG [pytest-args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-chk}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${@:2} > $OUT/pytest_gpu.log 2>&1
echo "pytest exit $?" >> $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?" >> $OUT/bench.err; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/bench.py --no-extras --steps 512 --warmup 32 > $OUT/bench_trace.log 2>&1 || exit 4
