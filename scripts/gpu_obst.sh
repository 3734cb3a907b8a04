#!/bin/bash
# GPU box: parity tests (all), then the bench with and without obstacles.  Usage: gpu_obst.sh TAG [pytest-args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-obst}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${@:2} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log
[ $rc -ge 124 ] && exit 10
timeout -k 10 300 python bench.py --no-extras --obstacles 1 > $OUT/bench_obst.json 2> $OUT/bench_obst.err || exit 11
timeout -k 10 300 python bench.py --no-extras --obstacles 0 > $OUT/bench_noobst.json 2> $OUT/bench_noobst.err || exit 12
echo done > $OUT/done
