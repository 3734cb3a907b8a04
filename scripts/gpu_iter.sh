#!/bin/bash
# GPU box iteration: parity tests, stamps timeline, variant timings, bench line.
# Usage: gpu_iter.sh TAG [pytest-args].  Stops at the first crash / timeout of a GPU step
# (assertion failures in pytest are reported and the remaining steps still run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-iter}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
timeout -k 10 120 build/mathbench > $OUT/mathbench.txt 2>&1; rc=$?; fatal $rc && exit 9
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${@:2} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log; fatal $rc && exit 10
timeout -k 10 300 python scripts/stamps.py run > $OUT/stamps.log 2>&1
rc=$?; fatal $rc && exit 11
timeout -k 10 600 python scripts/ablate.py run > $OUT/ablate.log 2>&1
rc=$?; fatal $rc && exit 12
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; fatal $rc && exit 13
echo done > $OUT/done
