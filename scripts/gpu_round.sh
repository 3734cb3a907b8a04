#!/bin/bash
# GPU box, one call: parity tests, the default bench line, kernel-trace + PMC profiles of the step kernel
# on gate-only and obstacle tracks, kernel trace + SQ counters of the fused policy inference.  Usage: gpu_round.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-round}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log; fatal $rc && exit 10
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err; rc=$?; fatal $rc && exit 11
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err; rc=$?; fatal $rc && exit 11
bash scripts/gpu_profile.sh ${TAG}_g 65536 0 || exit 12
bash scripts/gpu_profile.sh ${TAG}_o 65536 1 || exit 13
bash scripts/prof_policy.sh ${TAG}_p || exit 14
bash scripts/prof_policy.sh ${TAG}_p32 --precision fp32 || exit 15
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- \
    python3 $R/scripts/prof_update.py --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
echo done > $OUT/done
