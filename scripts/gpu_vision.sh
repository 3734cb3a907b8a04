#!/bin/bash
# GPU box: vision task benches (env step, rollout step, training iteration) at several sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-vision}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
timeout -k 10 400 python scripts/bench_vision.py --envs 4096 --iters 2 > $OUT/v4096.json 2> $OUT/v4096.err; rc=$?; fatal $rc && exit 11
timeout -k 10 400 python scripts/bench_vision.py --envs 16384 --iters 1 > $OUT/v16384.json 2> $OUT/v16384.err; rc=$?; fatal $rc && exit 12
timeout -k 10 400 python scripts/bench_vision.py --envs 65536 --iters 0 > $OUT/v65536.json 2> $OUT/v65536.err; rc=$?; fatal $rc && exit 13
echo done > $OUT/done
