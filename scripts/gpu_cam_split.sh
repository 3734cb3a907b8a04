#!/bin/bash
# camera kernel: render / reuse ms with and without the policy-image noise, gate-only and obstacle tracks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-camsplit}
mkdir -p $OUT
cd $R
for args in "" "--no-noise" "--gates-only" "--gates-only --no-noise"; do
  timeout -k 10 120 python -u scripts/bench_camera.py --steps 16 --warmup 4 $args >> $OUT/split.jsonl 2>> $OUT/split.err || exit 11
done
echo done > $OUT/done
