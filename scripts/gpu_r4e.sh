#!/bin/bash
# Round 4: resident-terrain tests + regeneration bench leg, fused-MLP tests + timing (wgrad staging split)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4e}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "regeneration" > $OUT/pytest_regen.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_fused_mlp.py > $OUT/pytest_mlp.log 2>&1 || exit 14
timeout -k 10 200 python -u scripts/time_mlp.py > $OUT/time_mlp.jsonl 2> $OUT/time_mlp.err || exit 12
timeout -k 10 300 python -u bench.py --legs regen --steps 5 --warmup 2 > $OUT/bench_regen.json 2> $OUT/bench_regen.err || exit 13
echo done > $OUT/done
