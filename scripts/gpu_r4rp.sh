#!/bin/bash
# Round 4: where the C2 rollout step's host time goes (cProfile + synchronised pieces), fused fp32 rollout
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4rp}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/prof_rollout.py --envs 4096 --fused --out $OUT/rollout_fused.json > $OUT/rollout.log 2>&1; echo "rollout rc=$?" >> $OUT/steps.txt
echo done > $OUT/done
