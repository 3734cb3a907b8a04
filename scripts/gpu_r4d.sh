#!/bin/bash
# Round 4: per-kernel split of the fused MLP update (rocprofv3 over scripts/time_mlp.py) + the regeneration breakdown.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4d}
mkdir -p $OUT
cd $R
timeout -k 10 200 python -u scripts/time_mlp.py > $OUT/time_mlp.jsonl 2> $OUT/time_mlp.err || exit 11
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp -o mlp -- \
    python3 $R/scripts/time_mlp.py --reps 10 > $OUT/mlp_trace.log 2>&1) || exit 12
timeout -k 10 300 python -u scripts/prof_regen.py > $OUT/regen.json 2> $OUT/regen.err || exit 13
echo done > $OUT/done
