#!/bin/bash
# Round 4: regeneration breakdown + bench leg, camera counter pass, the round-3 timing variants re-timed
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4h}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1 || exit 11
timeout -k 10 300 python -u bench.py --legs regen --steps 5 --warmup 2 > $OUT/bench_regen.json 2> $OUT/bench_regen.err || exit 12
bash scripts/prof_camera_valu.sh ${1:-r4h}_cam || exit 13
REPS=2 bash scripts/time_libs.sh ${1:-r4h}_variants.txt variants/l2table_gates/libgr.so variants/barrier2_lds_only/libgr.so \
    variants/state_plain_obs_nt/libgr.so variants/state_plain_obs_sc1/libgr.so variants/state_nt_obs_sc1/libgr.so || exit 14
echo done > $OUT/done
