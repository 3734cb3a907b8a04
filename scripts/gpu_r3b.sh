#!/bin/bash
# GPU box, one call: the default bench line and the driver's (--steps 20 --warmup 5), kernel-trace + PMC profiles
# of the step kernel (gate-only and obstacle tracks), the camera (trace + SQ pass) and one PPO iteration at 65 536
# envs (graphed update).  Usage: gpu_r3b.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3b}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 11
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err || exit 11
bash scripts/gpu_profile.sh ${TAG}_g 65536 0 || exit 12
bash scripts/gpu_profile.sh ${TAG}_o 65536 1 || exit 13
bash scripts/prof_camera_valu.sh ${TAG}_cam || exit 14
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- \
    python3 $R/scripts/prof_update.py --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
echo done > $OUT/done
