#!/bin/bash
# Round 4 profiles: kernel traces of the C2 and 65 536-env training iterations (fused MLP update) and the headline
# step kernel's trace + PMC passes (scripts/gpu_profile.sh).  Usage: gpu_r4c.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train4096 -o train -- \
    python3 $R/scripts/prof_update.py --envs 4096 --fused --graph --iters 2 > $OUT/train4096.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train65536 -o train -- \
    python3 $R/scripts/prof_update.py --envs 65536 --fused --graph --iters 1 > $OUT/train65536.log 2>&1 || exit 12
cd $R && bash scripts/gpu_profile.sh $TAG 65536 0 || exit 13
echo done > $OUT/done
