#!/bin/bash
# Round 4: regeneration stamps, fused-MLP tests + timing (double-buffered bwd fragments, new mlp_final),
# barrier-2 variant A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4i}
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1 || exit 11
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_fused_mlp.py tests/test_gpu_ppo_c2_golden.py > $OUT/pytest_mlp.log 2>&1 || exit 12
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp -o mlp -- \
    python3 $R/scripts/time_mlp.py --reps 10 > $OUT/mlp_trace.log 2>&1) || exit 13
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_camera.py > $OUT/pytest_cam.log 2>&1 || exit 15
bash scripts/gpu_cam_split.sh ${1:-r4i}_camsplit || exit 16
REPS=4 bash scripts/time_libs.sh ${1:-r4i}_b2.txt variants/barrier2_lds_only/libgr.so || exit 14
echo done > $OUT/done
