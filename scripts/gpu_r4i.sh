#!/bin/bash
# Round 4 combined call: regeneration stamps, fused-MLP / camera tests, MLP trace, camera split, barrier-2 A/B,
# the whole GPU suite and the bench.  A failing step is recorded and the next runs, unless the step timed out
# or crashed (124 / 137 / 134 / 139): then nothing more touches the GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4i}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc" >> $OUT/steps.txt
  case $rc in 124|137|134|139) echo "stop after $name" >> $OUT/steps.txt; exit $rc;; esac
  return 0
}
step regen timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1
step mlp_tests bash -c "timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused_mlp.py tests/test_gpu_ppo_c2_golden.py tests/test_gpu_camera.py > $OUT/pytest_mlp_cam.log 2>&1"
step mlp_trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp -o mlp -- python3 $R/scripts/time_mlp.py --reps 10 > $OUT/mlp_trace.log 2>&1"
step mlp_wgrad512 bash -c "GR_LIB_PATH=$R/variants/wgrad_512/libgr.so timeout -k 10 200 python -u scripts/time_mlp.py > $OUT/time_mlp_wgrad512.jsonl 2>&1 && timeout -k 10 200 python -u scripts/time_mlp.py > $OUT/time_mlp_tree.jsonl 2>&1"
step camsplit bash scripts/gpu_cam_split.sh ${T}_camsplit
step b2 env REPS=4 bash scripts/time_libs.sh ${T}_b2.txt variants/barrier2_lds_only/libgr.so
step gpu_suite bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1"
step bench bash -c "timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err"
echo done > $OUT/done
