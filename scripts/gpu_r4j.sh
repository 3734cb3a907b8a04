#!/bin/bash
# Round 4: regeneration after the pinned pool, regen + MLP + camera tests, MLP trace, regen bench leg
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4j}
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
step tests_regen bash -c "timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k regeneration > $OUT/pytest_regen.log 2>&1"
step tests bash -c "timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_fused_mlp.py tests/test_gpu_camera.py tests/test_gpu_ppo_c2_golden.py > $OUT/pytest.log 2>&1"
step regen timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1
step bench_regen bash -c "timeout -k 10 300 python -u bench.py --legs regen,camera --steps 5 --warmup 2 > $OUT/bench_regen.json 2> $OUT/bench_regen.err"
step mlp_trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp -o mlp -- python3 $R/scripts/time_mlp.py --reps 10 > $OUT/mlp_trace.log 2>&1"
echo done > $OUT/done
