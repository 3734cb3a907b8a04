#!/bin/bash
# Round 4: the fused MLP kernels' tests + the C2 golden update + the earlier new tests, then the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4b}
mkdir -p $OUT
cd $R
if [ -z "$SKIP_DONE" ]; then
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_fused_mlp.py \
  > $OUT/pytest_mlp.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_mlp.log; [ $rc -ne 0 ] && exit 10
fi
if [ -z "$SKIP_DONE" ]; then
  T1="tests/test_gpu_ppo_c2_golden.py tests/test_gpu_noise_golden.py tests/test_gpu_parity.py::test_full_size_teacher_forced_slices tests/test_gpu_parity.py::test_terrain_regeneration_matches_oracle tests/test_gpu_parity.py::test_wrapper_across_terrain_regeneration"
fi
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T1 \
  tests/test_gpu_graph_update.py tests/test_gpu_bench_multirank.py tests/test_gpu_units.py > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit 11
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 12
echo done > $OUT/done
