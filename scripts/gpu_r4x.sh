#!/bin/bash
# Round 4: stem backward passes with the gradient rows prefetched one tile group ahead — tests, timing and vision A/B against the build without it, trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4x}
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
step tests bash -c "timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_stem1.py tests/test_gpu_fused_bn.py > $OUT/pytest.log 2>&1"
for rep in 1 2; do
  for v in tree stem_noprefetch; do
    lib=""; [ $v != tree ] && lib="GR_LIB_PATH=$R/variants/$v/libgr.so"
    step time_${v}_$rep bash -c "$lib timeout -k 10 120 python -u scripts/time_stem1.py >> $OUT/time_stem1.jsonl 2>> $OUT/time_stem1.err"
  done
done
step trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stem -o stem -- python3 $R/scripts/time_stem1.py --reps 10 > $OUT/stem_trace.log 2>&1"
step vis_ab bash -c "timeout -k 10 1000 bash scripts/time_vision_ab.sh $T/vis_ab.txt variants/stem_noprefetch/libgr.so > $OUT/vis_ab.log 2>&1"
echo done > $OUT/done
