#!/bin/bash
# Round 4: obstacle hit batches with mixed kinds (tree) against batches per hit branch and one slot per pass, camera legs, twice; camera tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4pc}
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
step tests bash -c "timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py tests/test_obstacles.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1"
grep -q ' passed' $OUT/tests.log && ! grep -q -E ' failed| error' $OUT/tests.log || { echo 'tests not green' >> $OUT/steps.txt; exit 1; }
for rep in 1 2; do
  for v in tree cam_obst_per_branch cam_obst_per_slot; do
    lib=""; [ $v != tree ] && lib="GR_LIB_PATH=$R/variants/$v/libgr.so"
    step cam_${v}_$rep bash -c "$lib timeout -k 10 200 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/cam_${v}_$rep.json 2>> $OUT/cam.err"
  done
done
echo done > $OUT/done
