#!/bin/bash
# Round 4: the tile masks without the frustum-plane cull (obstacles; gates) against the tree, camera legs, twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4y}
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
for rep in 1 2; do
  for v in tree cam_no_obst_planecull cam_no_gate_planecull; do
    lib=""; [ $v != tree ] && lib="GR_LIB_PATH=$R/variants/$v/libgr.so"
    step cam_${v}_$rep bash -c "$lib timeout -k 10 200 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/cam_${v}_$rep.json 2>> $OUT/cam.err"
  done
done
echo done > $OUT/done
