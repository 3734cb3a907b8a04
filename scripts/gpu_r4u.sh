#!/bin/bash
# Round 4: where the obstacle re-render goes — camera legs of the tree against timing builds without the obstacle
# hit passes (cam_no_obst_pass) and without any obstacle work (cam_no_obst), alternating, twice
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4u}
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
  for v in tree cam_no_obst_pass cam_no_obst; do
    lib=""; [ $v != tree ] && lib="GR_LIB_PATH=$R/variants/$v/libgr.so"
    step cam_${v}_$rep bash -c "$lib timeout -k 10 200 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/cam_${v}_$rep.json 2>> $OUT/cam.err"
  done
done
echo done > $OUT/done
