#!/bin/bash
# GPU box: camera parity (tree + variant libraries) and camera A/B timings.  Usage: gpu_cam3.sh TAG [variant libs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cam3}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_camera.py -v --timeout 300 --timeout-method thread > $OUT/cam_parity_tree.log 2>&1
rc=$?; echo "exit $rc" >> $OUT/cam_parity_tree.log; [ $rc -ne 0 ] && exit 10
for so in "$@"; do
  n=$(basename $(dirname $so))
  GR_LIB_PATH=$R/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -q -k "not runner" --timeout 240 --timeout-method thread > $OUT/cam_parity_$n.log 2>&1
  rc=$?; echo "exit $rc" >> $OUT/cam_parity_$n.log; [ $rc -ge 124 ] && exit 12
done
OUT=$TAG bash scripts/ab_camera_libs.sh "$@" || exit 13
echo done > $OUT/done
