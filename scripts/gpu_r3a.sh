#!/bin/bash
# GPU box: the whole GPU test suite, the default bench line (with extras), then camera variants (parity + timing).
# Usage: gpu_r3a.sh TAG [variant libs...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3a}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log; [ $rc -ge 124 ] && exit 10
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 11
for so in "$@"; do
  GR_LIB_PATH=$R/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -q --timeout 240 --timeout-method thread > $OUT/cam_parity_$(basename $(dirname $so)).log 2>&1
  rc=$?; echo "exit $rc" >> $OUT/cam_parity_$(basename $(dirname $so)).log; [ $rc -ge 124 ] && exit 12
done
[ $# -gt 0 ] && { OUT=$TAG bash scripts/ab_camera_libs.sh "$@" || exit 13; }
echo done > $OUT/done
