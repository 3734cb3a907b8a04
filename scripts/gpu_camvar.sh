#!/bin/bash
# GPU box: camera bench across build variants in build/var (GR_LIB_PATH override).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-camvar}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
timeout -k 10 200 python scripts/bench_camera.py > $OUT/base.json 2>> $OUT/err.log; rc=$?; fatal $rc && exit 11
for f in build/var/*.so; do
  n=$(basename $f .so)
  GR_LIB_PATH=$R/$f timeout -k 10 200 python scripts/bench_camera.py > $OUT/$n.json 2>> $OUT/err.log; rc=$?; fatal $rc && exit 12
done
echo done > $OUT/done
