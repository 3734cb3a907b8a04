#!/bin/bash
# GPU box: depth-camera parity tests, camera bench (+ ablations), rocprofv3 kernel trace and
# HBM PMC passes of the camera bench.  Usage: gpu_camera.sh TAG [quick].
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-cam}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
fatal() { [ "$1" -ge 124 ] && [ "$1" -ne 0 ]; }
timeout -k 10 600 python -m pytest tests/test_gpu_camera.py -x -q > $OUT/pytest_camera.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_camera.log; fatal $rc && exit 10
timeout -k 10 300 python scripts/bench_camera.py > $OUT/bench_camera.json 2> $OUT/bench_camera.err
rc=$?; fatal $rc && exit 11
timeout -k 10 300 python scripts/bench_camera.py --no-noise > $OUT/bench_camera_nonoise.json 2>> $OUT/bench_camera.err
rc=$?; fatal $rc && exit 11
[ "$2" == "quick" ] && { echo done > $OUT/done; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o cam -- python3 $R/scripts/bench_camera.py --steps 20 > $OUT/prof.log 2>&1
rc=$?; fatal $rc && exit 12
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$ctr -o pmc -- python3 $R/scripts/bench_camera.py --steps 8 --warmup 2 > $OUT/pmc_$ctr.log 2>&1
  rc=$?; fatal $rc && exit 13
done
echo done > $OUT/done
