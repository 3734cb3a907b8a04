#!/bin/bash
# Round 4: obstacle hits in inverse depth (one division per hit) — camera tests bit-exact vs the oracle, camera bench legs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4l}
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
step tests bash -c "timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_camera.py > $OUT/pytest.log 2>&1"
step bench_cam bash -c "timeout -k 10 300 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/bench_cam.json 2> $OUT/bench_cam.err"
step bench_cam2 bash -c "timeout -k 10 300 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/bench_cam2.json 2> $OUT/bench_cam2.err"
echo done > $OUT/done
