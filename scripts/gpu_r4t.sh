#!/bin/bash
# Round 4 closing call: smoke, the whole GPU suite, the default bench line, the driver-form line, the stamped
# regeneration profile.  A failing step is recorded and the next runs, unless it timed out or crashed.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4t}
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
step smoke bash -c "timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")' > $OUT/smoke.log 2>&1"
step gpu_suite bash -c "timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1"
step bench bash -c "timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver bash -c "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs none > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step regen timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1
echo done > $OUT/done
