#!/bin/bash
# Round 4: env calls through the raw current-stream accessor — the whole GPU suite, smoke, the regeneration profile and
# bench leg, the default bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4zz}
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
step regen timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1
step bench bash -c "timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err"
echo done > $OUT/done
