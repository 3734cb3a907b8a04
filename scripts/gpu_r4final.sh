#!/bin/bash
# Round 4 final evidence on one box: the default bench line, the driver-form line, the step kernel's rocprofv3 trace
# + PMC passes (scripts/gpu_profile.sh) and the env-only timeline trace, so the committed summaries and the line agree
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4final}
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
step bench bash -c "timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err"
step bench_driver bash -c "timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --legs none > $OUT/bench_driver.json 2> $OUT/bench_driver.err"
step profile bash scripts/gpu_profile.sh ${T}
step envonly_trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/envonly -o envonly -- python3 $R/bench.py --legs policy --steps 64 --warmup 8 > $OUT/envonly.log 2>&1"
echo done > $OUT/done
