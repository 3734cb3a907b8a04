#!/bin/bash
# Round 4 final call: smoke, the whole GPU suite, the default bench line, and the step kernel's rocprofv3 trace +
# PMC passes (scripts/gpu_profile.sh).  A failing step is recorded and the next runs, unless it timed out or
# crashed (124 / 137 / 134 / 139): then nothing more touches the GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4z}
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
step stem_time bash -c "timeout -k 10 120 python -u scripts/time_stem1.py > $OUT/time_stem1.jsonl 2> $OUT/time_stem1.err"
step stem_trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stem -o stem -- python3 $R/scripts/time_stem1.py --reps 10 > $OUT/stem_trace.log 2>&1"
step envonly_trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/envonly -o envonly -- python3 $R/bench.py --legs policy --steps 64 --warmup 8 > $OUT/envonly.log 2>&1"
step profile bash scripts/gpu_profile.sh ${T}
echo done > $OUT/done
