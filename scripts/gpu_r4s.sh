#!/bin/bash
# Round 4: stem first-block PMC passes (where the tile pipeline's time goes) + the eager regeneration step after the
# host-path trim (regeneration tests, stamped profile, bench leg)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4s}
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
step tests_regen bash -c "timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k regeneration > $OUT/pytest_regen.log 2>&1"
step regen timeout -k 10 300 python -u scripts/prof_regen.py --out $OUT/regen.json > $OUT/regen.log 2>&1
step bench_regen bash -c "timeout -k 10 300 python -u bench.py --legs regen --steps 5 --warmup 2 > $OUT/bench_regen.json 2> $OUT/bench_regen.err"
cd /tmp && export TMPDIR=/tmp
step pmc1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc1 -o pmc -- python3 $R/scripts/time_stem1.py --reps 3
step pmc2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc2 -o pmc -- python3 $R/scripts/time_stem1.py --reps 3
echo done > $OUT/done
