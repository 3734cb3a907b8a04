#!/bin/bash
# GPU box: kernel trace + SQ counters of the fused policy inference (scripts/bench_policy.py).
# Usage: prof_policy.sh TAG [bench_policy.py args, e.g. --precision fp32]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-profpol}
shift
ARGS="$@"
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/scripts/bench_policy.py $ARGS > $OUT/trace.log 2>&1 || exit 11
i=0
for ctr in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc$i -o pmc -- \
      python3 $R/scripts/bench_policy.py $ARGS > $OUT/pmc$i.log 2>&1 || exit 12
done
echo done > $OUT/done
