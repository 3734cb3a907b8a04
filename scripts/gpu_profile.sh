#!/bin/bash
# Profiling pass on the GPU box: kernel trace + stats of the bench, then PMC
# counters in separate passes (HBM bytes per launch: FETCH_SIZE, WRITE_SIZE;
# SQ instruction / wait mix).  Outputs under gpurun_out/prof_<tag>/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
N=${2:-65536}
OBST=${3:-0}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { echo "== $*" >> $OUT/cmds.txt; "$@"; }
run timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/bench.py --no-extras --steps 512 --warmup 32 --num-envs $N --obstacles $OBST > $OUT/bench_trace.log 2>&1 || exit 11
for ctr in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT"; do
  name=$(echo $ctr | tr ' ' '_' | cut -c1-40)
  run timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_$name -o pmc -- \
      python3 $R/bench.py --no-extras --no-graph --steps 64 --warmup 8 --num-envs $N --obstacles $OBST > $OUT/bench_$name.log 2>&1 || exit 12
done
echo done >> $OUT/cmds.txt
