#!/bin/bash
# GPU box: kernel trace + one SQ counter pass of the camera bench (obstacle tracks, 65 536 envs): the
# instruction mix of the re-render and reuse calls.  Usage: prof_camera_valu.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-camvalu}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- \
    python3 $R/scripts/bench_camera.py --steps 8 --warmup 2 > $OUT/trace.log 2>&1 || exit 11
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    --output-format csv -d $OUT/pmc1 -o pmc -- python3 $R/scripts/bench_camera.py --steps 8 --warmup 2 > $OUT/pmc1.log 2>&1 || exit 12
echo done > $OUT/done
