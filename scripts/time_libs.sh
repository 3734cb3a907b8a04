#!/bin/bash
# GPU box: headline step-kernel timing (bench.py --no-extras) for the in-tree libgr.so and each variant
# library given (GR_LIB_PATH), alternating, twice.  Usage: time_libs.sh OUT LIB...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$OUT
for rep in $(seq 1 ${REPS:-2}); do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then env_lib=""; else env_lib="GR_LIB_PATH=$lib"; fi
    line=$(env $env_lib timeout -k 10 120 python -u bench.py --no-extras --steps 1024 --warmup 64 ${BENCH_ARGS} 2>/dev/null | tail -1) || exit 3
    us=$(echo "$line" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['roofline']['kernel_us'],3), round(d['value']/1e9,3))")
    echo "$rep $lib $us" | tee -a gpurun_out/$OUT
  done
done
