#!/bin/bash
# GPU box: scripts/bench_policy.py for the in-tree libgr.so and each variant library given (GR_LIB_PATH),
# alternating, twice.  Usage: time_policy_libs.sh OUT LIB... (bench_policy args in POL_ARGS)
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$OUT
for rep in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then env_lib=""; else env_lib="GR_LIB_PATH=$lib"; fi
    env $env_lib timeout -k 10 200 python -u scripts/bench_policy.py ${POL_ARGS} 2>/dev/null | tail -1 >> gpurun_out/$OUT || exit 3
  done
done
