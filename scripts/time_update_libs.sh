#!/bin/bash
# GPU box: the update's memory-bound MLP ops (scripts/time_update_kernels.py) for the in-tree libgr.so and each variant
# library given, alternating, twice.  Usage: time_update_libs.sh OUT LIB...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$OUT
for rep in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then env_lib=""; else env_lib="GR_LIB_PATH=$lib"; fi
    env $env_lib timeout -k 10 120 python -u scripts/time_update_kernels.py ${UPD_ARGS} --out gpurun_out/$OUT > /dev/null || exit 3
  done
done
