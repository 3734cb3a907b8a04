#!/bin/bash
# GPU box: the vision recipe's training iteration (scripts/prof_vision_update.py) for the in-tree libgr.so and each
# variant library given, alternating, twice.  Usage: time_vision_libs.sh OUT LIB...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > gpurun_out/$OUT
for rep in 1 2; do
  for lib in tree "$@"; do
    if [ "$lib" = tree ]; then env_lib=""; else env_lib="GR_LIB_PATH=$lib"; fi
    env $env_lib timeout -k 10 200 python -u scripts/prof_vision_update.py --out gpurun_out/vis_tmp.json > /dev/null 2>&1 || exit 3
    python3 -c "import json; d=json.load(open('gpurun_out/vis_tmp.json')); print('$rep', '$lib', d['iteration']['fps'], round(d['iteration']['learn_time'], 4), round(d['update_wall_s'], 4))" | tee -a gpurun_out/$OUT
  done
done
