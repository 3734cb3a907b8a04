#!/bin/bash
# GPU box: vision iteration A/B — the in-tree build, the variant libraries given, and a copy of the tree with the
# fused L2C2 mix switched off (the torch expression), alternating, twice.  Usage: time_vision_ab.sh OUT LIB...
set -o pipefail
OUT=$1; shift
R=$(pwd)
mkdir -p gpurun_out /tmp/nomix
cp -r $R/generalizableracing_amd $R/scripts /tmp/nomix/
sed -i 's/^    if fused:$/    if False:/' /tmp/nomix/generalizableracing_amd/rsl_rl/ppo_l2c2.py
grep -q "^    if False:" /tmp/nomix/generalizableracing_amd/rsl_rl/ppo_l2c2.py || exit 4
: > gpurun_out/$OUT
for rep in 1 2; do
  for lib in tree nomix "$@"; do
    dir=$R; env_lib=""
    if [ "$lib" = nomix ]; then dir=/tmp/nomix; elif [ "$lib" != tree ]; then env_lib="GR_LIB_PATH=$R/$lib"; fi
    (cd $dir && env $env_lib timeout -k 10 200 python -u scripts/prof_vision_update.py --out $R/gpurun_out/vis_tmp.json > $R/gpurun_out/vis_ab_last.log 2>&1) || exit 3
    python3 -c "import json; d=json.load(open('$R/gpurun_out/vis_tmp.json')); print('$rep', '$lib', d['iteration']['fps'], round(d['iteration']['learn_time'], 4), round(d['update_wall_s'], 4))" | tee -a gpurun_out/$OUT
  done
done
