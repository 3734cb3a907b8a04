#!/bin/bash
# GPU box: scripts/bench_policy.py at 65 536 and 262 144 envs for the in-tree libgr.so and every
# build/var/libgr_*.so (scripts/build_variants.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-polvar}
mkdir -p $OUT
cd $R
for n in 65536 262144; do
  timeout -k 10 200 python scripts/bench_policy.py --envs $n >> $OUT/pol.jsonl 2>> $OUT/pol.err || exit 3
  for so in build/var/libgr_*.so; do
    GR_LIB_PATH=$R/$so timeout -k 10 200 python scripts/bench_policy.py --envs $n >> $OUT/pol.jsonl 2>> $OUT/pol.err || exit 4
  done
done
