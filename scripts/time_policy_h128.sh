#!/bin/bash
# GPU box: fused inference at hidden 128 (the reference's state cfg) for the tree lib and build/var variants.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-polh128}
mkdir -p $OUT
cd $R
for n in 65536 262144; do
  timeout -k 10 200 python scripts/bench_policy.py --envs $n --hidden 128 >> $OUT/pol.jsonl 2>> $OUT/pol.err || exit 3
  for so in build/var/libgr_*.so; do
    GR_LIB_PATH=$R/$so timeout -k 10 200 python scripts/bench_policy.py --envs $n --hidden 128 >> $OUT/pol.jsonl 2>> $OUT/pol.err || exit 4
  done
done
