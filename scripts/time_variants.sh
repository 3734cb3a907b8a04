#!/bin/bash
# GPU box: bench line of every build/var/libgr_*.so (and the in-tree libgr.so as "tree").
# Usage: time_variants.sh TAG [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-var}
mkdir -p $OUT
cd $R
timeout -k 10 200 python bench.py --no-extras --steps 512 ${@:2} > $OUT/tree.json 2> $OUT/tree.err || exit 3
for so in build/var/libgr_*.so; do
  n=$(basename $so .so); n=${n#libgr_}
  GR_LIB_PATH=$R/$so timeout -k 10 200 python bench.py --no-extras --steps 512 ${@:2} > $OUT/$n.json 2> $OUT/$n.err || exit 4
done
echo done > $OUT/done
