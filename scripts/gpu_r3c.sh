#!/bin/bash
# GPU box, round 3 (third session): full GPU suite + default bench on the in-tree build, then the state-plane
# store-policy variants timed against it, then L2 hit / miss counters of the step kernel (in-tree vs plain state stores).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 || exit 10
timeout -k 10 350 python bench.py > gpurun_out/bench.log 2>&1 || exit 11
bash scripts/time_libs.sh sst.txt $R/variants/sst0/libgr.so $R/variants/sst0o2/libgr.so $R/variants/sst1o2/libgr.so || exit 12
cd /tmp && export TMPDIR=/tmp
for lib in tree sst0; do
  if [ $lib = tree ]; then unset GR_LIB_PATH; else export GR_LIB_PATH=$R/variants/$lib/libgr.so; fi
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/tcc_$lib -o pmc -- \
      python3 $R/bench.py --no-extras --no-graph --steps 64 --warmup 8 > $R/gpurun_out/tcc_$lib.log 2>&1 || exit 13
done
unset GR_LIB_PATH
echo done > $R/gpurun_out/r3c_done
