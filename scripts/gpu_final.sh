#!/bin/bash
# GPU box, round-end rehearsal: the whole GPU test suite, smoke(), the default bench line and the driver-style
# short line (--steps 20 --warmup 5).  Usage: gpu_final.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-final}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest_gpu.log; [ $rc -ge 124 ] && exit 10
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 12
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench_steps20.json 2> $OUT/bench_steps20.err || exit 13
echo done > $OUT/done
