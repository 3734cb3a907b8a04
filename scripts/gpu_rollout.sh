#!/bin/bash
# GPU box: the rollout-bookkeeping and optimizer tests, the rollout-loop breakdown (scripts/prof_rollout.py) at 4 096
# envs (torch and fused fp32 inference) and 65 536, then the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-rollout}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_rollout_ops.py tests/test_gpu_units.py tests/test_gpu_graph_update.py \
    tests/test_gpu_ppo_c2_golden.py tests/test_gpu_train_cli.py -v -k "rollout or adam or graph or c2 or train or store or gae or episode or act_draw or combined or leaky or mlp or fused_ppo" \
    --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $OUT/pytest.log; [ $rc -ge 124 ] && exit 10
timeout -k 10 240 python -u scripts/prof_rollout.py --envs 4096 --out $OUT/r4096.json > $OUT/r4096.log 2>&1 || exit 11
timeout -k 10 240 python -u scripts/prof_rollout.py --envs 4096 --fused --out $OUT/r4096f.json > $OUT/r4096f.log 2>&1 || exit 12
timeout -k 10 240 python -u scripts/prof_rollout.py --envs 65536 --fused --out $OUT/r65536f.json > $OUT/r65536f.log 2>&1 || exit 13
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/update -o update -- python3 $R/scripts/prof_update.py --envs 4096 --fused --graph --iters 2 > $OUT/update.log 2>&1) || exit 16
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 17
echo done > $OUT/done
