#!/bin/bash
# Round 4: fused-MLP / Adam / graphed-update tests + MLP kernel trace + C2 update legs (quick A/B loop)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4g}
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_fused_mlp.py tests/test_gpu_ppo_c2_golden.py tests/test_gpu_graph_update.py \
    tests/test_gpu_units.py -k "mlp or c2 or graph or adam" > $OUT/pytest_mlp.log 2>&1 || exit 11
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/mlp -o mlp -- \
    python3 $R/scripts/time_mlp.py --reps 10 > $OUT/mlp_trace.log 2>&1) || exit 13
timeout -k 10 400 python -u bench.py --legs train4096 --steps 5 --warmup 2 > $OUT/bench_upd.json 2> $OUT/bench_upd.err || exit 14
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train4096 -o train -- \
    python3 $R/scripts/prof_update.py --envs 4096 --fused --graph --iters 2 > $OUT/train4096.log 2>&1) || exit 15
echo done > $OUT/done
