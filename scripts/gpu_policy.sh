set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/pol4; mkdir -p $O
timeout -k 10 180 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fused_inference.py > $O/test.log 2>&1 || exit 5
for n in 16384 65536 262144; do timeout -k 10 120 python scripts/bench_policy.py --envs $n >> $O/scale.jsonl 2>>$O/err || exit 6; done
bash scripts/prof_policy.sh profpol4
