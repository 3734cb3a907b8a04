set -o pipefail
mkdir -p gpurun_out/t6
timeout -k 10 240 python -u scripts/diag_c2_grads2.py > gpurun_out/t6/diag.txt 2>&1 || exit 5
timeout -k 10 200 python -u scripts/diag_regen.py > gpurun_out/t6/regen.txt 2>&1 || exit 6
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_c2_golden.py tests/test_gpu_c5_full_size.py tests/test_gpu_distributions.py tests/test_gpu_env_golden.py -v --timeout 300 --timeout-method thread > gpurun_out/t6/pytest.log 2>&1; echo rc=$? >> gpurun_out/t6/pytest.log
