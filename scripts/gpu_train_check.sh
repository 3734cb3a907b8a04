mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_units.py tests/test_gpu_graph_update.py tests/test_gpu_fused_inference.py -q --timeout 120 --timeout-method thread > gpurun_out/cs.log 2>&1 || exit 3
timeout -k 10 200 python -u scripts/train_breakdown.py > gpurun_out/train_bd.log 2>&1 || exit 4
GRAPH=1 FUSED=1 BF16=1 PROF=0 timeout -k 10 200 python -u scripts/train_breakdown.py > gpurun_out/train_bd2.log 2>&1
