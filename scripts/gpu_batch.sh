set -o pipefail
mkdir -p gpurun_out/t8
GR_LIB_PATH=variants/v13/libgr.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "free_run or ragged or teacher or obstacle" --timeout 300 --timeout-method thread > gpurun_out/t8/parity_v13.log 2>&1; rc=$?; echo rc=$rc >> gpurun_out/t8/parity_v13.log; [ $rc -ge 124 ] && exit 9
bash scripts/time_libs.sh t8/tl_g.txt variants/v13/libgr.so || exit 3
BENCH_ARGS="--obstacles 1" bash scripts/time_libs.sh t8/tl_o.txt variants/v13/libgr.so || exit 3
BENCH_ARGS="--gates 32" bash scripts/time_libs.sh t8/tl_32.txt variants/v13/libgr.so || exit 3
