#!/bin/bash
# GPU box: learning curves of the round-3 stack (train.sh's command, stage 0): the state recipe at 4 096 envs for 2 000
# iterations with the fast options (graph-captured update, fused fp32 rollout), then the registered vision recipe for
# 400 iterations.  Logs under gpurun_out/lc3*/ (the runner's scalars.csv).
set -o pipefail
mkdir -p gpurun_out
export TRAINING_STAGE=0
timeout -k 10 600 python -u standalone/rsl_rl/train.py --task DiffLab-Quadcopter-CTBR-Racing-v0 --num_envs 4096 \
    --headless --max_iterations 2000 --graph_update --fused_rollout_fp32 --log_root gpurun_out/lc3 \
    > gpurun_out/lc3.log 2>&1 || exit 10
timeout -k 10 600 python -u standalone/rsl_rl/train.py --task DiffLab-Quadcopter-CTBR-Racing-Vision-v0 --num_envs 4096 \
    --headless --max_iterations 400 --log_root gpurun_out/lc3v > gpurun_out/lc3v.log 2>&1 || exit 11
