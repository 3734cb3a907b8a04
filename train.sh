#!/bin/bash
# Same entry point as the reference's train.sh; add
#   python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1
# in front of the script path for one env shard per GPU.
python standalone/rsl_rl/train.py --task DiffLab-Quadcopter-CTBR-Racing-v0 --num_envs 1024 --headless "$@"
