#!/bin/bash
# Round 4 closing: the camera hit-batch A/B (r4pc), then the full validation (smoke, GPU suite, regeneration, bench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_r4pc.sh r4pc || exit $?
bash scripts/gpu_r4zz.sh r4zz5
