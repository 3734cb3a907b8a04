#!/bin/bash
# Build timing variants of libgr.so (compile-time -D flags) into build/var/libgr_<name>.so.
# Usage: [VAR_DIR=dir] build_variants.sh name1="-DFOO=1 -DBAR" name2="..."
# (VAR_DIR defaults to build/var, which .gpurunignore keeps off the GPU box: use e.g. VAR_DIR=var to ship them)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/generalizableracing_amd/csrc
V=$R/${VAR_DIR:-build/var}
mkdir -p $V
pids=()
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
    -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -fno-gpu-rdc $flags -shared \
    -o $V/libgr_$name.so $C/gr_kernels.hip $C/gr_camera.hip $C/gr_policy.hip $C/gr_policy_f32.hip $C/gr_bn.hip $C/gr_update.hip -x hip $C/gr_capi.cpp &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
