#!/bin/bash
# GPU box: rocprofv3 kernel traces of a timing script against the in-tree libgr.so and timing builds
# (variants/<name>/libgr.so, scripts/build_patched.py), one step per library (scripts/gpu.sh).
#   scripts/time_lib_variants.sh TAG "SCRIPT ARGS" name1 name2 ...
TAG=$1; CMD=$2; shift 2
specs=("tree 150 cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$OUT/tree -o t -- python3 \$R/$CMD")
for v in "$@"; do
  specs+=("$v 150 cd /tmp && export TMPDIR=/tmp && GR_LIB_PATH=\$R/variants/$v/libgr.so rocprofv3 --kernel-trace --stats --output-format csv -d \$OUT/$v -o t -- python3 \$R/$CMD")
done
exec bash "$(dirname "$0")/gpu.sh" "$TAG" "${specs[@]}"
