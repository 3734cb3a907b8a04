#!/bin/bash
# GPU box: camera timings of the in-tree libgr.so and of every build/var/libgr_*.so, no obstacles, same call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-abcam}
mkdir -p $OUT
cd $R
run() {
  timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, 'scripts'); import bench_camera
r = bench_camera.run(65536, obstacles=$2)
print(json.dumps({'lib': '$1', 'obstacles': $2, **{k: r[k] for k in r if k.startswith('ms_') or k == 'render_fraction'}}))" >> $OUT/cam.jsonl 2>> $OUT/cam.err
}
for rep in 1 2; do
  run tree False || exit 3
  for so in build/var/libgr_*.so; do GR_LIB_PATH=$R/$so run $so False || exit 4; done
  run tree True || exit 5
done
