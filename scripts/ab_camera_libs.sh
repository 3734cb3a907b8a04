#!/bin/bash
# GPU box: camera timings (gate-only and obstacle tracks, 65 536 envs) of the in-tree libgr.so and of the
# libraries given as arguments (paths relative to the repo root), twice each; JSON lines into gpurun_out/$OUT.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT:-abcam}
mkdir -p $OUT
cd $R
run() {
  timeout -k 10 200 python -c "
import sys, json; sys.path.insert(0, 'scripts'); import bench_camera
r = bench_camera.run(65536, obstacles=$2)
print(json.dumps({'lib': '$1', 'obstacles': $2, **{k: round(r[k], 4) for k in r if k.startswith('ms_')}}))" >> $OUT/cam.jsonl 2>> $OUT/cam.err
}
for rep in 1 2; do
  for ob in True False; do
    run tree $ob || exit 3
    for so in "$@"; do GR_LIB_PATH=$R/$so run $so $ob || exit 4; done
  done
done
