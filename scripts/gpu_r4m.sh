#!/bin/bash
# Round 4: the stem first block with LDS-staged images; gate + obstacle hits in inverse depth — tests, stem1 timing
# against the per-row VALU kernels, camera legs against the build before the camera change, vision A/B, stem trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r4m}
OUT=$R/gpurun_out/$T
mkdir -p $OUT
cd $R
step() {
  local name=$1; shift
  "$@"; local rc=$?
  echo "$name rc=$rc" >> $OUT/steps.txt
  case $rc in 124|137|134|139) echo "stop after $name" >> $OUT/steps.txt; exit $rc;; esac
  return 0
}
step tests bash -c "timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_stem1.py tests/test_gpu_fused_bn.py tests/test_gpu_camera.py > $OUT/pytest.log 2>&1"
for rep in 1 2; do
  step time_tree_$rep bash -c "timeout -k 10 120 python -u scripts/time_stem1.py >> $OUT/time_stem1.jsonl 2>> $OUT/time_stem1.err"
  step time_valu_$rep bash -c "GR_LIB_PATH=$R/variants/stem1_valu/libgr.so timeout -k 10 120 python -u scripts/time_stem1.py >> $OUT/time_stem1.jsonl 2>> $OUT/time_stem1.err"
  step cam_tree_$rep bash -c "timeout -k 10 200 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/cam_tree_$rep.json 2>> $OUT/cam.err"
  step cam_before_$rep bash -c "GR_LIB_PATH=$R/variants/cam_before/libgr.so timeout -k 10 200 python -u bench.py --legs camera --steps 5 --warmup 2 > $OUT/cam_before_$rep.json 2>> $OUT/cam.err"
done
step trace bash -c "cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stem -o stem -- python3 $R/scripts/time_stem1.py --reps 10 > $OUT/stem_trace.log 2>&1"
step vis_ab bash -c "timeout -k 10 900 bash scripts/time_vision_ab.sh $T/vis_ab.txt variants/stem1_valu/libgr.so > $OUT/vis_ab.log 2>&1"
echo done > $OUT/done
