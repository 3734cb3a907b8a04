#!/bin/bash
# One GPU call = a list of named steps, each under its own time limit, run in order from the repo root.
#
#   scripts/gpu.sh TAG 'NAME SECONDS COMMAND...' ['NAME SECONDS COMMAND...' ...]
#
# Each step's stdout + stderr go to gpurun_out/TAG/NAME.log and its exit status to gpurun_out/TAG/steps.txt.
# COMMAND is run by bash from the repo root and may use $R (repo root) and $OUT (gpurun_out/TAG); a rocprofv3
# step does `cd /tmp && export TMPDIR=/tmp && rocprofv3 ... -- python3 $R/...` (the program right after `--`).
# A failing step is recorded and the next one runs, unless it timed out, aborted or crashed
# (124 / 137 / 134 / 139): then nothing more touches the GPU in this call.
#
# Presets (a NAME alone, no seconds / command):
#   smoke        __graft_entry__.smoke()
#   gpu_suite    pytest -m gpu, verbose, 120 s per test
#   bench        the default bench line (bench.json)
#   bench_driver the driver's form, --steps 20 --warmup 5, headline only (bench_driver.json)
#   profile      scripts/gpu_profile.sh: step-kernel trace + PMC passes (prof_TAG/)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export R OUT

preset() {
  case $1 in
    smoke) echo "300 python -u -c 'import __graft_entry__ as g; g.smoke()'";;
    gpu_suite) echo "1100 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread";;
    bench) echo "600 python -u bench.py > \$OUT/bench.json";;
    bench_driver) echo "300 python -u bench.py --steps 20 --warmup 5 --legs none > \$OUT/bench_driver.json";;
    profile) echo "900 bash scripts/gpu_profile.sh $TAG";;
    *) echo "unknown preset $1" >&2; return 1;;
  esac
}

for spec in "$@"; do
  read -r name secs cmd <<< "$spec"
  if [ -z "$secs" ]; then
    p=$(preset "$name") || exit 2
    read -r secs cmd <<< "$p"
  fi
  echo "[gpu.sh $(date +%T)] $name ($secs s): $cmd" >&2
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc" >> "$OUT/steps.txt"
  case $rc in
    124|137|134|139) echo "stop after $name (rc=$rc)" >> "$OUT/steps.txt"; exit $rc;;
  esac
done
echo done >> "$OUT/steps.txt"
