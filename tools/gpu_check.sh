#!/bin/bash
# One GPU session: parity tests, smoke, a short bench, a rocprofv3 kernel-trace summary.
# Stops at the first step that faults / aborts / times out (exit codes other than 0 and 1).
# Usage: tools/gpu_check.sh <tag> [bench args...]
set -u
TAG=${1:-run}; shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  local t0=$(date +%s)
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench prof"}
for s in $STEPS; do
  case $s in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 900 python bench.py "$@" ;;
    prof)   run rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-dropin "$@" ;;
  esac
done
echo "all steps done"
