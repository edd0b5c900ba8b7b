#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary of the bench.
# Stops at the first step that faults, aborts or times out (exit codes other than 0/1).
# Usage (from the repo root, on the GPU box): bash tools/gpu_check.sh [tests|bench|prof|all] [bench args...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
what=${1:-all}
shift || true
export TMPDIR=/tmp

run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc=$rc)"
    exit $rc
  fi
  return 0
}

cd "$ROOT"
if [ "$what" = tests ] || [ "$what" = all ]; then
  run gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=20 -p no:cacheprovider
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$what" = bench ] || [ "$what" = all ]; then
  run bench 900 python -u bench.py "$@"
fi
if [ "$what" = prof ] || [ "$what" = all ]; then
  cd /tmp
  run prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --no-cpu "$@"
fi
