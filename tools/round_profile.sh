#!/bin/bash
# Full-size bench + the rocprofv3 evidence behind its roofline object (run on the GPU box from the repo root):
#   1. bench.py at its defaults (config 4, N = 1e9)                        → gpurun_out/bench_full.log
#   2. rocprofv3 --kernel-trace --stats of the same command (no CPU leg)    → gpurun_out/prof_stats/
#   3. PMC passes FETCH_SIZE and WRITE_SIZE (one counter group per run)     → gpurun_out/pmc_fetch/, pmc_write/
# Stops at the first step that faults or times out.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${PROF_DIR:-.}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 3 "$OUT/$name.log"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
cd "$ROOT"
step bench_full 600 python -u bench.py "$@"
cd /tmp
step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_stats" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu --no-e2e --no-ih --no-sparse --steps 3 --warmup 1 "$@"
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu --no-e2e --no-ih --no-sparse --steps 1 --warmup 0 "$@"
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu --no-e2e --no-ih --no-sparse --steps 1 --warmup 0 "$@"
