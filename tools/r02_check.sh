#!/bin/bash
# GPU check: device-batch parity tests, then the full-size bench + rocprof summary (round_profile.sh).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
PROF_DIR=${PROF_DIR:-prof} bash tools/round_profile.sh
