#!/bin/bash
# Whole -m gpu suite then the default bench (config 4) without CPU legs; stops at the first failure.
# usage (GPU box, repo root): bash tools/gpu_suite.sh [pytest selection...]
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
SEL=${*:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_tests.log 2>&1 || { tail -30 gpurun_out/suite_tests.log; exit 1; }
tail -3 gpurun_out/suite_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/suite_c4.log 2>&1 || { tail -5 gpurun_out/suite_c4.log; exit 1; }
tail -1 gpurun_out/suite_c4.log
