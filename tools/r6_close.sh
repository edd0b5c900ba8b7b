#!/bin/bash
# End of round 6: smoke(), then the whole -m gpu suite (the driver's round-end GPU tiers, on this tree).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/close_smoke.log 2>&1 || { tail -20 gpurun_out/close_smoke.log; exit 1; }
tail -2 gpurun_out/close_smoke.log
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/close_suite.log 2>&1 || { tail -30 gpurun_out/close_suite.log; exit 1; }
tail -3 gpurun_out/close_suite.log
