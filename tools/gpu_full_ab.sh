#!/bin/bash
# Whole -m gpu suite, then config 4 bench with the default stack kernels and the SM_STACK_V2=1 A/B.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_tests.log 2>&1 || { tail -30 gpurun_out/suite_tests.log; exit 1; }
tail -2 gpurun_out/suite_tests.log
for V in 0 1; do
  timeout -k 10 300 env SM_STACK_V2=$V python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_c4_v2_$V.log 2>&1 || { tail -5 gpurun_out/ab_c4_v2_$V.log; exit 1; }
  echo "== SM_STACK_V2=$V"; python3 tools/show_bench.py gpurun_out/ab_c4_v2_$V.log | grep -v "^\[bench\]\|amdgpu.ids"
done
