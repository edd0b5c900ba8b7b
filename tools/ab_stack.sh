#!/bin/bash
# Closed-form (bucket-stack) parity, then the config-4 bench with the default stack kernel and SM_STACK_V2=1 (A/B).
# Stops at the first failing step. Usage (GPU box, repo root): bash tools/ab_stack.sh [pytest -k expr]
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 600 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py tests/test_device_project.py tests/test_device_callbacks.py tests/test_persistence.py -m gpu -x -q --timeout 200 --timeout-method thread ${K:+-k "$K"} > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for V in 0 1; do
  timeout -k 10 300 env SM_STACK_V2=$V python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_c4_v2_$V.log 2>&1 || { tail -5 gpurun_out/ab_c4_v2_$V.log; exit 1; }
  echo "== SM_STACK_V2=$V"; python3 tools/show_bench.py gpurun_out/ab_c4_v2_$V.log | grep -v "^\[bench\]\|amdgpu.ids"
done
