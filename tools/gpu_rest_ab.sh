#!/bin/bash
# The -m gpu files from test_device_project on, then the config 4 A/B (default stack kernels vs SM_STACK_V2=1).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_project.py tests/test_device_stream.py tests/test_having.py tests/test_nfa_jit.py tests/test_partition.py tests/test_persistence.py tests/test_product_kat.py tests/test_shard_gloo.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/rest_tests.log 2>&1 || { tail -30 gpurun_out/rest_tests.log; exit 1; }
tail -2 gpurun_out/rest_tests.log
for V in 0 1; do
  timeout -k 10 300 env SM_STACK_V2=$V python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ab_c4_v2_$V.log 2>&1 || { tail -5 gpurun_out/ab_c4_v2_$V.log; exit 1; }
  echo "== SM_STACK_V2=$V"; python3 tools/show_bench.py gpurun_out/ab_c4_v2_$V.log | grep -v "^\[bench\]\|amdgpu.ids"
done
