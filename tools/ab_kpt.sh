#!/bin/bash
# Config 4 stack kernel A/B: default build vs SM_STACK_KPT=1 (siddhi_amd/lib_kpt1), plus device-stream parity of the
# variant.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 env SM_LIB_VARIANT=lib_kpt1 python -u -m pytest tests/test_device_stream.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/kpt1_tests.log 2>&1 || { tail -30 gpurun_out/kpt1_tests.log; exit 1; }
tail -1 gpurun_out/kpt1_tests.log
for L in lib lib_kpt1; do
  timeout -k 10 300 env SM_LIB_VARIANT=$L python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/kpt_$L.log 2>&1 || { tail -5 gpurun_out/kpt_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/kpt_$L.log | grep -v "^\[bench\]\|amdgpu.ids"
done
