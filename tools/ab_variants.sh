#!/bin/bash
# Config-4 bench (no CPU legs) for each library build given (siddhi_amd/<dir>), then the stamps build's phase split.
# Stops at the first failure. Usage (GPU box, repo root): bash tools/ab_variants.sh lib lib_r2 ...
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for L in "$@"; do
  timeout -k 10 300 env SM_LIB_VARIANT=$L python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/var_$L.log 2>&1 || { tail -5 gpurun_out/var_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/var_$L.log | grep -v "^\[bench\]\|amdgpu.ids" | grep -E "value|stack |key_pass0|order"
done
if [ -d siddhi_amd/lib_st ]; then
  timeout -k 10 300 env SM_LIB_VARIANT=lib_st SM_STACK_STAMPS=1 python -u bench.py --no-cpu --no-e2e --steps 2 --warmup 1 > gpurun_out/var_stamps.log 2>&1 || { tail -5 gpurun_out/var_stamps.log; exit 1; }
  grep "stack4 phases" gpurun_out/var_stamps.log | tail -2
fi
