#!/bin/bash
# order2_kernel phase clock (siddhi_amd/lib_o2s, SM_ORDER2_STAMPS=1) on config 4
set -u
mkdir -p gpurun_out
SM_LIB_VARIANT=lib_o2s timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 2 --warmup 1 \
  > gpurun_out/o2s.log 2>&1 || { tail -5 gpurun_out/o2s.log; exit 1; }
grep "order2 phases" gpurun_out/o2s.log | tail -2
