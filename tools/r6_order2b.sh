#!/bin/bash
# order2 tiles per workgroup (lib = 32, lib_gt16, lib_gt64) on config 4, then PMC bytes of order2 (lib) and the
# round-3 order kernel (lib_v1) at full size
set -u
mkdir -p gpurun_out
for L in lib lib_gt16 lib_gt64 lib; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 2 \
    > gpurun_out/o2b_bench_$L.log 2>&1 || { tail -5 gpurun_out/o2b_bench_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/o2b_bench_$L.log | grep -E "value|order"
done
for L in lib lib_v1; do
  echo "== PMC $L"
  SM_LIB_VARIANT=$L KRE=order PMC_EVENTS=1e9 PMC_ARGS="--no-e2e --no-ih --no-sparse" bash tools/pmc_kernel.sh FETCH_SIZE WRITE_SIZE || exit 1
  mkdir -p gpurun_out/pmc_$L && cp -r gpurun_out/pmc_1 gpurun_out/pmc_2 gpurun_out/pmc_$L/
done
