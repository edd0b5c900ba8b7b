#!/bin/bash
# Round 6: order2_kernel (order_dev.h) against the round-3 order kernel (siddhi_amd/lib_v1, SM_ORDER_V1=1): the
# closed-form suites that reach the order kernel with the default build, then config 4 alternating the two builds.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_order_tiles.py \
  tests/test_bench_shape.py tests/test_sparse_keys.py tests/test_device_stream.py tests/test_device_batch.py \
  > gpurun_out/o2_tests.log 2>&1 || { tail -40 gpurun_out/o2_tests.log; exit 1; }
tail -2 gpurun_out/o2_tests.log
for L in lib lib_v1 lib lib_v1; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 2 \
    > gpurun_out/o2_bench_$L.log 2>&1 || { tail -5 gpurun_out/o2_bench_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/o2_bench_$L.log
done
SM_LIB_VARIANT=lib_o2s timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 2 --warmup 1 \
  > gpurun_out/o2s.log 2>&1 || { tail -5 gpurun_out/o2s.log; exit 1; }
grep "order2 phases" gpurun_out/o2s.log | tail -1
