#!/bin/bash
# A/B of the record-pass down-sweeps: device tests (default build) + bench with SM_SORT_WC=1 and =0.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_device_batch.py -q -x --timeout 200 --timeout-method thread > gpurun_out/dev_tests.log 2>&1 || { tail -30 gpurun_out/dev_tests.log; exit 1; }
tail -1 gpurun_out/dev_tests.log
for v in 1 0; do
  SM_SORT_WC=$v timeout -k 10 400 python -u bench.py --no-cpu "$@" > gpurun_out/bench_wc$v.log 2>&1 || { tail -5 gpurun_out/bench_wc$v.log; exit 1; }
  echo "== SM_SORT_WC=$v"; python3 tools/show_bench.py gpurun_out/bench_wc$v.log
done
