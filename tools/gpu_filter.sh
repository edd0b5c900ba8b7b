#!/bin/bash
# Filter (config 2) + config 3 parity tests and benches on one GPU.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_device_filter.py -x -v --timeout 300 --timeout-method thread > gpurun_out/filter_tests.log 2>&1 || { tail -40 gpurun_out/filter_tests.log; exit 1; }
tail -3 gpurun_out/filter_tests.log
for c in 2 3; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 2 > gpurun_out/bench_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
  echo "== config $c"; python3 tools/show_bench.py gpurun_out/bench_c$c.log
done
