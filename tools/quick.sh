#!/bin/bash
# Quick GPU iteration: device-batch parity tests, then a short bench (args passed through).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_device_batch.py -q -x --timeout 200 --timeout-method thread > gpurun_out/dev_tests.log 2>&1
rc=$?
tail -2 gpurun_out/dev_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u bench.py --no-cpu "$@" > gpurun_out/bench_q.log 2>&1
rc=$?
tail -1 gpurun_out/bench_q.log
exit $rc
