#!/bin/bash
# A/B of two builds of the library (siddhi_amd/lib vs siddhi_amd/$1): the variant's config-5 device-event parity
# tests, then bench.py (remaining args) with each build. Stops at the first failing step.
# Usage on the GPU box: bash tools/ab_lib.sh <variant dir> [bench args...]
set -u
V=$1
shift
mkdir -p gpurun_out
SM_LIB_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_device_events.py -q -x --timeout 200 \
  --timeout-method thread > gpurun_out/ab_tests_$V.log 2>&1 || { tail -30 gpurun_out/ab_tests_$V.log; exit 1; }
tail -1 gpurun_out/ab_tests_$V.log
for L in lib $V; do
  SM_LIB_VARIANT=$L timeout -k 10 400 python -u bench.py --no-cpu "$@" > gpurun_out/ab_bench_$L.log 2>&1 \
    || { tail -5 gpurun_out/ab_bench_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/ab_bench_$L.log
done
