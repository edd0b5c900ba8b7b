set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g6_tests.log 2>&1 || { tail -40 gpurun_out/g6_tests.log; exit 1; }
tail -1 gpurun_out/g6_tests.log
bash tools/ab_variants.sh lib lib_skip || exit 1
KRE=stack4_kernel bash tools/sq_stack.sh
