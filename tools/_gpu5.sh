set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py tests/test_device_project.py tests/test_device_callbacks.py tests/test_persistence.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g5_tests.log 2>&1 || { tail -40 gpurun_out/g5_tests.log; exit 1; }
tail -1 gpurun_out/g5_tests.log
bash tools/ab_variants.sh lib || exit 1
KRE=stack4_kernel bash tools/sq_stack.sh
