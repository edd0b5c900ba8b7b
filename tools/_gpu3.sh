timeout -k 10 600 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py tests/test_device_project.py tests/test_device_callbacks.py tests/test_persistence.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
bash tools/ab_variants.sh lib lib_r3
