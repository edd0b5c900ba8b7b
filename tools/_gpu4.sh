set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py tests/test_device_project.py tests/test_device_callbacks.py tests/test_persistence.py tests/test_device_events.py tests/test_product_kat.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g4_tests.log 2>&1 || { tail -40 gpurun_out/g4_tests.log; exit 1; }
tail -1 gpurun_out/g4_tests.log
bash tools/ab_variants.sh lib lib_tb13 lib_r3 || exit 1
timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/g4_c5.log 2>&1 || { tail -5 gpurun_out/g4_c5.log; exit 1; }
python3 tools/show_bench.py gpurun_out/g4_c5.log | grep -v "^\[bench\]\|amdgpu.ids"
