set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_events.py tests/test_product_kat.py tests/test_chaining.py tests/test_broadcast_order.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g24_tests.log 2>&1 || { tail -30 gpurun_out/g24_tests.log; exit 1; }
tail -1 gpurun_out/g24_tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 > gpurun_out/c5.log 2>&1 || { tail -5 gpurun_out/c5.log; exit 1; }
python3 tools/show_bench.py gpurun_out/c5.log | grep -v "^\[bench\]\|amdgpu.ids"
