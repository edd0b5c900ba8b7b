# select_records as ballot masks: NFA-path parity (device events, KATs, chaining, partitions), then config 5.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_events.py tests/test_product_kat.py tests/test_chaining.py tests/test_persistence.py tests/test_device_stream.py tests/test_partition.py tests/test_callbacks.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sel_tests.log 2>&1 || { tail -30 gpurun_out/sel_tests.log; exit 1; }
tail -1 gpurun_out/sel_tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/sel_c5.log 2>&1 || { tail -5 gpurun_out/sel_c5.log; exit 1; }
echo "== config 5"; python3 tools/show_bench.py gpurun_out/sel_c5.log | grep -v "^\[bench\]\|amdgpu.ids"
