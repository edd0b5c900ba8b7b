# Register-stack depth 5 as the default: closed-form parity (device batch / stream / projection), then config 4.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_batch.py tests/test_device_stream.py tests/test_device_project.py tests/test_persistence.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kc5_tests.log 2>&1 || { tail -30 gpurun_out/kc5_tests.log; exit 1; }
tail -1 gpurun_out/kc5_tests.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/kc5_bench.log 2>&1 || { tail -5 gpurun_out/kc5_bench.log; exit 1; }
python3 tools/show_bench.py gpurun_out/kc5_bench.log | grep -v "^\[bench\]\|amdgpu.ids"
