# Config 5: NFA parity (interpreter + query-specialised kernel), then the bench (literal query).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_events.py tests/test_callbacks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || { tail -30 gpurun_out/c5_tests.log; exit 1; }
tail -1 gpurun_out/c5_tests.log
timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_bench.log 2>&1 || { tail -5 gpurun_out/c5_bench.log; exit 1; }
python3 tools/show_bench.py gpurun_out/c5_bench.log
