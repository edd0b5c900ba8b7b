# Config-5 NFA kernel check: JIT parity tests (device events), then the config-5 bench (literal query and the
# emitting variant). Stops at the first failure.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_events.py tests/test_having.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c5j_tests.log 2>&1 || { tail -30 gpurun_out/c5j_tests.log; exit 1; }
tail -1 gpurun_out/c5j_tests.log
timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5j_bench5.log 2>&1 || { tail -5 gpurun_out/c5j_bench5.log; exit 1; }
echo "== config 5"; python3 tools/show_bench.py gpurun_out/c5j_bench5.log
timeout -k 10 400 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 > gpurun_out/c5j_bench5v.log 2>&1 || { tail -5 gpurun_out/c5j_bench5v.log; exit 1; }
echo "== config 5 emitting variant"; python3 tools/show_bench.py gpurun_out/c5j_bench5v.log
