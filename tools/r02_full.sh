# Round-end style check on one GPU box: the whole -m gpu suite, smoke(), then bench.py at its defaults
# (config 4, with the CPU legs). Stops at the first failure.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -30 gpurun_out/full_tests.log; exit 1; }
tail -1 gpurun_out/full_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -10 gpurun_out/full_smoke.log; exit 1; }
tail -2 gpurun_out/full_smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/full_bench.log 2>&1 || { tail -10 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log
