# Whole -m gpu suite, then config 5 and config 4 benches (no CPU legs). Stops at the first failure.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full2_tests.log 2>&1 || { tail -30 gpurun_out/full2_tests.log; exit 1; }
tail -1 gpurun_out/full2_tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/full2_c5.log 2>&1 || { tail -5 gpurun_out/full2_c5.log; exit 1; }
echo "== config 5"; python3 tools/show_bench.py gpurun_out/full2_c5.log | grep -v "^\[bench\]\|amdgpu.ids"
for L in lib lib_kc4; do
timeout -k 10 300 env SM_LIB_VARIANT=$L python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/full2_c4_$L.log 2>&1 || { tail -5 gpurun_out/full2_c4_$L.log; exit 1; }
echo "== config 4 $L"; python3 tools/show_bench.py gpurun_out/full2_c4_$L.log | grep -v "^\[bench\]\|amdgpu.ids"
done
