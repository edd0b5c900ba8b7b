# A/B of the bucket-stack kernel: parity of the new build (siddhi_amd/lib) on the device-batch / streaming tests,
# then config 4 with lib_base and lib. Stops at the first failure.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sab_tests.log 2>&1 || { tail -30 gpurun_out/sab_tests.log; exit 1; }
tail -1 gpurun_out/sab_tests.log
for L in lib_base lib; do
  SM_LIB_VARIANT=$L timeout -k 10 400 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/sab_bench_$L.log 2>&1 || { tail -5 gpurun_out/sab_bench_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/sab_bench_$L.log
done
SM_STACK_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 1 --warmup 0 2>&1 | grep "stack " 
