# A/B: register-stack depth 3 / 4 (default) / 5 on config 4 (slices of 4608); parity of the depth-3 build.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
SM_LIB_VARIANT=lib_kc3 timeout -k 10 600 python -u -m pytest tests/test_device_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kc3_tests.log 2>&1 || { tail -30 gpurun_out/kc3_tests.log; exit 1; }
tail -1 gpurun_out/kc3_tests.log
for L in lib lib_kc3 lib_kc5 lib; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/kc35_$L.log 2>&1 || { tail -5 gpurun_out/kc35_$L.log; exit 1; }
  echo "== config 4 $L"; python3 tools/show_bench.py gpurun_out/kc35_$L.log | grep "stack \|ms/step"
done
