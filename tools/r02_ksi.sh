# A/B: bucket-stack slice size (lib kSI 8 = 4096 records vs lib_ksi9 = 4608), config 4; parity of the variant.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
SM_LIB_VARIANT=lib_ksi9 timeout -k 10 600 python -u -m pytest tests/test_device_stream.py tests/test_device_project.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ksi_tests.log 2>&1 || { tail -30 gpurun_out/ksi_tests.log; exit 1; }
tail -1 gpurun_out/ksi_tests.log
for L in lib lib_ksi9 lib; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/ksi_$L.log 2>&1 || { tail -5 gpurun_out/ksi_$L.log; exit 1; }
  echo "== config 4 $L"; python3 tools/show_bench.py gpurun_out/ksi_$L.log | grep "stack \|ms/step"
done
