# Round-2 check: device parity (NFA interpreter + query-specialised kernel, bucket-stack pipeline), then config 4
# (lib_base vs lib) and config 5 (literal + emitting variant). Stops at the first failure.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_events.py tests/test_device_stream.py tests/test_device_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/c2_tests.log 2>&1 || { tail -30 gpurun_out/c2_tests.log; exit 1; }
tail -1 gpurun_out/c2_tests.log
for L in lib_base lib; do
  SM_LIB_VARIANT=$L timeout -k 10 400 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/c2_bench4_$L.log 2>&1 || { tail -5 gpurun_out/c2_bench4_$L.log; exit 1; }
  echo "== config 4 $L"; python3 tools/show_bench.py gpurun_out/c2_bench4_$L.log
done
timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c2_bench5.log 2>&1 || { tail -5 gpurun_out/c2_bench5.log; exit 1; }
echo "== config 5"; python3 tools/show_bench.py gpurun_out/c2_bench5.log
timeout -k 10 400 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 > gpurun_out/c2_bench5v.log 2>&1 || { tail -5 gpurun_out/c2_bench5v.log; exit 1; }
echo "== config 5 emitting variant"; python3 tools/show_bench.py gpurun_out/c2_bench5v.log
