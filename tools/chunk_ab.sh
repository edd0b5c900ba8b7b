# Chunk-sorted key pass 0 for the bucket-stack pipeline: parity of the streaming / device-batch tests, then config 4
# with the chunk-sorted layout (default) and with the global-bucket pass (SM_STACK_CHUNKED=0).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ch_tests.log 2>&1 || { tail -30 gpurun_out/ch_tests.log; exit 1; }
tail -1 gpurun_out/ch_tests.log
for C in 1 0; do
  SM_STACK_CHUNKED=$C timeout -k 10 400 python -u bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/ch_bench_$C.log 2>&1 || { tail -5 gpurun_out/ch_bench_$C.log; exit 1; }
  echo "== chunked=$C"; python3 tools/show_bench.py gpurun_out/ch_bench_$C.log
done
