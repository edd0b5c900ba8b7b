set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g7_tests.log 2>&1 || { tail -40 gpurun_out/g7_tests.log; exit 1; }
tail -1 gpurun_out/g7_tests.log
for V in 1 0; do
  timeout -k 10 300 env SM_PASS0_V2=$V python -u bench.py --no-cpu --no-e2e --steps 5 --warmup 2 > gpurun_out/p0_$V.log 2>&1 || { tail -5 gpurun_out/p0_$V.log; exit 1; }
  echo "== SM_PASS0_V2=$V"; python3 tools/show_bench.py gpurun_out/p0_$V.log | grep -v "^\[bench\]\|amdgpu.ids" | grep -E "value|stack |key_pass0|order|prep"
done
KRE=pass0_kernel PMC_EVENTS=1e9 bash tools/pmc_kernel.sh "FETCH_SIZE" "WRITE_SIZE" || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 2>&1 | tail -8
for W in 3 2 1 4; do
  timeout -k 10 300 env SM_NFA_JIT_WAVES=$W python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5_w$W.log 2>&1 || { tail -5 gpurun_out/c5_w$W.log; exit 1; }
  echo "== waves $W"; python3 tools/show_bench.py gpurun_out/c5_w$W.log | grep -E "value|nfa "
done
