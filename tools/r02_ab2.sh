# A/B: stack kernel register-stack depth (lib kC=6, lib_kc4, lib_kc8) on config 4; then the main build (5 state words
# per pre processor) on config 5 with its device-event parity tests.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for L in lib lib_kc4 lib_kc8; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/ab2_$L.log 2>&1 || { tail -5 gpurun_out/ab2_$L.log; exit 1; }
  echo "== config 4 $L"; python3 tools/show_bench.py gpurun_out/ab2_$L.log | grep -v "^\[bench\]\|amdgpu.ids"
done
timeout -k 10 600 python -u -m pytest tests/test_device_events.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab2_c5tests.log 2>&1 || { tail -30 gpurun_out/ab2_c5tests.log; exit 1; }
tail -1 gpurun_out/ab2_c5tests.log
timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/ab2_c5.log 2>&1 || { tail -5 gpurun_out/ab2_c5.log; exit 1; }
echo "== config 5"; python3 tools/show_bench.py gpurun_out/ab2_c5.log | grep -v "^\[bench\]\|amdgpu.ids"
