set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests/test_partition.py tests/test_device_stream.py tests/test_device_batch.py tests/test_device_events.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g13_tests.log 2>&1 || { tail -30 gpurun_out/g13_tests.log; exit 1; }
tail -1 gpurun_out/g13_tests.log
timeout -k 10 300 python -u bench.py --config 3 --no-cpu --steps 5 --warmup 2 > gpurun_out/c3.log 2>&1 || { tail -5 gpurun_out/c3.log; exit 1; }
python3 tools/show_bench.py gpurun_out/c3.log | grep -v "^\[bench\]\|amdgpu.ids"
rm -rf gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/c5prof" -o run -- python3 "$ROOT/bench.py" --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c5prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:18]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.3f} ms")
PY
