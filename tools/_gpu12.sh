set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g12_tests.log 2>&1 || { tail -30 gpurun_out/g12_tests.log; exit 1; }
tail -1 gpurun_out/g12_tests.log
rm -rf gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/c5prof" -o run -- python3 "$ROOT/bench.py" --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c5prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.3f} ms")
PY
