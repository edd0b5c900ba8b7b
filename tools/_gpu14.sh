set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
rm -rf gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/c5prof" -o run -- python3 "$ROOT/bench.py" --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5prof.log 2>&1 || { tail -5 gpurun_out/c5prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c5prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:18]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e6:8.3f} ms")
PY
python3 tools/show_bench.py gpurun_out/c5prof.log | grep -E "value|nfa"
