#!/bin/bash
# One SQ pass (waves, cycles, waits, instruction mix) of the NFA kernel for several config-5 diagnostic queries.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
grp="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS"
i=0
while [ $# -gt 0 ]; do
  i=$((i+1)); q=$1; shift
  rm -rf "$ROOT/gpurun_out/sq1_$i"
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex sm_nfa_jit --output-format csv -d "$ROOT/gpurun_out/sq1_$i" -o run -- python3 "$ROOT/bench.py" --no-cpu --config 5 --query5 "$q" --select5 "select e1.timestamp as a having a < 0" --steps 1 --warmup 0 > "$ROOT/gpurun_out/sq1_$i.log" 2>&1
  rc=$?
  [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 "$ROOT/gpurun_out/sq1_$i.log"; exit $rc; }
  python3 - "$i" "$q" <<'PY'
import csv, glob, collections, os, sys
root = os.environ.get("GRAFT_REPO_ROOT", ".")
agg = collections.defaultdict(float)
for f in glob.glob(os.path.join(root, "gpurun_out", f"sq1_{sys.argv[1]}", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
w = agg["SQ_WAVES"] or 1
print(sys.argv[2])
print("  per wave: " + "  ".join(f"{k[3:]} {v / w:.3g}" for k, v in sorted(agg.items()) if k != "SQ_WAVES"))
print(f"  wait share {agg['SQ_WAIT_ANY'] / agg['SQ_WAVE_CYCLES']:.3f}  active share {agg['SQ_ACTIVE_INST_ANY'] / agg['SQ_WAVE_CYCLES']:.3f}")
PY
done
