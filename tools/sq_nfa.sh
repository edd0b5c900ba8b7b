#!/bin/bash
# SQ / SQC counters of the config-5 NFA kernel (KRE, default the query-specialised kernel sm_nfa_jit; ARGS: bench
# arguments). One step per pass; CSVs under gpurun_out/${OUT:-sqn}_<i>/ (tools/sq_summary.py turns them into a table).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_IFETCH SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  P=${OUT:-sqn}
  rm -rf "$ROOT/gpurun_out/${P}_$i"
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-sm_nfa_jit}" --output-format csv -d "$ROOT/gpurun_out/${P}_$i" -o run -- python3 "$ROOT/bench.py" --no-cpu ${ARGS:---config 5 --variant pattern_count_not5s} --steps 1 --warmup 0 > "$ROOT/gpurun_out/${P}_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && tail -5 "$ROOT/gpurun_out/${P}_$i.log" && exit $rc
done
python3 - <<'PY'
import csv, glob, collections, os
root = os.environ.get("GRAFT_REPO_ROOT", ".")
agg = collections.defaultdict(float)
for f in glob.glob(os.path.join(root, "gpurun_out", os.environ.get("OUT", "sqn") + "_*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k:32s} {v:18.0f}")
PY
exit 0
