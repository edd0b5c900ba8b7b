#!/bin/bash
# lane_balance on / off for config 5 (ARGS: bench arguments): time (3 steps) and FETCH_SIZE / WRITE_SIZE of the NFA
# kernel (separate passes, one step each). Round 5: re-decides the option on PMC bytes as well as time.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for bal in default 0; do
  envs=""
  [ "$bal" = "0" ] && envs="SM_NFA_BALANCE=0"
  env $envs timeout -k 10 400 python3 "$ROOT/bench.py" --no-cpu --config 5 ${ARGS:-} --steps 3 --warmup 1 > "$ROOT/gpurun_out/bal_${bal}.log" 2>&1 || { echo "bench $bal failed"; tail -5 "$ROOT/gpurun_out/bal_${bal}.log"; exit 1; }
  python3 "$ROOT/tools/show_bench.py" "$ROOT/gpurun_out/bal_${bal}.log" | grep -E "value|nfa "
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf "$ROOT/gpurun_out/bal_${bal}_$c"
    env $envs timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "sm_nfa_jit" --output-format csv -d "$ROOT/gpurun_out/bal_${bal}_$c" -o run -- python3 "$ROOT/bench.py" --no-cpu --config 5 ${ARGS:-} --steps 1 --warmup 0 > "$ROOT/gpurun_out/bal_${bal}_$c.log" 2>&1 || { echo "pmc $bal $c failed"; exit 1; }
  done
  python3 - "$ROOT" "$bal" <<'PY'
import csv, glob, sys
root, bal = sys.argv[1], sys.argv[2]
v = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"{root}/gpurun_out/bal_{bal}_{c}/**/*counter_collection.csv", recursive=True):
        v[c] = sum(float(r["Counter_Value"]) for r in csv.DictReader(open(f)))
rd = 2 * v.get("FETCH_SIZE", 0) * 1024 / 1e9
wr = v.get("WRITE_SIZE", 0) * 1024 / 1e9
print(f"balance {bal}: NFA kernel HBM read {rd:.1f} GB (FETCH_SIZE x2), write {wr:.1f} GB, total {rd + wr:.1f} GB")
PY
done
