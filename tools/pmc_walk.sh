#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over a short bench; CSV output under gpurun_out/pmc_<i>/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/gpurun_out/pmc_$i" -o run -- python3 "$ROOT/bench.py" --no-cpu --events ${PMC_EVENTS:-1e7} --steps 1 --warmup 0 > "$ROOT/gpurun_out/pmc_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && tail -5 "$ROOT/gpurun_out/pmc_$i.log" && exit $rc
done
exit 0
