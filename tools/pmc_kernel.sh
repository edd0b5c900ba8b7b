#!/bin/bash
# PMC passes restricted to kernels matching $KRE over a short bench; CSV under gpurun_out/pmc_<i>/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  rm -rf "$ROOT/gpurun_out/pmc_$i"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-walk}" --output-format csv -d "$ROOT/gpurun_out/pmc_$i" -o run -- python3 "$ROOT/bench.py" --no-cpu ${PMC_ARGS:-} --events ${PMC_EVENTS:-1e7} --steps 1 --warmup 0 > "$ROOT/gpurun_out/pmc_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && tail -5 "$ROOT/gpurun_out/pmc_$i.log" && exit $rc
done
exit 0
