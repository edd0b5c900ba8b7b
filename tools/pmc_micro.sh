#!/bin/bash
# Phase stamps + PMC passes over the sort/walk micro-benchmark (tests/native/build/micro_sort*).
# Usage: tools/pmc_micro.sh [N] "GROUP1" "GROUP2" ...   CSVs under gpurun_out/pmcm_<i>/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
N=$1; shift
B=$ROOT/tests/native/build
timeout -k 10 120 $B/micro_sort $N > $ROOT/gpurun_out/micro.log 2>&1 || { cat $ROOT/gpurun_out/micro.log; exit 1; }
cat $ROOT/gpurun_out/micro.log
timeout -k 10 120 $B/micro_sort_stamps $N > $ROOT/gpurun_out/micro_stamps.log 2>&1 || { cat $ROOT/gpurun_out/micro_stamps.log; exit 1; }
grep shares $ROOT/gpurun_out/micro_stamps.log | sort | uniq -c | head -20
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  rm -rf "$ROOT/gpurun_out/pmcm_$i"
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/gpurun_out/pmcm_$i" -o run -- $B/micro_sort $N > "$ROOT/gpurun_out/pmcm_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && tail -5 "$ROOT/gpurun_out/pmcm_$i.log" && exit $rc
done
exit 0
