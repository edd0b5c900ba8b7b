#!/bin/bash
# Stamps + write/read request counters of the micro-benchmark's down-sweeps.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
B=$ROOT/tests/native/build
cd /tmp
timeout -k 10 120 $B/micro_sort_stamps ${N:-100000000} > $ROOT/gpurun_out/micro_stamps.log 2>&1 || exit 1
grep shares $ROOT/gpurun_out/micro_stamps.log | sort | uniq -c
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"; do
  i=$((i+1))
  rm -rf $ROOT/gpurun_out/pmcw_$i
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-downsweep}" --output-format csv -d $ROOT/gpurun_out/pmcw_$i -o run -- $B/micro_sort ${N:-100000000} > $ROOT/gpurun_out/pmcw_$i.log 2>&1 || { tail -3 $ROOT/gpurun_out/pmcw_$i.log; exit 1; }
done
