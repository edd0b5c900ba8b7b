#!/bin/bash
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
B=$ROOT/tests/native/build
cd /tmp
for v in micro_sort micro_ntl micro_s_1024_8 micro_s_1024_4; do
  echo "=== $v"
  timeout -k 10 60 $B/$v 100000000 2>&1 | grep -v "^walk\|pair" | head -8 || exit 1
  rm -rf $ROOT/gpurun_out/pmcv_$v
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex downsweep --output-format csv -d $ROOT/gpurun_out/pmcv_$v -o run -- $B/$v 100000000 > $ROOT/gpurun_out/pmcv_$v.log 2>&1 || { tail -3 $ROOT/gpurun_out/pmcv_$v.log; exit 1; }
done
