#!/bin/bash
# SQ counters of one kernel (KRE, default the config-4 stack kernel; SQ_ARGS: the bench arguments, default config 4 at
# full size), one step, two passes; CSVs under gpurun_out/sq_<i>/.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  rm -rf "$ROOT/gpurun_out/sq_$i"
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "${KRE:-stack4_kernel}" --output-format csv -d "$ROOT/gpurun_out/sq_$i" -o run -- python3 "$ROOT/bench.py" --no-cpu ${SQ_ARGS:---no-e2e --no-ih --no-sparse --events 1e9} --steps 1 --warmup 0 > "$ROOT/gpurun_out/sq_$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  [ $rc -ne 0 ] && tail -5 "$ROOT/gpurun_out/sq_$i.log" && exit $rc
done
exit 0
