#!/bin/bash
# A/B of the input-handler path: the library in siddhi_amd/lib_base (SM_LIB_VARIANT=lib_base) against the in-tree one,
# alternating, ROUNDS times; prints the via_input_handler line of each run.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in lib_base lib; do
    SM_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 1 --warmup 1 > gpurun_out/abih_$v.log 2>&1 || { tail -5 gpurun_out/abih_$v.log; exit 1; }
    python3 -c "
import json,sys
for l in open('gpurun_out/abih_$v.log'):
    if l.startswith('{'):
        ih=json.loads(l)['via_input_handler']; print('$v', '%.3g' % ih['value'], round(ih['ms'],1), {k: round(x,1) for k,x in ih['host_ms_last_run'].items()})
"
  done
done
