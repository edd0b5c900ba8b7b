#!/bin/bash
# NFA kernel time of config 5 (literal and emitting variant) per JIT occupancy hint (SM_NFA_JIT_WAVES).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for q in "" "--variant pattern_count_not5s"; do
  for wv in ${WAVES:-2 4 1}; do
    SM_NFA_JIT_WAVES=$wv timeout -k 10 400 python -u bench.py --no-cpu --config 5 $q --steps 3 --warmup 1 > gpurun_out/wv_$wv.log 2>&1 || { tail -5 gpurun_out/wv_$wv.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/wv_$wv.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$q waves=$wv step', round(d['ms_per_step'],2), 'nfa', round(d['roofline']['avg_launch_ms'],2))
"
  done
done
