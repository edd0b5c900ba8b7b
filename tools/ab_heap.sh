#!/bin/bash
# Config-5 NFA kernel time per heap_words (per-key arena words per semispace), emitting variant and literal query.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for q in "--variant pattern_count_not5s" ""; do
  for hw in ${HW:-2048 4096 8192}; do
    timeout -k 10 400 python -u bench.py --no-cpu --config 5 $q --heap-words $hw --steps 3 --warmup 1 > gpurun_out/hw_$hw.log 2>&1 || { tail -2 gpurun_out/hw_$hw.log; continue; }
    python3 -c "
import json
for l in open('gpurun_out/hw_$hw.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$q hw=$hw step', round(d['ms_per_step'],2), 'nfa', round(d['roofline']['avg_launch_ms'],2))
"
  done
done
