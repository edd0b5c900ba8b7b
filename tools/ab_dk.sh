#!/bin/bash
# Sparse-key side line (dense-id lookup) with the XCD-sliced lookup (default) and without (SM_DK_XCD=0), plus the
# sparse-key tests. Prints ms per step and the ratio to the dense step of each run.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sparse_keys.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dk_tests.log 2>&1 || { tail -20 gpurun_out/dk_tests.log; exit 1; }
tail -1 gpurun_out/dk_tests.log
for r in 1 2; do
  for v in 1 0; do
    SM_DK_XCD=$v timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --steps 3 --warmup 1 > gpurun_out/dk_$v.log 2>&1 || { tail -5 gpurun_out/dk_$v.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/dk_$v.log'):
    if l.startswith('{'):
        d=json.loads(l); sp=d['sparse_keys']; print('xcd=$v dense', round(d['ms_per_step'],2), 'sparse', round(sp['ms_per_step'],2), 'ratio', round(sp['ratio_to_dense'],3))
"
  done
done
