#!/bin/bash
# Round 6: config-5 emitting variant, pending arrays' LDS head size and occupancy: default (20 KiB per workgroup, 7
# entries, 2 waves per SIMD), 40 KiB (25 entries, 1 wave per SIMD, 512 VGPRs: no scratch), no LDS head at 1 wave.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V="--config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2"
bash tools/step.sh \
  w_def 600 python -u bench.py $V -- \
  w_1k40 600 env SM_NFA_JIT_WAVES=1 SM_NFA_PA_KB=40 python -u bench.py $V -- \
  w_1nopa 600 env SM_NFA_JIT_WAVES=1 SM_NFA_PA=0 python -u bench.py $V -- \
  w_def2 600 python -u bench.py $V
