#!/bin/bash
# Round 6: config-5 NFA kernel, this build (pending arrays) against the round-5 NFA source (siddhi_amd/lib_r5: the same
# library with kernels/nfa_impl.h of round 5, linked pending lists with node operand caches), alternating on one box.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V="--config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2"
L="--config 5 --no-cpu --steps 5 --warmup 2"
bash tools/step.sh \
  v_new 600 python -u bench.py $V -- \
  v_r5 600 env SM_LIB_VARIANT=lib_r5 python -u bench.py $V -- \
  v_new2 600 python -u bench.py $V -- \
  v_r52 600 env SM_LIB_VARIANT=lib_r5 python -u bench.py $V -- \
  l_new 600 python -u bench.py $L -- \
  l_r5 600 env SM_LIB_VARIANT=lib_r5 python -u bench.py $L
