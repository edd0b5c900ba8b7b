#!/bin/bash
# Round 6: config-5 NFA kernel, every kernel compiled on the box: round-5 tree (r5full/, 7064da0), this tree, and this
# tree with the round-5 nfa_impl.h (mix/); emitting variant and literal query.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/jc
V="--config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2"
L="--config 5 --no-cpu --steps 5 --warmup 2"
export SM_NFA_JIT_CACHE=
bash tools/step.sh \
  r5v 600 bash -c "cd r5full && python -u bench.py $V" -- \
  curv 600 env SM_NFA_JIT_CACHE=gpurun_out/jc python -u bench.py $V -- \
  mixv 600 bash -c "cd mix && python -u bench.py $V" -- \
  r5l 600 bash -c "cd r5full && python -u bench.py $L" -- \
  curl 600 env SM_NFA_JIT_CACHE=gpurun_out/jc python -u bench.py $L -- \
  mixl 600 bash -c "cd mix && python -u bench.py $L"
