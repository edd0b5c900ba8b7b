#!/bin/bash
# Round-6 closing evidence, part 2 (same build as part 1): tools/round_profile.sh for configs 2 and 3, the SQ counter
# passes of the NFA kernel (emitting variant, literal query) and of the config-4 stack kernel.
# Summaries: tools/summarize_profile.py, tools/sq_summary.py.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PROF_DIR=r06_c2 bash tools/round_profile.sh --config 2 || exit 1
PROF_DIR=r06_c3 bash tools/round_profile.sh --config 3 || exit 1
OUT=sqv bash tools/sq_nfa.sh || exit 1
OUT=sql ARGS="--config 5" bash tools/sq_nfa.sh || exit 1
bash tools/sq_stack.sh || exit 1
