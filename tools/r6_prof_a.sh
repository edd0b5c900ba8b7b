#!/bin/bash
# Round-6 closing evidence, part 1 (one library build): tools/round_profile.sh for config 4 (default bench), config 5
# (literal) and the config-5 emitting variant. Summaries: tools/summarize_profile.py r06_<c> <config>.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PROF_DIR=r06_c4 bash tools/round_profile.sh || exit 1
PROF_DIR=r06_c5 bash tools/round_profile.sh --config 5 || exit 1
PROF_DIR=r06_c5v bash tools/round_profile.sh --config 5 --variant pattern_count_not5s || exit 1
