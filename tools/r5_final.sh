set -u
# Round-5 closing evidence from one library build: rocprof stats + PMC bytes for config 4, config 5 (literal), the
# emitting variant, configs 2 and 3 (tools/round_profile.sh), then the SQ counter passes of the NFA kernel for both
# config-5 queries (tools/sq_nfa.sh). Summaries: tools/summarize_profile.py, tools/sq_summary.py.
cd $GRAFT_REPO_ROOT
bash tools/r5_profiles.sh || exit 1
PROF_DIR=r05_c2 bash tools/round_profile.sh --config 2 || exit 1
PROF_DIR=r05_c3 bash tools/round_profile.sh --config 3 || exit 1
OUT=sqv bash tools/sq_nfa.sh || exit 1
OUT=sql ARGS="--config 5" bash tools/sq_nfa.sh || exit 1
