set -u
# Round-5 closing evidence from one library build: rocprof stats + PMC bytes for config 4, config 5 (literal) and the
# emitting variant (tools/round_profile.sh), then the SQ counter passes of the NFA kernel for both config-5 queries.
cd $GRAFT_REPO_ROOT
bash tools/r5_profiles.sh || exit 1
OUT=sqv bash tools/sq_nfa.sh || exit 1
OUT=sql ARGS="--config 5" bash tools/sq_nfa.sh || exit 1
