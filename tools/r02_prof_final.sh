# Round-2 final evidence: config 4 (bench defaults) and config 5 through tools/round_profile.sh
# (bench line + rocprofv3 --kernel-trace --stats + FETCH_SIZE / WRITE_SIZE passes).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PROF_DIR=r02c4g bash tools/round_profile.sh || exit 1
PROF_DIR=r02c5g bash tools/round_profile.sh --config 5 || exit 1
