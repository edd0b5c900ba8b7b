set -u
cd $GRAFT_REPO_ROOT
PROF_DIR=r05_c4 bash tools/round_profile.sh || exit 1
PROF_DIR=r05_c5 bash tools/round_profile.sh --config 5 || exit 1
PROF_DIR=r05_c5v bash tools/round_profile.sh --config 5 --variant pattern_count_not5s || exit 1
