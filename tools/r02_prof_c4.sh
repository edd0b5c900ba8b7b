# Config 4 (bench defaults) profile of the final round-2 build into gpurun_out/r02c4h.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PROF_DIR=r02c4h bash tools/round_profile.sh || exit 1
