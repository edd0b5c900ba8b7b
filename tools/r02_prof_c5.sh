# Config-5 profile of the current build (rocprofv3 stats + PMC into gpurun_out/r02c5b), then the stack kernel's
# phase stamps on config 4 (1 step).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PROF_DIR=r02c5b bash tools/round_profile.sh --config 5 || exit 1
SM_STACK_STAMPS=1 timeout -k 10 300 python -u bench.py --no-cpu --steps 1 --warmup 0 > gpurun_out/c4_stamps.log 2>&1 || { tail -5 gpurun_out/c4_stamps.log; exit 1; }
grep "stack " gpurun_out/c4_stamps.log
