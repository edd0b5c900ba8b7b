set -u
# End of round 5: the whole -m gpu suite and the default bench (tools/gpu_suite.sh), then the closing profiles of the
# same build (tools/r5_final.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_suite.sh || exit 1
bash tools/r5_final.sh > gpurun_out/r5_final.log 2>&1 || { tail -20 gpurun_out/r5_final.log; exit 1; }
grep -E "== .*rc=" gpurun_out/r5_final.log | tail -30
