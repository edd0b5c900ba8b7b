set -u
cd $GRAFT_REPO_ROOT
bash tools/step.sh r5_stream2 600 python -u -m pytest tests/test_device_stream.py -x -q --timeout 300 --timeout-method thread -k "monotone or step_back or earlier or split_batches or automatic" || exit 1
bash tools/step.sh r5_lean2 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 -- r5_full2 300 env SM_LEAN_PREP=0 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 || exit 1
for f in r5_lean2 r5_full2; do python3 tools/show_bench.py gpurun_out/$f.log | grep -v amdgpu; done
