set -u
cd $GRAFT_REPO_ROOT
bash tools/step.sh r5_ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread || exit 1
bash tools/step.sh r5_c5v 400 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 -- r5_c5 400 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 || exit 1
for f in r5_c5v r5_c5; do python3 tools/show_bench.py gpurun_out/$f.log | grep -v amdgpu; done
bash tools/step.sh r5_stream3 600 python -u -m pytest tests/test_device_stream.py -x -q --timeout 300 --timeout-method thread -k "monotone or step_back or earlier or split_batches or automatic" || exit 1
bash tools/step.sh r5_lean3 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 || exit 1
python3 tools/show_bench.py gpurun_out/r5_lean3.log | grep -v amdgpu
SM_LIB_VARIANT=lib_x2 bash tools/step.sh r5_x2_tests 600 python -u -m pytest tests/test_order_tiles.py tests/test_device_stream.py -x -q --timeout 300 --timeout-method thread -k "order or split_batches or automatic or large" || exit 1
bash tools/step.sh r5_x2_bench 300 env SM_LIB_VARIANT=lib_x2 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 || exit 1
python3 tools/show_bench.py gpurun_out/r5_x2_bench.log | grep -v amdgpu
