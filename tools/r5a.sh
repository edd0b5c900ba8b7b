set -u
cd $GRAFT_REPO_ROOT
rocprofv3 -L > gpurun_out/r5_counters.txt 2>&1 || true
bash tools/step.sh r5_stream 600 python -u -m pytest tests/test_device_stream.py -x -q --timeout 300 --timeout-method thread || exit 1
bash tools/step.sh r5_lean 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 -- r5_full 300 env SM_LEAN_PREP=0 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 || exit 1
for f in r5_lean r5_full; do python3 tools/show_bench.py gpurun_out/$f.log | grep -v amdgpu; done
bash tools/step.sh r5_hw1024 300 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 --heap-words 1024 -- r5_hw8192 300 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 --heap-words 8192 -- r5_nobal 300 env SM_NFA_BALANCE=0 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 3 --warmup 1 || exit 1
for f in r5_hw1024 r5_hw8192 r5_nobal; do python3 tools/show_bench.py gpurun_out/$f.log | grep -v amdgpu; done
