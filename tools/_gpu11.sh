set -u
mkdir -p gpurun_out
bash tools/gpu_suite.sh || exit 1
for B in 1 0; do
  timeout -k 10 300 env SM_NFA_BALANCE=$B python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 > gpurun_out/c5_bal$B.log 2>&1 || { tail -5 gpurun_out/c5_bal$B.log; exit 1; }
  echo "== balance $B"; python3 tools/show_bench.py gpurun_out/c5_bal$B.log | grep -E "value|nfa"
done
