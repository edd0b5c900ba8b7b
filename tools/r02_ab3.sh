# A/B: LDS staging of the key-state words on / off x occupancy hint, config 5 (env knobs, same build).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for V in "1 3" "0 3" "0 4" "0 5"; do
  set -- $V
  SM_NFA_JIT_LDS=$1 SM_NFA_JIT_WAVES=$2 timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/ab3_$1_$2.log 2>&1 || { tail -5 gpurun_out/ab3_$1_$2.log; exit 1; }
  echo "== lds $1 waves $2"; python3 tools/show_bench.py gpurun_out/ab3_$1_$2.log | grep "nfa \|ms/step"
done
