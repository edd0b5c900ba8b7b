# A/B of the query-specialised NFA kernel's occupancy hint (SM_NFA_JIT_WAVES) on config 5.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for W in ${WAVES:-2 3 4}; do
  SM_NFA_JIT_WAVES=$W timeout -k 10 300 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5w_$W.log 2>&1 || { tail -5 gpurun_out/c5w_$W.log; exit 1; }
  echo "== waves $W"; python3 tools/show_bench.py gpurun_out/c5w_$W.log | grep -v "^\[bench\]\|amdgpu.ids"
done
