# Configs 2 and 3 on the current build (bench lines with CPU legs).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for C in 2 3; do
  timeout -k 10 400 python -u bench.py --config $C --steps 5 --warmup 2 > gpurun_out/c23_$C.log 2>&1 || { tail -5 gpurun_out/c23_$C.log; exit 1; }
  echo "== config $C"; python3 tools/show_bench.py gpurun_out/c23_$C.log | grep -v "^\[bench\]\|amdgpu.ids"
done
