#!/bin/bash
# Order-kernel A/B (round 5): parity of the variant build, config-4 bench per build, FETCH_SIZE of the order kernel.
# Usage (GPU box, repo root): bash tools/ab_order.sh VARIANT_DIR [OTHER_DIR...]
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$1
SM_LIB_VARIANT=$V timeout -k 10 600 python -u -m pytest tests/test_order_tiles.py tests/test_device_stream.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abo_tests_$V.log 2>&1 || { tail -30 gpurun_out/abo_tests_$V.log; exit 1; }
tail -n 1 gpurun_out/abo_tests_$V.log
for L in lib "$@"; do
  SM_LIB_VARIANT=$L timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 5 --warmup 2 > gpurun_out/abo_bench_$L.log 2>&1 || { tail -5 gpurun_out/abo_bench_$L.log; exit 1; }
  echo "== $L"; python3 tools/show_bench.py gpurun_out/abo_bench_$L.log | grep -v "amdgpu.ids\|^\[bench\]"
done
for L in lib "$@"; do
  rm -rf gpurun_out/abo_pmc_$L
  (cd /tmp && SM_LIB_VARIANT=$L timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "order_kernel|pass0_kernel|prep_kernel" --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/abo_pmc_$L -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/gpurun_out/abo_pmc_$L.log 2>&1) || { echo "pmc $L failed"; tail -5 gpurun_out/abo_pmc_$L.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/abo_pmc_$L 2>&1 | tail -n 8
done
