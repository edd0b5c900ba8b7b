#!/bin/bash
# Round 6: LDS bank spread of the ranking count rows (pass0_dev.h p0_slot, stack_dev.h rank4_slot): the closed form's
# parity tests on the new build, then config 4 alternating with the previous build (siddhi_amd/lib_base). Measured 44.6
# against 43.6 ms per step; reverted.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
B="--no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 3"
bash tools/step.sh \
  c4tests 900 python -u -m pytest tests/test_order_tiles.py tests/test_device_stream.py tests/test_device_batch.py tests/test_sparse_keys.py tests/test_host_closed_form.py -x -q --timeout 600 --timeout-method thread -- \
  shape4 900 python -u -m pytest tests/test_bench_shape.py -x -q -k "config4" --timeout 800 --timeout-method thread -- \
  b_new 400 python -u bench.py $B -- \
  b_old 400 env SM_LIB_VARIANT=lib_base python -u bench.py $B -- \
  b_new2 400 python -u bench.py $B -- \
  b_old2 400 env SM_LIB_VARIANT=lib_base python -u bench.py $B
