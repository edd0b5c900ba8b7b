#!/bin/bash
# Round 6, config 4 order kernel (2^14-ordinal tiles, two placement passes, stack.hip kSplit): parity of the closed
# form's pipelines (order tiles, streaming batches, device batches), the bench-size config-4 shape test, then the
# default bench against the round-5 tiling (SM_ORDER_TB=13 build in siddhi_amd/lib_tb13), alternating.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/step.sh \
  c4tests 900 python -u -m pytest tests/test_order_tiles.py tests/test_device_stream.py tests/test_device_batch.py tests/test_sparse_keys.py -x -q --timeout 600 --timeout-method thread -- \
  shape4 900 python -u -m pytest tests/test_bench_shape.py -x -v -k "config4 or config3" --timeout 800 --timeout-method thread -- \
  b_new 400 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 3 -- \
  b_old 400 env SM_LIB_VARIANT=lib_tb13 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 3 -- \
  b_new2 400 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 3 -- \
  b_old2 400 env SM_LIB_VARIANT=lib_tb13 python -u bench.py --no-cpu --no-e2e --no-ih --no-sparse --steps 10 --warmup 3
