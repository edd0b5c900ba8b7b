#!/bin/bash
# Round 6: config-3 j order by output tiles (fastpath3.hip jt_place_kernel): the unkeyed tests (new j-tile test, the
# split / compare / variant suites, the bench-size config-3 shape), then config 3 with the tiles and with the LSD
# passes (SM_JTILE=0), alternating.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
B="--config 3 --no-cpu --steps 10 --warmup 3"
bash tools/step.sh \
  jt 600 python -u -m pytest tests/test_device_stream.py -x -q -k "j_tile" --timeout 300 --timeout-method thread -- \
  ds 900 python -u -m pytest tests/test_device_stream.py tests/test_device_batch.py -x -q --timeout 600 --timeout-method thread -- \
  shape3 900 python -u -m pytest tests/test_bench_shape.py -x -q -k "config3" --timeout 800 --timeout-method thread -- \
  c3_tile 300 python -u bench.py $B -- \
  c3_lsd 300 env SM_JTILE=0 python -u bench.py $B -- \
  c3_tile2 300 python -u bench.py $B -- \
  c3_lsd2 300 env SM_JTILE=0 python -u bench.py $B
