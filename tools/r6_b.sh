#!/bin/bash
# Round 6: NFA pending arrays (config-5 emitting variant with / without the LDS head, literal), the columns
# StreamCallback tests and the drop-in path's bench line, the config-5 two-rank record comparison.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/step.sh \
  ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread -- \
  cb 900 python -u -m pytest tests/test_host_closed_form.py tests/test_callbacks.py -x -q --timeout 600 --timeout-method thread -- \
  var_pa 600 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2 -- \
  var_nopa 600 env SM_NFA_PA=0 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2 -- \
  lit 600 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 -- \
  ih 600 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 5 --warmup 2 -- \
  x5 900 python -u -m pytest tests/test_exchange_gpu.py -x -q -k config5 --timeout 900 --timeout-method thread
