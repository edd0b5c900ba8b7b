#!/bin/bash
# Round 6: columns StreamCallback with the callbacks overlapping the deferred output copies: callback tests, then the
# default bench's drop-in line (via_input_handler) twice.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/step.sh \
  cb 900 python -u -m pytest tests/test_host_closed_form.py tests/test_callbacks.py tests/test_device_callbacks.py -x -q --timeout 600 --timeout-method thread -- \
  ih 600 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 5 --warmup 2 -- \
  ih2 600 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 5 --warmup 2
