#!/bin/bash
# Round 6: NFA parity and the config-5 benches (emitting variant, literal) with the code-object cache of this tree.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/step.sh \
  ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread -- \
  var 600 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2 -- \
  lit 600 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2
