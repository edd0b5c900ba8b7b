#!/bin/bash
# Round 6: NFA register trims (one-entry pending-array window, plan-constant entry width): device-event parity, the
# config-5 emitting variant with and without pending arrays, the literal config 5.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V="--config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2"
bash tools/step.sh \
  ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread -- \
  var_pa 600 python -u bench.py $V -- \
  var_nopa 600 env SM_NFA_PA=0 python -u bench.py $V -- \
  lit 600 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 -- \
  var_pa2 600 python -u bench.py $V
