#!/bin/bash
# Round 6, NFA pending arrays (nfa_impl.h SM_NFA_PA): device-event parity (interpreter + query-specialised kernel, which
# loads the code objects tools/jit_precompile.py put in siddhi_amd/jit_cache), the config-5 emitting variant at its
# bench size, then config 5 (emitting variant with / without the arrays, literal) in the bench.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash tools/step.sh \
  ev 900 python -u -m pytest tests/test_device_events.py tests/test_broadcast_order.py -x -v --timeout 600 --timeout-method thread -- \
  shape5 600 python -u -m pytest tests/test_bench_shape.py -x -v -k config5 --timeout 600 --timeout-method thread -- \
  var_pa 600 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2 -- \
  lit 600 python -u bench.py --config 5 --no-cpu --steps 5 --warmup 2 -- \
  var_nopa 900 env SM_NFA_PA=0 python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 5 --warmup 2
