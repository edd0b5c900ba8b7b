# JIT NFA kernel with / without LDS staging of the per-key state words (config 5, heap_words 4096), then parity.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
B="python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1"
run() { name=$1; shift; echo "== $name $*"; timeout -k 10 400 env "$@" $B > gpurun_out/$name.log 2>&1; rc=$?; echo "rc=$rc"; grep -o '"nfa": {[^}]*}' gpurun_out/$name.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log; return $rc; }
run jd_lds SM_NFA_JIT=1 && run jd_nolds SM_NFA_JIT=1 SM_NFA_JIT_LDS=0 && run jd_lds2 SM_NFA_JIT=1 SM_NFA_JIT_WAVES=2 && \
{ echo "== jit parity (LDS)"; timeout -k 10 600 python -u -m pytest tests/test_device_events.py -x -q -k jit --timeout 300 --timeout-method thread > gpurun_out/jd_par.log 2>&1; rc=$?; tail -3 gpurun_out/jd_par.log; exit $rc; }
