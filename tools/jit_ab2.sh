# JIT NFA kernel: heap size sweep on config 5, then the JIT parity tests (config-5 variants vs the oracle).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
B="python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1"
run() { name=$1; hw=$2; shift 2; echo "== $name heap_words=$hw $*"; timeout -k 10 400 env "$@" $B --heap-words $hw > gpurun_out/$name.log 2>&1; rc=$?; echo "rc=$rc"; grep -o '"nfa": {[^}]*}' gpurun_out/$name.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log; return $rc; }
J="SM_NFA_JIT=1 SM_NFA_JIT_WAVES=3 SM_NFA_JIT_INLINE_ALL=1"
run jc_j2048 2048 $J && run jc_j4096 4096 $J && run jc_i2048 2048 SM_NFA_JIT=0 && \
{ echo "== jit parity"; SM_NFA_JIT_WAVES=3 SM_NFA_JIT_INLINE_ALL=1 timeout -k 10 600 python -u -m pytest tests/test_device_events.py -x -q -k jit --timeout 300 --timeout-method thread > gpurun_out/jc_par.log 2>&1; rc=$?; tail -3 gpurun_out/jc_par.log; exit $rc; }
