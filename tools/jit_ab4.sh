# Config-5 emitting variant (pattern_count_not5s): interpreter vs query-specialised kernel variants.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
B="python -u bench.py --config 5 --variant pattern_count_not5s --no-cpu --steps 2 --warmup 1"
run() { name=$1; shift; echo "== $name $*"; timeout -k 10 400 env "$@" $B > gpurun_out/$name.log 2>&1; rc=$?; echo "rc=$rc"; grep -o '"nfa": {[^}]*}' gpurun_out/$name.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log; return $rc; }
run je_i SM_NFA_JIT=0 && run je_nolds SM_NFA_JIT=1 SM_NFA_JIT_LDS=0 && run je_w4 SM_NFA_JIT=1 SM_NFA_JIT_WAVES=4 && run je_ni SM_NFA_JIT=1 SM_NFA_JIT_INLINE_ALL=0 SM_NFA_JIT_WAVES=4
