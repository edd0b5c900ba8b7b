# A/B of NFA kernel variants on config 5 (N = 1e8): the interpreter vs the query-specialised (JIT) kernel, with
# the per-key heap size and the JIT's occupancy / inlining knobs. Stops at the first failing run.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
B="python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1"
run() { name=$1; hw=$2; shift 2; echo "== $name heap_words=$hw $*"; timeout -k 10 400 env "$@" $B --heap-words $hw > gpurun_out/$name.log 2>&1; rc=$?; echo "rc=$rc"; grep -o '"nfa": {[^}]*}' gpurun_out/$name.log; grep -o '"ms_per_step": [0-9.]*' gpurun_out/$name.log; return $rc; }
run jb_i256 256 SM_NFA_JIT=0 && run jb_i512 512 SM_NFA_JIT=0 && \
run jb_j256 256 SM_NFA_JIT=1 SM_NFA_JIT_WAVES=4 SM_NFA_JIT_INLINE_ALL=1 && \
run jb_j1024 1024 SM_NFA_JIT=1 SM_NFA_JIT_WAVES=4 SM_NFA_JIT_INLINE_ALL=1 && \
run jb_j3 1024 SM_NFA_JIT=1 SM_NFA_JIT_WAVES=3 SM_NFA_JIT_INLINE_ALL=1
