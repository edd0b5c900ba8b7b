set -u
mkdir -p gpurun_out
KRE=sm_nfa_jit SQ_ARGS="--config 5" bash tools/sq_stack.sh || exit 1
KRE=sm_nfa_jit PMC_ARGS="--config 5" PMC_EVENTS=1e8 bash tools/pmc_kernel.sh "FETCH_SIZE" "WRITE_SIZE" || exit 1
