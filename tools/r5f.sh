set -u
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }; echo "== $name"; python3 tools/show_bench.py gpurun_out/$name.log | grep -E "value|nfa "; }
run f_var --variant pattern_count_not5s
run f_var_noidx --variant pattern_count_not5s --heap-words 4096 2>/dev/null
SM_NFA_CLOCK_INDEX=0 run f_var_gallop --variant pattern_count_not5s
run f_lit
bash tools/step.sh f_ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread || exit 1
