set -u
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }; echo "== $name"; python3 tools/show_bench.py gpurun_out/$name.log | grep -E "value|nfa "; }
run h_var --variant pattern_count_not5s
run h_lit
bash tools/step.sh h_ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread || exit 1
bash tools/step.sh h_kat 900 python -u -m pytest tests/test_product_kat.py tests/test_callbacks.py -x -q --timeout 600 --timeout-method thread || exit 1
