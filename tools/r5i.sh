set -u
cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 400 python -u bench.py --config 5 --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/$name.log; exit 1; }; echo "== $name"; python3 tools/show_bench.py gpurun_out/$name.log | grep -E "value|nfa "; }
run i_var --variant pattern_count_not5s
run i_lit
bash tools/step.sh i_hcf 900 python -u -m pytest tests/test_host_closed_form.py tests/test_device_callbacks.py -x -q --timeout 600 --timeout-method thread || exit 1
timeout -k 10 500 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 3 --warmup 1 > gpurun_out/i_ih.log 2>&1 || { tail -5 gpurun_out/i_ih.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/i_ih.log'):
    if l.startswith('{'):
        d=json.loads(l); ih=d['via_input_handler']; print('config4', round(d['ms_per_step'],2), 'ms; via_input_handler', '%.3g' % ih['value'], 'ev/s', round(ih['ms'],1), 'ms', ih['host_ms_last_run'])
"
bash tools/step.sh i_ev 900 python -u -m pytest tests/test_device_events.py -x -q --timeout 600 --timeout-method thread || exit 1
bash tools/step.sh i_kat 900 python -u -m pytest tests/test_product_kat.py tests/test_callbacks.py -x -q --timeout 600 --timeout-method thread || exit 1
