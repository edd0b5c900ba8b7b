set -u
cd $GRAFT_REPO_ROOT
bash tools/step.sh j_hcf 900 python -u -m pytest tests/test_host_closed_form.py tests/test_device_callbacks.py tests/test_device_project.py tests/test_callbacks.py -x -q --timeout 600 --timeout-method thread || exit 1
timeout -k 10 500 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 3 --warmup 1 > gpurun_out/j_ih.log 2>&1 || { tail -5 gpurun_out/j_ih.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/j_ih.log'):
    if l.startswith('{'):
        d=json.loads(l); ih=d['via_input_handler']; print('config4', round(d['ms_per_step'],2), 'ms; via_input_handler', '%.3g' % ih['value'], 'ev/s', round(ih['ms'],1), 'ms', ih['host_ms_last_run'])
"
