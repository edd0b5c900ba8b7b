set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for c in 8388608 16777216 33554432; do
    timeout -k 10 300 python -u bench.py --no-cpu --no-e2e --no-sparse --steps 1 --warmup 1 --ih-chunk $c > gpurun_out/ihc_$c.log 2>&1 || { tail -5 gpurun_out/ihc_$c.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/ihc_$c.log'):
    if l.startswith('{'):
        ih=json.loads(l)['via_input_handler']; print('chunk $c', '%.3g' % ih['value'], round(ih['ms'],1), {k: round(x,1) for k,x in ih['host_ms_last_run'].items()})
"
  done
done
