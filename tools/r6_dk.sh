#!/bin/bash
# Sparse 64-bit keys (config 4's sparse_keys side line): remap_kernel variants, alternating builds
# (lib; lib_dknt: nontemporal key / id columns; lib_dk0: table of id capacity x 1 entries instead of x 2)
set -u
mkdir -p gpurun_out
for L in lib lib_dknt lib_dk0 lib lib_dknt lib_dk0; do
  SM_LIB_VARIANT=$L timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --no-ih --steps 5 --warmup 1 \
    > gpurun_out/dk_$L.log 2>&1 || { tail -5 gpurun_out/dk_$L.log; exit 1; }
  echo "== $L $(python3 - gpurun_out/dk_$L.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d=json.loads(l); s=d.get('sparse_keys') or {}
        print('dense %.2f ms  sparse %.2f ms  ratio %.3f' % (d['ms_per_step'], s.get('ms_per_step',0), s.get('ratio_to_dense',0)))
PY
)"
done
