#!/bin/bash
# One-GPU rehearsal of bench.py --gpus 4 (config 4, the exchanged stream; config 5's emitting variant: exchange,
# clock heartbeats, output merge, compared record for record): 4 ranks over gloo sharing the card (SM_BENCH_BACKEND=gloo; shard.py stages the
# collectives through host memory) against one rank on the same stream.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
A="--events 2e7 --keys 200000 --ts-div 10 --steps 2 --warmup 1 --no-cpu --no-e2e --no-ih --no-sparse"
timeout -k 10 400 python -u bench.py --gpus 1 $A > gpurun_out/w1.log 2>&1 || { tail -5 gpurun_out/w1.log; exit 1; }
SM_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 $A > gpurun_out/w4.log 2>&1 || { tail -20 gpurun_out/w4.log; exit 1; }
B="--config 5 --variant pattern_count_not5s --events 4e5 --keys 4000 --ts-div 1 --steps 1 --warmup 1 --no-cpu"
SM_BENCH_DUMP=gpurun_out/r4w1 timeout -k 10 400 python -u bench.py --gpus 1 $B > gpurun_out/w1c5.log 2>&1 || { tail -5 gpurun_out/w1c5.log; exit 1; }
SM_BENCH_DUMP=gpurun_out/r4w4 SM_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 $B > gpurun_out/w4c5.log 2>&1 || { tail -20 gpurun_out/w4c5.log; exit 1; }
python3 - <<'PY'
import json
for tag in ("", "c5"):
    r = {}
    for w in (1, 4):
        for l in open(f"gpurun_out/w{w}{tag}.log"):
            if l.startswith("{"):
                r[w] = json.loads(l)
    for w, d in r.items():
        print(tag or "c4", w, "ranks: matches", d["config"]["matches"], "ms/step", round(d["ms_per_step"], 2))
    assert r[4]["config"]["matches"] == r[1]["config"]["matches"] > 0
    print(tag or "c4", "world 4 == world 1")
# config 5: the four ranks' merged output records in rank order = the one-rank records, record for record (all words
# but the key's local slot, word 6)
import sys
sys.path.insert(0, "tests")
from test_exchange_gpu import assert_rank_records_equal
assert_rank_records_equal("gpurun_out/r4w1", "gpurun_out/r4w4", 4, r[1]["config"]["matches"])
print("c5 world 4 records == world 1 records")
PY
