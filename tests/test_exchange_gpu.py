"""The multi-GPU config-4 step with the HIP matcher: shard.partitioned_step — packed-record
partition by owner (sm_partition_by_owner), all-to-all, sm_unpack_records, the bucket-stack / sort-walk pipelines on
each rank's keys, the match return and sm_order_matches — run by 2 and 3 ranks. The one-GPU box cannot give RCCL
several ranks on one device, so the ranks share cuda:0 over a gloo group (shard.py stages the collectives through
host memory); everything else is the code bench.py runs over RCCL. The ranks' outputs in rank order must equal the
single-GPU output of the whole stream exactly (core/partition/PartitionStreamReceiver.java:156-168: one stream, one
output order). The bench itself is also run with two ranks (SM_BENCH_BACKEND=gloo) and must report the same match
count as one rank."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K, DIV = 2_000_003, 20_000, 10


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _hip_match(app, dev, stack):
    hs = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def match(cols, ords):
        sym, price, ts = cols
        app.set_option("reset", 0)
        app.process_device_batch("StockStream", ts, [sym, price, price, price], ordinals=ords, hip_stream=hs)
        m = app.device_matches("q")[1]
        out = torch.empty(max(m, 1), dtype=torch.int64, device=dev)
        app.copy_device_matches("q", out)
        return out[:m]
    return match


def _rank(rank, world, port, outfile, stack):
    from siddhi_amd.shard import partitioned_step
    from siddhi_amd.testing import ProductApp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = N * rank // world, N * (rank + 1) // world
        sym, price, _, _, ts = bench.gen_stock(lo, hi, K, DIV, dev, bench.seed_for(4))
        app = ProductApp(bench.APP, fast_stack=stack)
        app.set_collect(False)
        mine = partitioned_step(sym, [sym, price, ts], world, lo, N, _hip_match(app, dev, stack))
        torch.cuda.synchronize()
        parts = [None] * world
        dist.all_gather_object(parts, mine.cpu().tolist())
        app.close()
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(parts, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,stack", [(2, 1), (3, 2)])
def test_exchange_step_with_hip_matcher_equals_one_gpu(tmp_path, world, stack):
    from siddhi_amd.shard import partitioned_step
    from siddhi_amd.testing import ProductApp
    out = str(tmp_path / "parts.json")
    mp.start_processes(_rank, args=(world, _free_port(), out, stack), nprocs=world, join=True, start_method="spawn")
    parts = json.load(open(out))
    dev = torch.device("cuda", 0)
    sym, price, _, _, ts = bench.gen_stock(0, N, K, DIV, dev, bench.seed_for(4))
    app = ProductApp(bench.APP, fast_stack=stack)
    app.set_collect(False)
    single = partitioned_step(sym, [sym, price, ts], 1, 0, N, _hip_match(app, dev, stack)).cpu()
    app.close()
    assert single.numel() > 0.05 * N
    got = torch.tensor([x for p in parts for x in p], dtype=torch.int64)
    assert got.numel() == single.numel()
    assert torch.equal(got, single)
    assert all(len(p) > 0 for p in parts)


@pytest.mark.timeout(600)
def test_bench_two_ranks_report_the_one_stream():
    """bench.py --gpus 2 (its own launcher, the exchange default) on one GPU over gloo: the same match count as one
    rank on the same stream, value counted once (strong scaling)."""
    common = ["--events", "2e6", "--keys", "20000", "--ts-div", "10", "--steps", "2", "--warmup", "1", "--no-cpu",
              "--no-e2e", "--no-ih", "--no-sparse"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    lines = []
    for g, extra in ((1, {}), (2, {"SM_BENCH_BACKEND": "gloo"})):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(g)] + common,
                           env={**env, **extra}, capture_output=True, text=True, timeout=500)
        assert r.returncode == 0, r.stderr[-3000:]
        js = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
        assert len(js) == 1
        lines.append(js[0])
    one, two = lines
    assert two["n_gpus"] == 2 and two["scaling"] == "strong"
    assert two["config"]["matches"] == one["config"]["matches"] > 0
    assert two["config"]["events"] == one["config"]["events"] == 2_000_000
    assert abs(two["value"] - 2e6 / (two["ms_per_step"] * 1e-3)) < 1e-6 * two["value"]
    assert one["config"]["rccl_world"] is None and two["config"]["rccl_world"] is None  # gloo rehearsal


def assert_rank_records_equal(one_prefix, many_prefix, world, n):
    """bench.py SM_BENCH_DUMP files: one rank's output records against the concatenation of `world` ranks' (int64
    words of sm_out_rec + select values + ordinals), all words but the key slot (word 6)."""
    import torch
    ref = torch.load(f"{one_prefix}.rank0.pt", weights_only=True)
    got = torch.cat([torch.load(f"{many_prefix}.rank{r}.pt", weights_only=True) for r in range(world)])
    assert ref.shape[0] == n and got.shape == ref.shape
    keep = [w for w in range(ref.shape[1]) if w != 6]
    bad = (got[:, keep] != ref[:, keep]).any(dim=1).nonzero()
    assert bad.numel() == 0, f"first differing record {int(bad[0])}: {got[int(bad[0])].tolist()} != {ref[int(bad[0])].tolist()}"


@pytest.mark.timeout(900)
def test_bench_config5_two_ranks_merge_to_one_stream(tmp_path):
    """bench.py --config 5 --gpus 2 (its own launcher, over gloo on the one GPU): the key exchange, the global clock
    heartbeats (sm_merge_heartbeats) and the output merge (shard.merge_outputs / sm_order_outputs) inside the timed
    step, with the HIP NFA kernel on each rank; the emitting variant must report the same output count as one rank."""
    common = ["--config", "5", "--variant", "pattern_count_not5s", "--events", "3e5", "--keys", "3000", "--ts-div", "1",
              "--steps", "1", "--warmup", "1", "--no-cpu"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    lines = []
    dumps = {}
    for g, extra in ((1, {}), (2, {"SM_BENCH_BACKEND": "gloo"})):
        dumps[g] = os.path.join(str(tmp_path), f"w{g}")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(g)] + common,
                           env={**env, **extra, "SM_BENCH_DUMP": dumps[g]}, capture_output=True, text=True,
                           timeout=800)
        assert r.returncode == 0, r.stderr[-3000:]
        js = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
        assert len(js) == 1
        lines.append(js[0])
    one, two = lines
    assert two["n_gpus"] == 2 and two["config"]["events"] == one["config"]["events"] == 300_000
    assert two["config"]["matches"] == one["config"]["matches"] > 100
    # record for record. The ranks' merged records (bench.py's timed path: merge_outputs) in rank order
    # are the one-rank delivery order: trigger ordinal, step time, key first-seen ordinal, output timestamp, phase /
    # query / scheduler / emission rank, every select value with its null flag, every matched event's ordinal. Only
    # word 6 differs by construction (the key's slot in the rank's own table, a diagnostic).
    assert_rank_records_equal(dumps[1], dumps[2], 2, one["config"]["matches"])
