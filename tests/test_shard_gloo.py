"""Multi-rank path of the partitioned pattern (config 4) on CPU with the gloo backend, world size 2 and 3:
contiguous ingest slices → key exchange (siddhi_amd.shard.exchange_by_key, the same code bench.py runs over
RCCL) → per-rank matching with global ordinals → merge_matches must equal the single-process reference output.
The per-rank matcher here is the CPU oracle (this test checks the sharding logic, not the kernels; the GPU
kernels on a rank's key subset are checked in tests/test_device_batch.py::test_sharded_ordinals_match_oracle_subset)."""
import ctypes
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import synth
from oracle_lib import OracleApp, lib as olib

APP = ("define stream StockStream (symbol int, price double, volume long, timestamp long); "
       "partition with (symbol of StockStream) begin "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.timestamp as i, e2.timestamp as j insert into OutputStream; end;")
N, K, DIV = 20000, 97, 7


def oracle_refs(cols, ts):
    a = OracleApp(APP)
    a.start()
    cs = [np.ascontiguousarray(c) for c in cols]
    ptrs = (ctypes.c_void_p * len(cs))(*[c.ctypes.data for c in cs])
    err = ctypes.create_string_buffer(512)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    rc = olib().cr_send_columns(a.h, a.stream_index("StockStream"), len(ts), ts.ctypes.data, ptrs, err, 512)
    assert rc == 0, err.value
    out = a.outputs()["streams"].get("OutputStream", [])
    a.close()
    return np.array([r[2] for r in out], dtype=np.int64).reshape(-1, 2)


def _worker(rank, world, port, outfile):
    from siddhi_amd.shard import exchange_by_key
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = N * rank // world, N * (rank + 1) // world
        sym, price, vol, tsa, ts = synth.gen_stock(lo, hi, K, DIV, synth.seed_for(4))
        t = [torch.from_numpy(x) for x in (sym, price, vol, tsa, ts)]
        ordinals = torch.arange(lo, hi, dtype=torch.int64)
        (r_sym, r_price, r_vol, r_tsa, r_ts, r_ord), counts = exchange_by_key(t[0], t + [ordinals], world)
        assert sum(counts) == r_ord.numel()
        ords = r_ord.numpy()
        assert (np.diff(ords) > 0).all(), "received rows not in global arrival order"
        assert (np.remainder(r_sym.numpy(), world) == rank).all()
        local = oracle_refs([r_sym.numpy(), r_price.numpy(), r_vol.numpy(), r_tsa.numpy()], r_ts.numpy())
        glob = ords[local] if len(local) else local
        parts = [None] * world
        dist.all_gather_object(parts, glob.tolist())
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(parts, f)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_and_merge_equal_single_process(world, tmp_path):
    from siddhi_amd.shard import merge_matches
    out = str(tmp_path / "parts.json")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    with open(out) as f:
        parts = json.load(f)
    got = merge_matches(parts)
    sym, price, vol, tsa, ts = synth.gen_stock(0, N, K, DIV, synth.seed_for(4))
    exp = oracle_refs([sym, price, vol, tsa], ts)
    assert len(exp) > 1000
    np.testing.assert_array_equal(got, exp)


def test_merge_keeps_same_trigger_order():
    from siddhi_amd.shard import merge_matches
    a = [[1, 5], [0, 5], [2, 9]]
    b = [[3, 4], [4, 7]]
    np.testing.assert_array_equal(merge_matches([a, b]), [[3, 4], [1, 5], [0, 5], [4, 7], [2, 9]])
