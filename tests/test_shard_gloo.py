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
        from siddhi_amd.shard import exchange_with_ordinals
        (w_sym, w_price), w_ord, w_counts = exchange_with_ordinals(t[0], [t[0], t[1]], world, lo)
        assert w_counts == counts and torch.equal(w_ord, r_ord)
        assert torch.equal(w_sym, r_sym) and torch.equal(w_price, r_price)
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


# ---- config 5 (five streams, playback timers): key exchange + global clock-advance heartbeats (bench.py
# clock_ticks / merge_ticks) must reproduce every output of the single-process run, with the same timestamps,
# and each rank's outputs in the global relative order.
N5, K5 = 20000, 400
BODIES5 = ["every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 1 sec",
           "every e1=A, e2=B[price>e1.price]<1:3>, (e3=C or e4=D), not E for 1 sec"]


def replay5(text, sid, ts, cols):
    """Oracle over a rank's merged sequence: events (stream >= 0) and heartbeats (-1 -> advance_time)."""
    a = OracleApp(text)
    a.start()
    i, n = 0, len(ts)
    while i < n:
        if sid[i] < 0:
            a.advance_time(int(ts[i]))
            i += 1
            continue
        j = i
        while j < n and sid[j] >= 0:
            j += 1
        a.send_interleaved(sid[i:j], ts[i:j], [c[i:j] for c in cols])
        i = j
    a.flush()
    out = a.outputs()["streams"].get("Out", [])
    a.close()
    return [[r[0], r[1]] for r in out]


def _worker5(rank, world, port, outfile, body):
    from bench import clock_ticks, merge_ticks
    from siddhi_amd.shard import exchange_by_key
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = N5 * rank // world, N5 * (rank + 1) // world
        sid, cols, ts = synth.gen5(lo, hi, K5, 1)
        t = [torch.from_numpy(np.ascontiguousarray(x)) for x in cols]
        tts = torch.from_numpy(ts)
        tsid = torch.from_numpy(sid)
        ords = torch.arange(lo, hi, dtype=torch.int64)
        ticks = clock_ticks(tts, lo, world)
        (r_sym, r_price, r_vol, r_tsa, r_ts, r_ord, r_sid), _ = exchange_by_key(t[0], t + [tts, ords, tsid], world)
        m_sid, m_ts, m_cols, m_ord = merge_ticks(r_sid, r_ts, [r_sym, r_price, r_vol, r_tsa], r_ord, ticks)
        assert (np.diff(m_ts.numpy()) >= 0).all()
        local = replay5(synth.app5(body), m_sid.numpy(), m_ts.numpy(), [c.numpy() for c in m_cols])
        parts = [None] * world
        dist.all_gather_object(parts, local)
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(parts, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("body", BODIES5)
def test_config5_sharded_with_heartbeats_equal_single_process(world, body, tmp_path):
    out = str(tmp_path / "parts5.json")
    mp.start_processes(_worker5, args=(world, _free_port(), out, body), nprocs=world, join=True,
                       start_method="spawn")
    parts = json.load(open(out))
    sid, cols, ts = synth.gen5(0, N5, K5, 1)
    full = replay5(synth.app5(body), sid, ts, cols)
    assert len(full) > 30
    key = lambda r: json.dumps(r)  # noqa: E731
    assert sorted(map(key, full)) == sorted(key(r) for p in parts for r in p)
    pos = {}
    for k, r in enumerate(full):
        pos.setdefault(key(r), []).append(k)
    for p in parts:
        idx = [pos[key(r)].pop(0) for r in p]
        assert idx == sorted(idx), "a rank's outputs are out of the global order"
