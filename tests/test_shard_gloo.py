"""Multi-rank path of the partitioned pattern (config 4) on CPU with the gloo backend, world size 2 and 3:
contiguous ingest slices → key exchange (siddhi_amd.shard.exchange_with_ordinals: one packed record per event,
the same code bench.py runs over RCCL) → per-rank matching with global ordinals → return_matches (every tuple to
the rank that ingested its e2, ordered there) — the ranks' outputs concatenated in rank order must equal the
single-process reference output. Config 2 (filter, index-range shards): concat_ordered of the per-rank kept rows.
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
        from siddhi_amd.shard import owner_of, pack_pairs, return_matches, slice_starts, unpack_pairs
        assert (owner_of(r_sym, world) == rank).all()
        local = oracle_refs([r_sym.numpy(), r_price.numpy(), r_vol.numpy(), r_tsa.numpy()], r_ts.numpy())
        glob = ords[local] if len(local) else local.reshape(-1, 2)
        packed = pack_pairs(torch.from_numpy(glob[:, 0]), torch.from_numpy(glob[:, 1]))
        mine = return_matches(packed, slice_starts(lo, world, packed.device), N, world)
        e1, e2 = unpack_pairs(mine)
        assert ((e2 >= lo) & (e2 < hi)).all()
        parts = [None] * world
        dist.all_gather_object(parts, [glob.tolist(), torch.stack([e1, e2], 1).tolist()])
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
    sym, price, vol, tsa, ts = synth.gen_stock(0, N, K, DIV, synth.seed_for(4))
    exp = oracle_refs([sym, price, vol, tsa], ts)
    assert len(exp) > 1000
    np.testing.assert_array_equal(merge_matches([p[0] for p in parts]), exp)  # host merge of per-key-rank tuples
    returned = np.concatenate([np.asarray(p[1], dtype=np.int64).reshape(-1, 2) for p in parts])
    np.testing.assert_array_equal(returned, exp)  # per-slice outputs in rank order = the single output


APP2 = ("define stream StockStream (symbol int, price double, volume long, timestamp long); "
        "@info(name='q') from StockStream[price > 70 and volume < 1000] select timestamp insert into Out;")


def oracle_filter(cols, ts):
    a = OracleApp(APP2)
    a.start()
    cs = [np.ascontiguousarray(c) for c in cols]
    ptrs = (ctypes.c_void_p * len(cs))(*[c.ctypes.data for c in cs])
    err = ctypes.create_string_buffer(512)
    ts = np.ascontiguousarray(ts, dtype=np.int64)
    rc = olib().cr_send_columns(a.h, a.stream_index("StockStream"), len(ts), ts.ctypes.data, ptrs, err, 512)
    assert rc == 0, err.value
    out = a.outputs()["streams"].get("Out", [])
    a.close()
    return np.array([r[1][0] for r in out], dtype=np.int64)  # the selected timestamp = global ordinal


def _worker2(rank, world, port, outfile):
    from siddhi_amd.shard import concat_ordered
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = N * rank // world, N * (rank + 1) // world
        sym, price, vol, tsa, ts = synth.gen_stock(lo, hi, K, 1, synth.seed_for(2))
        kept = oracle_filter([sym, price, vol, tsa], ts)  # the timestamp attribute = global ordinal
        assert ((kept >= lo) & (kept < hi)).all()
        allrows = concat_ordered(torch.from_numpy(kept), world)
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(allrows.tolist(), f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 3])
def test_config2_index_range_shards_concat_equal_single_process(world, tmp_path):
    out = str(tmp_path / "rows.json")
    mp.start_processes(_worker2, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    got = np.asarray(json.load(open(out)), dtype=np.int64)
    sym, price, vol, tsa, ts = synth.gen_stock(0, N, K, 1, synth.seed_for(2))
    exp = oracle_filter([sym, price, vol, tsa], ts)
    assert len(exp) > 1000
    np.testing.assert_array_equal(got, exp)


def test_owner_hash_spreads_structured_keys():
    """Keys that are all multiples of the world size still spread over every rank (a plain key mod world would
    send them all to rank 0), and the owner is a function of the key only."""
    from siddhi_amd.shard import owner_of
    keys = torch.arange(0, 8 * 10000, 8, dtype=torch.int64)
    cnt = torch.bincount(owner_of(keys, 8), minlength=8)
    assert int(cnt.min()) > 1000
    assert torch.equal(owner_of(keys.to(torch.int32), 8), owner_of(keys, 8))
    with pytest.raises(TypeError):
        owner_of(keys.to(torch.float64), 8)


def test_owner_hash_known_values():
    """hi32(splitmix64 finaliser) of a few keys, computed independently with Python integers."""
    from siddhi_amd.shard import owner_of

    def ref(k, world):
        z = k & (2**64 - 1)
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
        z ^= z >> 31
        return (z >> 32) % world
    keys = [0, 1, -1, 7, 123456789, -(2**40) + 3, 2**62 + 11, -(2**63)]
    for w in (2, 3, 7, 8, 64):
        got = owner_of(torch.tensor(keys, dtype=torch.int64), w).tolist()
        assert got == [ref(k, w) for k in keys]


def test_pack_unpack_round_trip():
    from siddhi_amd.shard import pack_by_owner, unpack, owner_of
    g = torch.Generator().manual_seed(3)
    n = 1000
    keys = torch.randint(-50, 50, (n,), generator=g, dtype=torch.int64).to(torch.int32)
    cols = [keys, torch.rand(n, generator=g, dtype=torch.float64), torch.arange(n, dtype=torch.int64),
            torch.randint(0, 255, (n,), generator=g, dtype=torch.uint8), torch.arange(n, dtype=torch.int32)]
    rec, counts, lay = pack_by_owner(keys, cols, 5)
    assert rec.shape == (n, 4)  # 8 + 8 + 4 + 4 + 1 -> 32 bytes
    got = unpack(rec, lay, [c.dtype for c in cols])
    order = torch.argsort(owner_of(keys, 5), stable=True)
    for a, c in zip(got, cols):
        assert torch.equal(a, c[order])
    assert counts == torch.bincount(owner_of(keys, 5), minlength=5).tolist()


def test_order_matches_host():
    from siddhi_amd.shard import order_matches, pack_pairs, unpack_pairs
    runs = [[(1, 10), (3, 10), (2, 12)], [(0, 11), (5, 13), (4, 13)], [(6, 14)]]
    e1 = torch.tensor([p[0] for r in runs for p in r])
    e2 = torch.tensor([p[1] for r in runs for p in r])
    a, b = unpack_pairs(order_matches(pack_pairs(e1, e2), 10, 15))
    assert b.tolist() == [10, 10, 11, 12, 13, 13, 14] and a.tolist() == [1, 3, 0, 2, 5, 4, 6]


def test_merge_keeps_same_trigger_order():
    from siddhi_amd.shard import merge_matches
    a = [[1, 5], [0, 5], [2, 9]]
    b = [[3, 4], [4, 7]]
    np.testing.assert_array_equal(merge_matches([a, b]), [[3, 4], [1, 5], [0, 5], [4, 7], [2, 9]])


# ---- config 5 (five streams, playback timers): key exchange + global clock-advance heartbeats (shard.py
# clock_ticks / merge_heartbeats), then the output merge (shard.merge_outputs: every output to the rank that ingested
# its trigger, ordered there by trigger, timers before the event, timers in instance creation order): the ranks'
# outputs concatenated in rank order must be the single-process output list exactly.
N5, K5 = 20000, 400
BODIES5 = ["every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 1 sec",
           "every e1=A, e2=B[price>e1.price]<1:3>, (e3=C or e4=D), not E for 1 sec"]


def replay5(text, sid, ts, cols):
    """The single-process reference: one oracle app over the whole stream."""
    a = OracleApp(text)
    a.start()
    a.send_interleaved(sid, ts, cols)
    out = a.outputs()["streams"].get("Out", [])
    order = a.output_order("Out")
    a.close()
    return [[r[0], r[1]] for r in out], order


def out_records(order, rank):
    """Output records in the sm_app_copy_device_outputs layout (trigger ordinal, clock step, creation ordinal, ts,
    phase | query << 32, sched | seq << 32, key | pad << 32) + one payload column: (rank << 32) | index."""
    m = len(order)
    rec = torch.zeros((m, 8), dtype=torch.int64)
    if m:
        o = torch.from_numpy(order)
        rec[:, 0], rec[:, 4], rec[:, 1], rec[:, 2] = o[:, 0], o[:, 1], o[:, 2], o[:, 3]
        rec[:, 7] = (rank << 32) | torch.arange(m, dtype=torch.int64)
    return rec


def _worker5(rank, world, port, outfile, body):
    from siddhi_amd.shard import clock_ticks, exchange_by_key, merge_heartbeats, merge_outputs, slice_starts
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
        m_sid, m_ts, m_cols, m_ord = merge_heartbeats(r_sid, r_ts, [r_sym, r_price, r_vol, r_tsa], r_ord, ticks)
        assert (np.diff(m_ts.numpy()) >= 0).all()
        assert (m_ord.numpy()[m_sid.numpy() < 0] >= 0).all(), "a heartbeat carries its trigger's ordinal"
        a = OracleApp(synth.app5(body))
        a.start()
        a.send_interleaved_ord(m_sid.numpy(), m_ts.numpy(), m_ord.numpy(), [c.numpy() for c in m_cols])
        rows = [[r[0], r[1]] for r in a.outputs()["streams"].get("Out", [])]
        order = a.output_order("Out")
        a.close()
        mine = merge_outputs(out_records(order, rank), slice_starts(lo, world, torch.device("cpu")), N5, world)
        assert ((mine[:, 0] >= lo) & (mine[:, 0] < hi)).all(), "an output merged away from its trigger's slice"
        parts = [None] * world
        dist.all_gather_object(parts, [rows, mine[:, 7].tolist()])
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(parts, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("body", BODIES5)
def test_config5_sharded_outputs_merge_to_single_process_order(world, body, tmp_path):
    out = str(tmp_path / "parts5.json")
    mp.start_processes(_worker5, args=(world, _free_port(), out, body), nprocs=world, join=True,
                       start_method="spawn")
    parts = json.load(open(out))
    sid, cols, ts = synth.gen5(0, N5, K5, 1)
    full, order = replay5(synth.app5(body), sid, ts, cols)
    assert len(full) > 30 and (order[:, 1] == 0).any(), "the stream must fire timers"
    merged = [parts[p >> 32][0][p & 0xFFFFFFFF] for r in range(world) for p in parts[r][1]]
    assert merged == full


def test_output_order_key_sorts_single_process_output():
    """The order key itself: the single-process output list is already sorted by (trigger, phase, step, creation)
    with its own records, so order_outputs leaves it unchanged (also on records fed in a shuffled run split)."""
    from siddhi_amd.shard import order_outputs
    sid, cols, ts = synth.gen5(0, N5, K5, 1)
    full, order = replay5(synth.app5(BODIES5[0]), sid, ts, cols)
    rec = out_records(order, 0)
    assert torch.equal(order_outputs(rec)[:, 7], rec[:, 7])
    # two runs (every other creation ordinal's outputs first), each in order: merged back to the single order
    odd = (rec[:, 2] % 2) == 1
    runs = torch.cat([rec[odd], rec[~odd]])
    assert torch.equal(order_outputs(runs)[:, 7], rec[:, 7])


def test_narrow_keys_rejected_consistently():
    """Partition keys are 32- or 64-bit integers on both the host (torch) and the device (sm_partition_by_owner)
    paths: a narrower key has no signedness on the device, so it is refused on both instead of hashed two ways."""
    import pytest as _pt
    from siddhi_amd import shard
    for dt in (torch.int8, torch.uint8, torch.int16):
        with _pt.raises(TypeError):
            shard.owner_of(torch.arange(10, dtype=dt), 3)
        with _pt.raises(TypeError):
            shard.partition_by_owner(torch.arange(10, dtype=dt), [torch.arange(10)], 3)
