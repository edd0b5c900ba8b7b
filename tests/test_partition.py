"""HIP stable partition by owner rank (sm_partition_by_owner), the send side of the multi-GPU key exchange:
identical to a stable sort by owner (shard.owner_of, the splitmix64 key hash) for int32 / int64 keys, negative
keys, ragged sizes and 1/2/4/8-byte columns; the packed-record form and the match-ordering kernel."""
import pytest
import torch

from siddhi_amd.shard import (owner_of, pack_by_owner, partition_by_owner, order_matches, pack_pairs, unpack,
                              unpack_with_ordinals)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 4095, 4097, 100_003, 3_000_000])
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kdt", [torch.int32, torch.int64])
def test_partition_equals_stable_sort(n, world, kdt):
    g = torch.Generator().manual_seed(n * 31 + world)
    keys = torch.randint(-10**6, 10**6, (n,), generator=g, dtype=torch.int64).to(kdt)
    cols = [keys.clone(), torch.rand(n, generator=g, dtype=torch.float64), torch.arange(n, dtype=torch.int64),
            torch.randint(0, 5, (n,), generator=g, dtype=torch.int32), torch.randint(0, 255, (n,), generator=g,
                                                                                    dtype=torch.uint8),
            torch.randint(0, 999, (n,), generator=g, dtype=torch.int16)]
    dev = torch.device("cuda", 0)
    got, counts = partition_by_owner(keys.to(dev), [c.to(dev) for c in cols], world)
    owner = owner_of(keys, world)
    order = torch.argsort(owner, stable=True)
    assert counts == torch.bincount(owner, minlength=world).tolist()
    for a, c in zip(got, cols):
        assert torch.equal(a.cpu(), c[order])
    rec, pc, lay = pack_by_owner(keys.to(dev), [c.to(dev) for c in cols], world)
    assert pc == counts
    rec_h, _, _ = pack_by_owner(keys, cols, world)  # the torch (gloo / CPU) form
    if n:
        assert torch.equal(rec.cpu().view(torch.uint8).view(n, -1)[:, :sum(w for _, w in lay)],
                           rec_h.view(torch.uint8).view(n, -1)[:, :sum(w for _, w in lay)])
    for a, c in zip(unpack(rec, lay, [c.dtype for c in cols]), cols):
        assert torch.equal(a.cpu(), c[order])


def test_partition_rejects_float_keys():
    dev = torch.device("cuda", 0)
    with pytest.raises(TypeError):
        partition_by_owner(torch.rand(10, device=dev), [torch.rand(10, device=dev)], 2)


@pytest.mark.parametrize("n_src,per", [(1, 1000), (3, 50000), (8, 200000)])
def test_order_matches_kernel_equals_stable_sort(n_src, per):
    """sm_order_matches over runs the way return_matches receives them (each run e2-ordered, an e2's tuples in
    one run) equals a stable sort by e2."""
    g = torch.Generator().manual_seed(n_src * 7 + per)
    lo, hi = 1000, 1000 + 4 * per * n_src
    e2all = torch.randperm(hi - lo, generator=g)[:per * n_src] + lo
    runs = []
    for r in range(n_src):
        e2 = torch.sort(e2all[r::n_src]).values
        rep = torch.randint(1, 4, (e2.numel(),), generator=g)
        e2 = torch.repeat_interleave(e2, rep)
        e1 = e2 - torch.randint(1, 900, (e2.numel(),), generator=g)
        # within one e2, e1 in reference order (arbitrary but fixed): keep generation order
        runs.append(pack_pairs(e1, e2))
    pairs = torch.cat(runs)
    exp = pairs[torch.argsort(pairs >> 32, stable=True)]
    got = order_matches(pairs.to(torch.device("cuda", 0)), lo, hi)
    assert torch.equal(got.cpu(), exp)


@pytest.mark.parametrize("n,m,overlap", [(0, 5, 0.0), (7, 0, 0.0), (1000, 300, 0.3), (200_000, 50_000, 0.5)])
def test_merge_heartbeats_hip_equals_torch(n, m, overlap):
    """sm_merge_heartbeats (HIP merge path) = the torch form of shard.merge_heartbeats: a rank's events (ascending
    global ordinals) with the global clock-advance points, a point at an ordinal the rank holds dropped."""
    from siddhi_amd.shard import merge_heartbeats
    g = torch.Generator().manual_seed(n + m)
    ords = torch.sort(torch.randperm(4 * (n + m) + 8, generator=g)[:n].to(torch.int64)).values
    held = ords[torch.randperm(n, generator=g)[:int(overlap * min(n, m))]] if n else torch.zeros(0, dtype=torch.int64)
    others = torch.randperm(4 * (n + m) + 8, generator=g)[:m - held.numel()].to(torch.int64)
    tord = torch.unique(torch.cat([held, others]))
    ticks = torch.stack([tord, tord // 3 + 7], 1)
    sid = torch.randint(0, 5, (n,), generator=g, dtype=torch.int32)
    ts = ords // 3
    cols = [torch.randint(-100, 100, (n,), generator=g, dtype=torch.int32), torch.rand(n, generator=g,
                                                                                      dtype=torch.float64)]
    want = merge_heartbeats(sid, ts, cols, ords, ticks)
    dev = torch.device("cuda", 0)
    got = merge_heartbeats(sid.to(dev), ts.to(dev), [c.to(dev) for c in cols], ords.to(dev), ticks.to(dev))
    for a, b in zip([got[0], got[1], got[3]] + got[2], [want[0], want[1], want[3]] + want[2]):
        assert torch.equal(a.cpu(), b)
    assert got[0].numel() == n + tord.numel() - torch.isin(tord, ords).sum().item()


@pytest.mark.parametrize("n,world", [(1, 1), (1000, 3), (300_001, 8), (70_000, 64)])
def test_unpack_with_ordinals_hip_equals_torch(n, world):
    """sm_unpack_records (one pass over the received packed records: columns + global ordinals) against the torch
    unpack + ordinal arithmetic of the same records, on records packed by the partition kernel."""
    d = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(n + world)
    sym = torch.randint(-2**31, 2**31 - 1, (n,), generator=g, dtype=torch.int64).to(torch.int32).to(d)
    price = torch.rand(n, generator=g, dtype=torch.float64).to(d)
    ts = torch.randint(0, 2**40, (n,), generator=g, dtype=torch.int64).to(d)
    off = torch.randint(0, 2**32 - 1, (n,), generator=g, dtype=torch.int64).to(torch.int32).to(d)
    cols = [sym, price, ts, off]
    rec, counts, lay = pack_by_owner(sym, cols, world)
    starts = [int(x) for x in torch.randint(0, 2**50, (world,), generator=g, dtype=torch.int64)]
    got_cols, got_ord = unpack_with_ordinals(rec, lay, [c.dtype for c in cols], counts, starts)
    exp = unpack(rec, lay, [c.dtype for c in cols])
    for a, b in zip(got_cols, exp[:-1]):
        assert torch.equal(a, b)
    base = torch.repeat_interleave(torch.tensor(starts, dtype=torch.int64), torch.tensor(counts, dtype=torch.int64))
    assert torch.equal(got_ord.cpu(), base + exp[-1].cpu().to(torch.int64) % 2**32)


# ---- config 5 across ranks: each rank's device-events batch (its keys' events with their global
# ordinals, plus the global clock advances as heartbeats) exports its output records with their triggers' global
# ordinals (sm_app_copy_device_outputs); sending each record to its trigger's slice and ordering there
# (sm_order_outputs) must give exactly the single app's records, in its order. Ranks are simulated on one GPU.
BODIES5 = ["every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 1 sec",
           "every e1=A, e2=B[price>e1.price]<1:3>, (e3=C or e4=D), not E for 1 sec"]


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("body", BODIES5)
def test_config5_rank_outputs_merge_to_single_app(world, body):
    import synth
    from siddhi_amd.shard import clock_ticks, merge_heartbeats, order_outputs, owner_of
    from siddhi_amd.testing import ProductApp
    d = torch.device("cuda", 0)
    N, K = 30000, 500
    sid, cols, ts = synth.gen5(0, N, K, 1)
    text = synth.app5(body)
    t_sid = torch.from_numpy(sid).to(d)
    t_ts = torch.from_numpy(ts).to(d)
    t_cols = [torch.from_numpy(c).to(d) for c in cols]
    ords = torch.arange(N, dtype=torch.int64, device=d)

    def run(s, t, c, o):
        app = ProductApp(text, keep_outputs=1)
        app.start()
        torch.cuda.synchronize()
        app.process_device_events(s, t, c, ordinals=o)
        recs = app.copy_device_outputs("q")
        app.close()
        return recs

    full = run(t_sid, t_ts, t_cols, ords)
    assert full.shape[0] > 30 and bool(((full[:, 4] & 0xFFFFFFFF) == 0).any()), "the stream must fire timers"
    ticks = clock_ticks(t_ts, 0, 1)
    per_rank = []
    for r in range(world):
        mine = owner_of(t_cols[0], world) == r
        m = merge_heartbeats(t_sid[mine], t_ts[mine], [c[mine] for c in t_cols], ords[mine], ticks)
        per_rank.append(run(m[0], m[1], m[2], m[3]))
    starts = [N * r // world for r in range(world)] + [N]
    got = []
    for dst in range(world):  # what rank dst receives: each source's records of its slice, in rank order
        runs = [rec[(rec[:, 0] >= starts[dst]) & (rec[:, 0] < starts[dst + 1])] for rec in per_rank]
        got.append(order_outputs(torch.cat(runs)))
    got = torch.cat(got)
    keep = [c for c in range(full.shape[1]) if c != 6]  # column 6: key slot (differs between apps) | pad
    assert torch.equal(got[:, keep], full[:, keep])
