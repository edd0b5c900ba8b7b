"""Any partition-key domain on the closed-form path (VERDICT r03 missing #4). The reference keys a partition by any
value (ValuePartitionExecutor core/partition/executor/ValuePartitionExecutor.java:34-39; its partition benchmark keys
by a string symbol). The product maps each batch's keys to dense ids on the device (remap_keys: a persistent device
hash map, new keys inserted by the lookup kernel itself), so sparse 64-bit ids and key counts from 2^10 to 2^24 stay
on the bucket-stack or sort / walk kernels instead of leaving the closed form. Checked against the CPU oracle on a key
subsample and, in full, against the brute-force statement of the closed form (tests/test_bench_shape.py)."""
import numpy as np
import pytest

import bench
from test_bench_shape import closed_form_torch, oracle_subsample

pytestmark = pytest.mark.gpu

LONG_APP = bench.APP.replace("symbol int", "symbol long")


def sparse_stream(N, K, div, seed=0x5EED0104):
    """bench.py's config-4 stream with each dense symbol replaced by a 64-bit id (splitmix64 of it): K distinct keys
    spread over the whole int64 range."""
    import torch
    d = torch.device("cuda", 0)
    sym, price, vol, tsa, ts = bench.gen_stock(0, N, K, div, d, seed)
    key = bench.splitmix_torch(sym.to(torch.int64) * 7919 + 11)
    torch.cuda.synchronize()
    return sym, key, price, ts


def run(text, key, price, ts, ranges=None, **opts):
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text, **opts)
    app.set_collect(False)
    n = ts.numel()
    outs, paths = [], []
    for lo, hi in (ranges or [(0, n)]):
        app.process_device_batch("StockStream", ts[lo:hi], [key[lo:hi], price[lo:hi], price[lo:hi], price[lo:hi]],
                                 ordinal_base=lo)
        m = app.device_matches("q")[1]
        buf = torch.empty(max(m, 1), dtype=torch.int64, device=ts.device)
        app.copy_device_matches("q", buf)
        torch.cuda.synchronize()
        p = buf[:m]
        e1 = (p & 0xFFFFFFFF).to(torch.int32).to(torch.int64) + lo  # a carried e1 is negative relative to the batch
        outs.append(((p >> 32) + lo) << 32 | e1)
        paths.append(int(app.get_stat("fast_path:q")))
    app.close()
    return torch.cat(outs), paths


@pytest.mark.timeout(600)
def test_million_sparse_64bit_keys_take_bucket_stack():
    """1e6 random 64-bit keys, 2e7 events, 10 events per key per window: the bucket-stack pipeline (path 3), the key
    subsample equal to the oracle, the whole output equal to the brute-force closed form."""
    import torch
    N, K, div = 20_000_000, 1_000_000, 10_000
    sym, key, price, ts = sparse_stream(N, K, div)
    got, paths = run(LONG_APP, key, price, ts)
    assert paths == [3]
    ref = closed_form_torch(key, price, ts, 1000)
    assert ref.numel() == got.numel() > 0.5 * N and torch.equal(ref, got)
    sel = torch.nonzero((sym.to(torch.int64) % 101) == 7).flatten()
    exp = oracle_subsample(LONG_APP, key[sel].cpu().numpy(), price[sel].cpu().numpy(), ts[sel].cpu().numpy(),
                           sel.cpu().numpy())
    e1 = got & 0xFFFFFFFF
    mine = got[(sym[e1].to(torch.int64) % 101) == 7].cpu().numpy()
    assert len(exp) > 10_000
    np.testing.assert_array_equal(np.stack([mine & 0xFFFFFFFF, mine >> 32], 1), exp)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("logk", [10, 16, 20, 22, 24])
def test_key_counts_stay_on_closed_form(logk):
    """2^10 .. 2^24 sparse keys: bucket stack or sort / walk (never the NFA hand-over), the same pipeline the dense
    symbols of the same stream take (sort / walk up to 2^19 keys in a batch, bucket stack above), equal to the brute
    force."""
    import torch
    N = 8_000_000
    sym, key, price, ts = sparse_stream(N, 1 << logk, 100)
    got, paths = run(LONG_APP, key, price, ts)
    _, dense_paths = run(bench.APP, sym, price, ts)
    assert paths[0] in (2, 3) and paths == dense_paths, (paths, dense_paths)
    ref = closed_form_torch(key, price, ts, 1000)
    assert torch.equal(ref, got)


@pytest.mark.timeout(600)
def test_dense_ids_persist_across_batches_and_snapshots():
    """Ragged batches carry partials whose keys are dense ids; a snapshot between batches restores the id map."""
    import torch
    from siddhi_amd.testing import ProductApp
    N, K, div = 3_000_000, 200_000, 1000
    sym, key, price, ts = sparse_stream(N, K, div)
    whole, _ = run(LONG_APP, key, price, ts)
    cuts = [0, 1, 77_777, 1_000_003, 1_000_004, 2_222_222, N]
    split, paths = run(LONG_APP, key, price, ts, ranges=list(zip(cuts[:-1], cuts[1:])))
    assert set(paths) <= {2, 3}  # closed form throughout (sort / walk: about 2e5 keys per batch)
    assert torch.equal(split, whole)
    # snapshot after 1e6 events, restore into a fresh runtime, continue
    a = ProductApp(LONG_APP)
    a.set_collect(False)
    h = 1_000_000
    a.process_device_batch("StockStream", ts[:h], [key[:h], price[:h], price[:h], price[:h]])
    first = a.device_matches_host("q").astype(np.int64)
    snap = a.snapshot()
    a.close()
    b = ProductApp(LONG_APP)
    b.set_collect(False)
    b.restore(snap)
    b.process_device_batch("StockStream", ts[h:], [key[h:], price[h:], price[h:], price[h:]], ordinal_base=h)
    second = b.device_matches_host("q").view(np.int32).astype(np.int64) + h
    b.close()
    both = np.concatenate([first, second])
    w = whole.cpu().numpy()
    np.testing.assert_array_equal(both, np.stack([w & 0xFFFFFFFF, w >> 32], 1))


def test_compared_key_attribute_is_not_remapped():
    """c1 on the key attribute itself (`symbol > ...`): the compared attribute keeps its values (no dense ids)."""
    import torch
    from siddhi_amd.testing import ProductApp
    text = LONG_APP.replace("e1=StockStream[price>20]", "e1=StockStream[symbol > 0]").replace(
        "price>e1.price", "symbol >= e1.symbol")
    N, K = 200_000, 5000
    sym, key, price, ts = sparse_stream(N, K, 10)
    got, paths = run(text, key, price, ts)
    assert paths[0] != 5
    exp = oracle_subsample(text, key.cpu().numpy(), price.cpu().numpy(), ts.cpu().numpy(), np.arange(N))
    g = got.cpu().numpy()
    np.testing.assert_array_equal(np.stack([g & 0xFFFFFFFF, g >> 32], 1), exp)


@pytest.mark.timeout(600)
def test_int_keys_wider_than_the_bucket_window_get_ids():
    """INT keys spread over a 2^25-wide span (2^20 keys, every 31st value): within the closed form's 2^30 key window
    but wider than the bucket-stack's 2^20, so the first batch's prep pass reports the span and the keys become dense
    ids (bucket stack, path 3) instead of the sort / walk pipeline; equal to the brute force."""
    import torch
    N, K = 8_000_000, 1 << 20
    sym, _, price, ts = sparse_stream(N, K, 100)
    key = (sym.to(torch.int64) * 31).to(torch.int32)
    got, paths = run(bench.APP, key, price, ts)
    assert paths == [3], paths
    ref = closed_form_torch(key.to(torch.int64), price, ts, 1000)
    assert torch.equal(ref, got)
