"""The device-batch path as a streaming receiver: a stream fed through sm_app_process_device_batch in ragged
pieces must produce exactly the reference's matches for the whole stream. The reference keeps the e2
pre-processor's pending list across InputHandler.send calls (StreamPreStateProcessor.java:208-221 addState,
:268-271 updateState, :274-327 processAndReturn); the product carries each key's open partials across device
batches. Both device pipelines are checked: the bucket-stack kernels (fast_stack=1, path 3) and the sort / walk
kernels (fast_stack=2, path 2), keyed (config 4 shape) and unkeyed (config 3 shape)."""
import numpy as np
import pytest

import synth
from test_device_batch import PART, Q, SCHEMA, app_text, oracle_pairs, stock, value_column

pytestmark = pytest.mark.gpu

SPLITS = [1, 8191, 8193, 33333]


def pieces(n, splits=SPLITS):
    """[lo, hi) ranges: the given ragged lengths, then the rest in one piece."""
    out, lo = [], 0
    for ln in splits:
        if lo >= n:
            break
        out.append((lo, min(n, lo + ln)))
        lo = out[-1][1]
    if lo < n:
        out.append((lo, n))
    return out


def run_stream(text, cols, ts, ranges, ordinals=None, stack=0, expect_path=None):
    """Feed [lo, hi) pieces as device batches; return global (e1, e2) ordinals of every batch's matches in order."""
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text, fast_stack=stack)
    dev = torch.device("cuda", 0)
    got = []
    for lo, hi in ranges:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi], dtype=np.int64)).to(dev)
        if ordinals is not None:
            tord = torch.from_numpy(np.ascontiguousarray(ordinals[lo:hi])).to(dev)
            base = 0
        else:
            tord, base = None, lo
        torch.cuda.synchronize()
        app.process_device_batch("StockStream", tts, tcols, ordinals=tord, ordinal_base=base)
        pr = app.device_matches_host("q")
        if expect_path is not None and hi > lo:
            assert app.get_stat("fast_path:q") == expect_path
        rel = pr.view(np.int32).astype(np.int64)  # e1 of a carried partial is negative (earlier batch)
        got.append(rel + base)
    app.close()
    return np.concatenate(got) if got else np.zeros((0, 2), np.int64)


@pytest.mark.parametrize("stack", [1, 2])
@pytest.mark.parametrize("n,K,div", [(20000, 200, 10), (60000, 50, 3), (120000, 3000, 30)])
def test_partitioned_split_batches(stack, n, K, div):
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n), stack=stack, expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
def test_partitioned_single_batch_both_pipelines(stack):
    n, K, div = 200000, 1000, 100
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, [(0, n)], stack=stack, expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp)


def test_stack_pipeline_automatic_for_many_keys():
    """A key span of more than 2^19 keys takes the bucket-stack kernels by itself (path 3)."""
    n, K, div = 200000, 700000, 1
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n, [77777]), expect_path=3)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("splits", [SPLITS, [5000] * 10, [1] * 50 + [999]])
def test_unpartitioned_split_batches(splits):
    n = 40000
    cols, _ = stock(n, 10, 1, config=1)
    ts = np.arange(n, dtype=np.int64)  # config 1/3: 1 event per ms, a 1000-event window
    text = app_text(partitioned=False)
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n, splits), expect_path=2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("c2", ["price > e1.price", "e1.price <= price", "price < e1.price", "price <= e1.price",
                                "price == e1.price"])
@pytest.mark.parametrize("kind", ["double_ties", "double_special", "float", "int", "long_wide"])
def test_unpartitioned_ordered_compares(c2, kind):
    """Unkeyed walk (config 3 shape) for every ordered compare and value kind (ties, NaN, -0.0, infinities): the
    scans step over 16-record blocks whose extreme value cannot satisfy c2; windows of 1000 / 4000 events, so long
    scans, block skips across the window end and scans past the staged records all occur."""
    n = 30000
    rng = np.random.default_rng(abs(hash((c2, kind))) % (1 << 32))
    vt, price = value_column(kind, n, rng)
    sym = rng.integers(0, 10, n).astype(np.int32)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    tsa = np.arange(n, dtype=np.int64)
    for within, div in ((" within 1 sec", 1), (" within 4 sec", 1), ("", 1)):
        text = (f"define stream StockStream (symbol int, price {vt}, volume long, timestamp long); "
                + Q.format(c1="", c2=c2, within=within))
        cols = [sym, price, vol, tsa]
        exp = oracle_pairs(text, cols, tsa // div)
        got = run_stream(text, cols, tsa // div, pieces(n, [1, 8191, 3333]), expect_path=2)
        np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
@pytest.mark.parametrize("variant", ["no_within", "c2_ge", "c2_lt", "c2_le", "c1_and", "long_keys"])
def test_split_variants(stack, variant):
    n, K, div = 30000, 300, 20
    kw, kd, ko = {}, np.int32, 0
    if variant == "no_within":
        kw["within"] = ""
    elif variant == "c2_ge":
        kw["c2"] = "e1.price <= price"
    elif variant == "c2_lt":
        kw["c2"] = "price < e1.price"
    elif variant == "c2_le":
        kw["c2"] = "price <= e1.price"
    elif variant == "c1_and":
        kw["c1"] = "[price > 30 and volume < 1500]"
    elif variant == "long_keys":
        kw["kt"] = "long"
        kd, ko = np.int64, 1 << 40
    cols, ts = stock(n, K, div, key_dtype=kd, key_offset=ko)
    text = app_text(**kw)
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n), stack=stack, expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
def test_split_with_idle_keys_and_time_gaps(stack):
    """Keys that vanish for several batches keep their partials (only an event of the same key expires them), and
    batches far apart in time expire everything they touch."""
    n, K = 24000, 120
    cols, ts = stock(n, K, 5)
    sym = cols[0]
    sym[8000:16000] = np.where(sym[8000:16000] < 60, sym[8000:16000] + 60, sym[8000:16000])  # keys < 60 idle
    ts = ts.copy()
    ts[12000:] += 5000  # a gap longer than the window
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n, [4000, 4000, 4000, 4000, 1, 3999]), stack=stack,
                     expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
@pytest.mark.parametrize("kind", ["double_ties", "int", "long_narrow", "long_wide", "float"])
def test_split_value_codes(stack, kind):
    n, K, div = 30000, 200, 20
    rng = np.random.default_rng(abs(hash(kind)) % (1 << 32))
    vt, price = value_column(kind, n, rng)
    if vt in ("double", "float"):  # NaN is not an order: the stack kernels hand such batches to the walk kernels
        price = np.where(np.isnan(price), 0, price).astype(price.dtype)
    sym = rng.integers(0, K, n).astype(np.int32)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    tsa = np.arange(n, dtype=np.int64)
    ts = tsa // div
    text = (f"define stream StockStream (symbol int, price {vt}, volume long, timestamp long); "
            + PART.format(q=Q.format(c1="", c2="price > e1.price", within=" within 1 sec")))
    cols = [sym, price, vol, tsa]
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n), stack=stack, expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
def test_split_sharded_ordinals(stack):
    """One rank of a key-sharded stream, fed in pieces with its global ordinals."""
    n, K, div = 60000, 400, 30
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    sym = cols[0]
    sel = np.nonzero(sym % 2 == 1)[0]
    sub = [c[sel] for c in cols]
    got = run_stream(text, sub, ts[sel], pieces(len(sel)), ordinals=sel.astype(np.int64), stack=stack,
                     expect_path=3 if stack == 1 else 2)
    np.testing.assert_array_equal(got, exp[sym[exp[:, 0]] % 2 == 1])


def test_nan_batch_takes_walk_kernels():
    """A NaN compared value is not ordered: the batch leaves the stack kernels for the sort / walk kernels."""
    n, K, div = 20000, 100, 10
    cols, ts = stock(n, K, div)
    cols[1] = cols[1].copy()
    cols[1][::97] = np.nan
    text = (SCHEMA.format(kt="int") + PART.format(q=Q.format(c1="", c2="price > e1.price", within=" within 1 sec")))
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n), stack=1, expect_path=2)
    np.testing.assert_array_equal(got, exp)


def test_stack_equals_walk_large():
    n, K, div = 3_000_000, 20000, 1000
    cols, ts = stock(n, K, div)
    text = app_text()
    a = run_stream(text, cols, ts, [(0, n)], stack=1, expect_path=3)
    b = run_stream(text, cols, ts, [(0, n)], stack=2, expect_path=2)
    np.testing.assert_array_equal(a, b)
    c = run_stream(text, cols, ts, pieces(n, [1_000_003, 999_999]), stack=1, expect_path=3)
    np.testing.assert_array_equal(c, a)


# ---- the NFA hand-over (runtime.cpp nfa_device_batch): when a batch leaves the closed form's premise the general
# NFA kernel takes the query over, carried partials included, and keeps it; outputs stay the reference's.

def _shuffle_times(ts, lo, hi, seed=5):
    """Event time no longer monotone inside [lo, hi): swap a few neighbouring timestamps."""
    ts = ts.copy()
    rng = np.random.default_rng(seed)
    idx = rng.choice(np.arange(lo, hi - 1), size=max(1, (hi - lo) // 50), replace=False)
    for i in idx:
        ts[i], ts[i + 1] = ts[i + 1], ts[i]
    assert (np.diff(ts[lo:hi]) < 0).any()
    return ts


@pytest.mark.parametrize("stack", [1, 2])
def test_non_monotone_batch_hands_over_to_nfa(stack):
    n, K, div = 30000, 150, 5
    cols, ts = stock(n, K, div)
    ts = _shuffle_times(ts, 16000, 24000)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text, fast_stack=stack)
    dev = torch.device("cuda", 0)
    got, paths = [], []
    for lo, hi in [(0, 8000), (8000, 16000), (16000, 24000), (24000, 30000)]:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi])).to(dev)
        app.process_device_batch("StockStream", tts, tcols, ordinal_base=lo)
        got.append(app.device_matches_host("q").view(np.int32).astype(np.int64) + lo)
        paths.append(app.get_stat("fast_path:q"))
    app.close()
    assert paths == [3 if stack == 1 else 2] * 2 + [5, 5]  # taken over at the first non-monotone batch, for good
    np.testing.assert_array_equal(np.concatenate(got), exp)


@pytest.mark.parametrize("wide", [False, True])
def test_non_monotone_first_batch_hands_over(wide):
    """A first batch whose event times decrease reaches the NFA with the reference's outputs, also when its keys span
    more than the bucket-stack window (wide: the time check ranks before the key-span answer, so no dense ids are
    assigned to a batch the closed form never takes)."""
    n, K, div = 40000, 300, 5
    cols, ts = stock(n, K, div, key_dtype=np.int64)
    if wide:
        cols[0] = cols[0] * 5_000_011 - 7  # span of about 1.5e9 keys
    ts = _shuffle_times(ts, 30000, 38000)
    text = app_text(kt="long")
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, [(0, 38000), (38000, n)], expect_path=5)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("at", [8192, 8192 + 77, 255, 256, 4095, 37 * 256])
def test_single_time_step_back_is_found(at):
    """One event time lower than its predecessor's, at or off the prep kernel's wave-item and tile boundaries: the
    batch goes to the NFA, outputs stay the reference's."""
    n, K, div = 20000, 100, 4
    cols, ts = stock(n, K, div)
    ts = ts.copy()
    ts[at] = ts[at - 1] - 1
    assert ts[at] < ts[at - 1]
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, [(0, n)], expect_path=5)
    np.testing.assert_array_equal(got, exp)


def test_batch_earlier_than_carried_state_hands_over():
    """A batch whose first event is older than the last carried one (time going back across batches)."""
    n, K, div = 20000, 100, 5
    cols, ts = stock(n, K, div)
    ts = ts.copy()
    ts[10000:] -= 3  # a step back at the batch boundary, monotone afterwards
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, [(0, 10000), (10000, n)])
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("c2", ["price > e1.price and volume < e1.volume", "price > e1.price + 5.0"])
def test_outside_envelope_streams_through_nfa(c2):
    """Conditions outside the v2 kernels' envelope keep their partials across batches through the NFA kernel."""
    n, K, div = 24000, 120, 5
    cols, ts = stock(n, K, div)
    text = app_text(c2=c2)
    exp = oracle_pairs(text, cols, ts)
    got = run_stream(text, cols, ts, pieces(n, [5000, 1, 7000]), expect_path=5)
    np.testing.assert_array_equal(got, exp)


def test_host_events_then_device_batches():
    """Partials opened by host-API events continue into device batches: the host events take the closed form too
    (the app's only query is eligible, §1d), so the device batches continue its carry."""
    import torch
    from siddhi_amd.testing import ProductApp
    n, K, div = 20000, 80, 5
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    app = ProductApp(text)
    app.start()
    h = 7000
    app.send_columns("StockStream", np.ascontiguousarray(ts[:h]), [np.ascontiguousarray(c[:h]) for c in cols])
    app.flush()
    host = np.array([r[2] for r in app.outputs()["streams"].get("OutputStream", [])], dtype=np.int64).reshape(-1, 2)
    dev = torch.device("cuda", 0)
    got = [host]
    for lo, hi in [(h, 15000), (15000, n)]:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi])).to(dev)
        app.process_device_batch("StockStream", tts, tcols, ordinal_base=lo)
        assert app.get_stat("fast_path:q") in (2, 3)
        got.append(app.device_matches_host("q").view(np.int32).astype(np.int64) + lo)
    app.close()
    np.testing.assert_array_equal(np.concatenate(got), exp)


@pytest.mark.parametrize("stack", [1, 2])
def test_snapshot_restore_keeps_carried_partials(stack):
    """SiddhiAppRuntime.snapshot / restore between device batches: the carried partials travel in the snapshot."""
    import torch
    from siddhi_amd.testing import ProductApp
    n, K, div = 20000, 90, 5
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    dev = torch.device("cuda", 0)

    def batch(app, lo, hi):
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi])).to(dev)
        app.process_device_batch("StockStream", tts, tcols, ordinal_base=lo)
        return app.device_matches_host("q").view(np.int32).astype(np.int64) + lo

    a = ProductApp(text, fast_stack=stack)
    first = batch(a, 0, 9000)
    snap = a.snapshot()
    a.close()
    b = ProductApp(text, fast_stack=stack)
    b.restore(snap)
    second = batch(b, 9000, n)
    b.close()
    np.testing.assert_array_equal(np.concatenate([first, second]), exp)


# ---- the bucket-stack kernel's own limits (kernels/stack.hip): a batch that exceeds one of them is re-run on the
# sort / walk kernels (fast_path 2) and must still equal the reference. The reference's pending list is an
# unbounded LinkedList (StreamPreStateProcessor.java:58-59, processAndReturn :274-327), so none of these limits may
# change an output.

def _paths_and_pairs(text, cols, ts, ranges, stack=1):
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text, fast_stack=stack)
    dev = torch.device("cuda", 0)
    got, paths = [], []
    for lo, hi in ranges:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi], dtype=np.int64)).to(dev)
        app.process_device_batch("StockStream", tts, tcols, ordinal_base=lo)
        got.append(app.device_matches_host("q").view(np.int32).astype(np.int64) + lo)
        paths.append(int(app.get_stat("fast_path:q")))
    app.close()
    return np.concatenate(got), paths


def _overwrite(cols, ts, pos, keys, prices, t=None):
    cols[0][pos] = keys
    cols[1][pos] = prices
    if t is not None:
        ts[pos] = t


def test_stack_overflow_long_decreasing_run():
    """SE_OVERFLOW (stack.hip st_push): one key holds more than kC + kQ = 37 live partials (a strictly decreasing
    price run of 60 inside the window), then one event beats them all (60 matches for one e2)."""
    n, K, div = 30000, 100, 10
    cols, ts = stock(n, K, div)
    cols = [c.copy() for c in cols]
    ts = ts.copy()
    seg = cols[0][12000:12201]
    seg[seg == 7] = 8  # key 7 only through the run below inside this stretch
    run = 12000 + 3 * np.arange(60)
    _overwrite(cols, ts, run, 7, 90.0 - 0.5 * np.arange(60))
    _overwrite(cols, ts, np.array([12200]), 7, 99.9)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got, paths = _paths_and_pairs(text, cols, ts, [(0, 10000), (10000, 20000), (20000, n)])
    assert paths[0] == 3 and paths[1] == 2, paths
    assert ((exp[:, 1] == 12200).sum()) >= 60
    np.testing.assert_array_equal(got, exp)


def _many_match_slice(nkeys, depth, n_tail, seed=3):
    """Keys m * 1024 (all in bucket 0, H = 600 in-bucket keys, so 8 match-log slots per thread): the batch opens with
    `depth` rounds of decreasing prices over `nkeys` keys, then one event per key that beats its whole stack (depth
    matches for one e2), all in the first 4608-record slice; a random tail over 600 keys follows."""
    rng = np.random.default_rng(seed)
    keys = np.arange(nkeys, dtype=np.int32) * 1024
    head_k = np.concatenate([np.tile(keys, depth), keys])
    head_p = np.concatenate([np.repeat(80.0 - 0.5 * np.arange(depth), nkeys), np.full(nkeys, 99.5)])
    tail_k = rng.integers(0, 600, n_tail).astype(np.int32) * 1024
    tail_p = rng.random(n_tail) * 100.0
    sym = np.concatenate([head_k, tail_k])
    price = np.concatenate([head_p, tail_p])
    n = len(sym)
    tsa = np.arange(n, dtype=np.int64)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    return [sym, price, vol, tsa], tsa // 20


@pytest.mark.parametrize("nkeys", [40, 200])
def test_stack_match_log_overflow(nkeys):
    """Events that each pop a long run of partials (20 matches for one e2, in every key of a slice). 40 keys spill
    their matches beyond the per-thread log slots into the shared overflow log (kOvf = 1024): the stack kernel keeps
    the batch. 200 keys exceed that log (SE_LOG): the batch goes to the sort / walk kernels (the v3 kernels,
    SM_STACK_V3=1, keep it: their pops go to a per-bucket overflow region)."""
    import os
    depth = 20
    cols, ts = _many_match_slice(nkeys, depth, 20000)
    assert nkeys * (depth + 1) <= 4608
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got, paths = _paths_and_pairs(text, cols, ts, [(0, len(ts))])
    v3 = os.environ.get("SM_STACK_V3", "0") not in ("", "0")
    assert paths == [3 if nkeys == 40 or v3 else 2]
    assert (np.bincount(exp[:, 1]) >= depth).sum() >= nkeys
    np.testing.assert_array_equal(got, exp)


def _pending_tail(K, depth, n_head, seed=4):
    """A random head over K keys, then `depth` rounds of decreasing prices (all above c1's 20) over every key: each key
    ends the batch with more than `depth` pending partials (no `within`: nothing expires)."""
    rng = np.random.default_rng(seed)
    keys = np.arange(K, dtype=np.int32)
    sym = np.concatenate([rng.integers(0, K, n_head).astype(np.int32), np.tile(keys, depth)])
    price = np.concatenate([rng.random(n_head) * 100.0, np.repeat(30.0 - 0.25 * np.arange(depth), K)])
    n = len(sym)
    tsa = np.arange(n, dtype=np.int64)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    return [sym, price, vol, tsa], tsa // 10


def test_stack_carry_candidate_overflow():
    """SE_CAND (stack.hip put_all): 1024 keys (one in-bucket key, H = 1) end the batch with about 20 pending
    partials each, more than the 8 * H * 1024 + 1024 carry-out candidates the stack kernel reserves: the walk
    kernels take the batch, and the carry they leave feeds the next batch."""
    K, depth = 1024, 20
    cols, ts = _pending_tail(K, depth, 6000)
    n = len(ts)
    # a second batch: every key again, beating the carried stacks
    rng = np.random.default_rng(9)
    n2 = 8000
    cols2 = [rng.integers(0, K, n2).astype(np.int32), rng.random(n2) * 100.0, rng.integers(0, 2000, n2),
             np.arange(n, n + n2, dtype=np.int64)]
    cols = [np.concatenate([a, b.astype(a.dtype)]) for a, b in zip(cols, cols2)]
    ts = np.concatenate([ts, np.full(n2, ts[-1], dtype=np.int64) + np.arange(n2) // 10])
    text = app_text(within="")
    exp = oracle_pairs(text, cols, ts)
    got, paths = _paths_and_pairs(text, cols, ts, [(0, n), (n, n + n2)])
    assert paths[0] == 2, paths
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("stack", [1, 2])
def test_spilled_stacks_carried_into_key_range(stack):
    """More than kC = 5 pending partials per key (register stack full, entries in the HBM spill ring) at a batch
    end, no `within`, and every carried key inside the next batch's key range: the carry-out takes the one-key-sort
    form (stack.hip build_carry, key_runs_ordered), which relies on put_all writing each key's partials as one
    oldest-first run. Three batches, so a carry is also read back by the stack kernel."""
    K, depth = 120, 12
    cols, ts = _pending_tail(K, depth, 3000)
    n = len(ts)
    parts = [cols]
    tss = [ts]
    for b in range(2):
        rng = np.random.default_rng(20 + b)
        m = 3000
        base = n + b * (m + K * depth)
        k2 = np.concatenate([rng.integers(0, K, m).astype(np.int32), np.tile(np.arange(K, dtype=np.int32), depth)])
        p2 = np.concatenate([rng.random(m) * 100.0, np.repeat(25.0 - 0.25 * np.arange(depth), K)])
        ln = len(k2)
        parts.append([k2, p2, rng.integers(0, 2000, ln), np.arange(base, base + ln, dtype=np.int64)])
        tss.append(np.arange(base, base + ln, dtype=np.int64) // 10)
    cols = [np.concatenate([p[k].astype(parts[0][k].dtype) for p in parts]) for k in range(4)]
    ts = np.concatenate(tss)
    bounds = np.cumsum([0] + [len(t) for t in tss])
    text = app_text(within="")
    exp = oracle_pairs(text, cols, ts)
    got, paths = _paths_and_pairs(text, cols, ts, list(zip(bounds[:-1], bounds[1:])), stack=stack)
    assert paths == [3 if stack == 1 else 2] * 3, paths
    np.testing.assert_array_equal(got, exp)


def _run_unkeyed(text, cols, ts, ranges, ordinals=None):
    """run_stream for the unkeyed walk with phase timing on: the pairs, and whether the j-tile kernel ran."""
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text, fast_stack=2, fast_timing=1)
    dev = torch.device("cuda", 0)
    got, tiled = [], 0
    for lo, hi in ranges:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi], dtype=np.int64)).to(dev)
        tord = None if ordinals is None else torch.from_numpy(np.ascontiguousarray(ordinals[lo:hi])).to(dev)
        base = lo if ordinals is None else 0
        torch.cuda.synchronize()
        app.process_device_batch("StockStream", tts, tcols, ordinals=tord, ordinal_base=base)
        tiled += int(app.get_stat("kernel_calls:j_tile"))
        got.append(app.device_matches_host("q").view(np.int32).astype(np.int64) + base)
    app.close()
    return np.concatenate(got), tiled


@pytest.mark.parametrize("case", ["spikes", "sharded", "window_8s_spikes", "long_wait", "no_within"])
def test_unpartitioned_j_tile_order(case, monkeypatch):
    """Round 6: the unkeyed walk's (e1, e2) pairs put in e2 order by output tiles of 2048 ordinals (fastpath3.hip
    jt_place_kernel) when no match lies more than 8192 ordinals after its e1; otherwise, or when a tile holds more
    than 4096 pairs, by the LSD j passes. Both equal the oracle: price spikes that complete hundreds to thousands of
    partials at one e2 (ties of j, i ascending), sharded ordinals with gaps, ragged batches with carried partials, and
    windows past the tile path's reach."""
    n = 60000
    rng = np.random.default_rng(11)
    price = rng.uniform(21.0, 60.0, n)
    within = " within 1 sec"
    if case in ("spikes", "sharded"):
        price[rng.integers(0, n, n // 300)] = 1000.0  # each spike completes every pending partial of the last second
    if case == "window_8s_spikes":
        within = " within 8 sec"
        price[np.arange(7000, n, 7000)] = 1000.0  # ~7000 partials per spike: more than a tile's workgroup holds
    if case == "long_wait":  # a falling run of 10000 events, then a spike: a match 10000 ordinals after its e1
        within = " within 30 sec"
        price[20000:30000] = np.linspace(59.0, 21.5, 10000)
        price[30000] = 1000.0
    if case == "no_within":
        within = ""
    sym = rng.integers(0, 10, n).astype(np.int32)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    tsa = np.arange(n, dtype=np.int64)
    cols = [sym, price, vol, tsa]
    text = app_text(partitioned=False, within=within)
    exp = oracle_pairs(text, cols, tsa)
    ordinals = None
    if case == "sharded":  # this rank's events carry global ordinals 3 k + 1 (gaps of two)
        ordinals = 3 * np.arange(n, dtype=np.int64) + 1
        exp = 3 * exp + 1
    ranges = [(0, n)] if case == "long_wait" else pieces(n, [1, 8191, 20000])
    got, tiled = _run_unkeyed(text, cols, tsa, ranges, ordinals)
    np.testing.assert_array_equal(got, exp)
    if case in ("spikes", "sharded"):
        assert tiled > 0
    if case == "long_wait":
        assert tiled == 0
    monkeypatch.setenv("SM_JTILE", "0")
    lsd, tiled0 = _run_unkeyed(text, cols, tsa, ranges, ordinals)
    assert tiled0 == 0
    np.testing.assert_array_equal(lsd, exp)
