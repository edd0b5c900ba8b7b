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
    """Partials opened by host-API events (NFA state) continue into device batches."""
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
        assert app.get_stat("fast_path:q") == 5
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
