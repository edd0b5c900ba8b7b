"""Device-batch hot path (sm_app_process_device_batch) against the CPU oracle on the §8(d) synthetic stream:
the closed-form every/within kernels (onesweep form and general form) must return exactly the reference's
ordered (e1, e2) match tuples. Sizes are small enough for the oracle; full-size runs are checked through
size-independent properties (order, per-pair conditions, both kernel forms agree)."""
import ctypes

import numpy as np
import pytest

import synth
from oracle_lib import OracleApp, lib as olib

pytestmark = pytest.mark.gpu

SCHEMA = "define stream StockStream (symbol {kt}, price double, volume long, timestamp long); "
PART = "partition with (symbol of StockStream) begin {q} end;"
Q = ("@info(name='q') from every e1=StockStream{c1} -> e2=StockStream[{c2}]{within} "
     "select e1.timestamp as i, e2.timestamp as j insert into OutputStream;")


def app_text(partitioned=True, c1="[price>20]", c2="price>e1.price", within=" within 1 sec", kt="int"):
    q = Q.format(c1=c1, c2=c2, within=within)
    return SCHEMA.format(kt=kt) + (PART.format(q=q) if partitioned else q)


def oracle_pairs(text, cols, ts):
    a = OracleApp(text)
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


def device_pairs(text, cols, ts, ordinals=None, general=False):
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text)
    if general:
        app.set_option("fast_general", 1)
    dev = torch.device("cuda", 0)
    tcols = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    tts = torch.from_numpy(np.ascontiguousarray(ts, dtype=np.int64)).to(dev)
    tord = torch.from_numpy(ordinals).to(dev) if ordinals is not None else None
    torch.cuda.synchronize()
    app.process_device_batch("StockStream", tts, tcols, ordinals=tord, ordinal_base=0)
    out = app.device_matches_host("q").astype(np.int64)
    path = app.get_stat("fast_path:q")
    app.close()
    return out, path


def stock(n, K, ts_div, config=4, key_dtype=np.int32, key_offset=0):
    sym, price, vol, tsa, ts = synth.gen_stock(0, n, K, ts_div, synth.seed_for(config))
    sym = sym.astype(key_dtype) + key_dtype(key_offset)
    return [sym, price, vol, tsa], ts


@pytest.mark.parametrize("n,K,div", [(1, 4, 1), (2, 1, 1), (64, 3, 1), (8191, 50, 3), (8193, 50, 3),
                                     (20000, 200, 10), (200000, 1000, 100)])
def test_partitioned_matches_oracle(n, K, div):
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    got, path = device_pairs(text, cols, ts)
    assert path == 2
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("n", [1, 1000, 20000])
def test_unpartitioned_matches_oracle(n):
    cols, _ = stock(n, 10, 1, config=1)
    ts = np.arange(n, dtype=np.int64)  # config 1/3: 1 event per ms
    text = app_text(partitioned=False)
    exp = oracle_pairs(text, cols, ts)
    got, path = device_pairs(text, cols, ts)
    assert path == 2
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("variant", ["long_keys", "negative_keys", "c1_and", "c2_const", "no_within",
                                     "no_c1", "two_attrs", "c2_ge"])
def test_variants_match_oracle(variant):
    n, K, div = 30000, 300, 20
    kw = {}
    kd, ko = np.int32, 0
    expect_path = 2
    if variant == "long_keys":
        kw["kt"] = "long"
        kd, ko = np.int64, 1 << 40
    elif variant == "negative_keys":
        ko = -150
    elif variant == "c1_and":
        kw["c1"] = "[price > 30 and volume < 1500]"
    elif variant == "c2_const":
        kw["c2"] = "price > e1.price + 5.0"
        expect_path = 5  # not a fixed compare of the carried attribute: the NFA kernel takes the query
    elif variant == "no_within":
        kw["within"] = ""
    elif variant == "no_c1":
        kw["c1"] = ""
    elif variant == "two_attrs":
        kw["c2"] = "price > e1.price and volume < e1.volume"
        expect_path = 5
    elif variant == "c2_ge":
        kw["c2"] = "e1.price <= price"
    cols, ts = stock(n, K, div, key_dtype=kd, key_offset=ko)
    text = app_text(**kw)
    exp = oracle_pairs(text, cols, ts)
    got, path = device_pairs(text, cols, ts)
    assert path == expect_path
    np.testing.assert_array_equal(got, exp)


def test_sharded_ordinals_match_oracle_subset():
    """One rank of a key-sharded run: events of the keys it owns, with their global ordinals."""
    n, K, div = 100000, 400, 50
    cols, ts = stock(n, K, div)
    text = app_text()
    exp = oracle_pairs(text, cols, ts)
    sym = cols[0]
    for world in (2, 3):
        for rank in range(world):
            sel = np.nonzero(sym % world == rank)[0]
            sub = [c[sel] for c in cols]
            got, path = device_pairs(text, sub, ts[sel], ordinals=sel.astype(np.int64))
            mine = exp[sym[exp[:, 0]] % world == rank]
            np.testing.assert_array_equal(got, mine)


def test_onesweep_equals_general_large():
    n, K, div = 3_000_000, 20000, 1000
    cols, ts = stock(n, K, div)
    text = app_text()
    a, pa = device_pairs(text, cols, ts)
    b, pb = device_pairs(text, cols, ts, general=True)
    assert (pa, pb) == (2, 1)
    np.testing.assert_array_equal(a, b)


def test_full_size_properties():
    """Config 4 at K = 1e6 keys, 5e7 events: reference order, per-pair conditions, first-match property."""
    n, K, div = 50_000_000, 1_000_000, 10000
    cols, ts = stock(n, K, div)
    got, path = device_pairs(app_text(), cols, ts)
    assert path == 3  # K = 1e6 keys: the bucket-stack kernels
    i, j = got[:, 0], got[:, 1]
    assert len(got) > 0.6 * n
    order = np.lexsort((i, j))
    assert (order == np.arange(len(got))).all(), "output not ordered by (e2, e1)"
    sym, price = cols[0], cols[1]
    assert (sym[i] == sym[j]).all() and (price[j] > price[i]).all() and (price[i] > 20).all()
    assert (j > i).all() and (ts[j] - ts[i] <= 1000).all()
    assert len(np.unique(i)) == len(i), "a partial matched twice"
    # first-match property on a sample: no earlier same-key event in (i, j) satisfies c2 within the window
    rng = np.random.default_rng(1)
    for k in rng.choice(len(got), 200, replace=False):
        a, b = i[k], j[k]
        seg = np.arange(a + 1, b)
        seg = seg[sym[seg] == sym[a]]
        assert not (price[seg] > price[a]).any()


VALUE_KINDS = ["double_ties", "double_special", "float", "int", "long_narrow", "long_wide"]


def value_column(kind, n, rng):
    """Compared-attribute columns that exercise the keyed records' value codes: exact codes (INT, FLOAT, narrow
    LONG), high-half codes with ties resolved from the exact column values (DOUBLE, wide LONG), NaN and -0.0."""
    if kind == "double_ties":  # many values share the high 32 bits of their order-preserving image
        return ("double", 50.0 + rng.integers(0, 9, n).astype(np.float64) * 1e-9)
    if kind == "double_special":
        pool = np.array([np.nan, -0.0, 0.0, 1.0, -1.0, np.inf, -np.inf, 2.5], dtype=np.float64)
        return ("double", pool[rng.integers(0, len(pool), n)])
    if kind == "float":
        pool = np.array([np.nan, -0.0, 0.0, 1.5, -2.25, 3.0, np.inf], dtype=np.float32)
        return ("float", np.where(rng.random(n) < 0.5, pool[rng.integers(0, len(pool), n)],
                                  rng.normal(0, 10, n)).astype(np.float32))
    if kind == "int":
        return ("int", rng.integers(-50, 50, n).astype(np.int32))
    if kind == "long_narrow":
        return ("long", (rng.integers(0, 1000, n) + (1 << 40)).astype(np.int64))
    # wide LONG range (> 2^32) with ties in the high 32 bits
    return ("long", np.where(rng.random(n) < 0.5, rng.integers(0, 7, n), rng.integers(0, 7, n) + (1 << 45))
            .astype(np.int64) * np.where(rng.random(n) < 0.3, -1, 1))


@pytest.mark.parametrize("op", [">", ">=", "==", "!="])
@pytest.mark.parametrize("kind", VALUE_KINDS)
def test_value_codes_match_oracle(kind, op):
    n, K, div = 40000, 300, 20
    rng = np.random.default_rng(hash((kind, op)) % (1 << 32))
    vt, price = value_column(kind, n, rng)
    sym = rng.integers(0, K, n).astype(np.int32)
    vol = rng.integers(0, 2000, n).astype(np.int64)
    tsa = np.arange(n, dtype=np.int64)
    ts = tsa // div
    text = (f"define stream StockStream (symbol int, price {vt}, volume long, timestamp long); "
            + PART.format(q=Q.format(c1="", c2=f"price {op} e1.price", within=" within 1 sec")))
    cols = [sym, price, vol, tsa]
    exp = oracle_pairs(text, cols, ts)
    got, path = device_pairs(text, cols, ts)
    assert path == 2
    np.testing.assert_array_equal(got, exp)
    # one rank of a key-sharded run: the exact fallback finds rows through the (sorted) ordinals
    sel = np.nonzero(sym % 2 == 1)[0]
    got, _ = device_pairs(text, [c[sel] for c in cols], ts[sel], ordinals=sel.astype(np.int64))
    np.testing.assert_array_equal(got, exp[sym[exp[:, 0]] % 2 == 1])
