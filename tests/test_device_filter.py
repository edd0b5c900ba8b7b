"""Device-batch FilterProcessor (kernels/filter.hip) against the CPU oracle: `from S[cond] select ...` keeps the
rows whose condition holds, in arrival order (FilterProcessor.java:50-62; compare promotion and null / NaN
behaviour of the typed compare executors). The typed conjunction form (fast_path 4) and the interpreter form
(fast_path 3) must both return exactly the oracle's rows; at full size (> 2^31 rows) the kept rows are checked
against torch's own evaluation of the same predicate."""
import ctypes

import numpy as np
import pytest

import synth
from oracle_lib import OracleApp, lib as olib

pytestmark = pytest.mark.gpu

SCHEMA = "define stream StockStream (symbol int, price double, volume long, timestamp long, qty float); "


def app_text(cond):
    return SCHEMA + f"@info(name='q') from StockStream[{cond}] select timestamp insert into Out;"


def columns(n, seed=2, nan_frac=0.0):
    sym, price, vol, tsa, _ = synth.gen_stock(0, n, 50, 1, synth.seed_for(seed))
    rng = np.random.default_rng(seed)
    if nan_frac:
        price = price.copy()
        price[rng.random(n) < nan_frac] = np.nan
    qty = (rng.normal(0, 50, n)).astype(np.float32)
    return [sym, price, vol, tsa, qty]


def oracle_rows(text, cols):
    a = OracleApp(text)
    a.start()
    cs = [np.ascontiguousarray(c) for c in cols]
    ptrs = (ctypes.c_void_p * len(cs))(*[c.ctypes.data for c in cs])
    err = ctypes.create_string_buffer(512)
    ts = np.arange(len(cols[0]), dtype=np.int64)
    rc = olib().cr_send_columns(a.h, a.stream_index("StockStream"), len(ts), ts.ctypes.data, ptrs, err, 512)
    assert rc == 0, err.value
    out = a.outputs()["streams"].get("Out", [])
    a.close()
    return np.array([r[1][0] for r in out], dtype=np.int64)


def device_rows(text, cols, ordinals=None, base=0):
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(text)
    dev = torch.device("cuda", 0)
    tcols = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    tts = torch.arange(len(cols[0]), dtype=torch.int64, device=dev)
    tord = torch.from_numpy(ordinals).to(dev) if ordinals is not None else None
    torch.cuda.synchronize()
    app.process_device_batch("StockStream", tts, tcols, ordinals=tord, ordinal_base=base)
    out = app.device_rows_host("q").astype(np.int64)
    path = app.get_stat("fast_path:q")
    app.close()
    return out, path


CONFIG2 = "price > 70 and volume < 1000"


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4095, 4096, 4097, 100_000, 1_000_003])
def test_config2_matches_oracle(n):
    cols = columns(n)
    text = app_text(CONFIG2)
    exp = oracle_rows(text, cols)
    got, path = device_rows(text, cols)
    assert path == 4
    np.testing.assert_array_equal(got, exp)


TYPED = ["qty < 3L", "price > 70", "price >= 50.5", "price < 10", "price <= 0.5", "price == 25", "price != 25",
         "70 < price", "1000 > volume and price > 30", "volume == 1999", "volume != 7L", "symbol >= 25",
         "symbol < 25.5", "qty > 0", "qty <= -10.25", "qty == 0.0", "qty > 3 and qty < 1000000000000L",
         "price > 10 and volume < 1500 and symbol > 3", "(price > 10 and volume < 1500) and (symbol > 3 and qty < 20)",
         "volume > 100.5", "symbol == 7", "timestamp >= 500"]
INTERP = ["price > 70 or volume < 100", "not (price > 50)", "price > volume", "price + 1 > 50",
          "price > 10 and volume < 1500 and symbol > 3 and qty < 20 and timestamp > 9"]


@pytest.mark.parametrize("cond", TYPED + INTERP)
def test_predicates_match_oracle(cond):
    cols = columns(30_000, seed=3, nan_frac=0.05)
    text = app_text(cond)
    exp = oracle_rows(text, cols)
    got, path = device_rows(text, cols)
    assert path == (4 if cond in TYPED else 3)
    np.testing.assert_array_equal(got, exp)


def test_explicit_ordinals():
    """A shard of the stream with its global ordinals: kept rows come back as ordinal - base."""
    cols = columns(50_000, seed=4)
    text = app_text(CONFIG2)
    exp = oracle_rows(text, cols)
    sel = np.nonzero(np.arange(50_000) % 3 == 1)[0]
    got, _ = device_rows(text, [c[sel] for c in cols], ordinals=(sel + 1000).astype(np.int64), base=1000)
    np.testing.assert_array_equal(got, exp[exp % 3 == 1])


def test_empty_and_none_kept():
    cols = columns(10_000, seed=5)
    got, _ = device_rows(app_text("price > 1000"), cols)
    assert len(got) == 0
    got, _ = device_rows(app_text("price >= 0"), cols)
    np.testing.assert_array_equal(got, np.arange(10_000))


def test_full_size_beyond_2pow31():
    """2^31 + 4099 rows: the kept rows equal torch's own evaluation of the predicate (u32 rows past 2^31)."""
    import torch
    from siddhi_amd.testing import ProductApp
    n = (1 << 31) + 4099
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    price = torch.rand(n, dtype=torch.float64, device=dev, generator=g) * 100.0
    volume = torch.randint(0, 2000, (n,), dtype=torch.int64, device=dev, generator=g)
    sym = torch.zeros(1, dtype=torch.int32, device=dev).expand(n)
    ts = torch.zeros(1, dtype=torch.int64, device=dev).expand(n)
    qty = torch.zeros(1, dtype=torch.float32, device=dev).expand(n)
    app = ProductApp(app_text(CONFIG2))
    app.process_device_batch("StockStream", ts, [sym, price, volume, ts, qty])
    p, m = app.device_matches("q")
    assert m > 0.1 * n
    got = torch.empty(m, dtype=torch.int32, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    torch.cuda.synchronize()
    assert hip.hipMemcpy(got.data_ptr(), p, m * 4, 3) == 0  # device to device
    got = got.to(torch.int64) & 0xFFFFFFFF
    pos, step = 0, 1 << 28  # torch.nonzero in chunks (one call over > 2^31 elements is not supported)
    for c0 in range(0, n, step):
        c1 = min(n, c0 + step)
        exp = torch.nonzero((price[c0:c1] > 70) & (volume[c0:c1] < 1000)).squeeze(1) + c0
        assert torch.equal(got[pos:pos + exp.numel()], exp), f"rows differ in [{c0}, {c1})"
        pos += exp.numel()
    assert pos == m
    app.close()
