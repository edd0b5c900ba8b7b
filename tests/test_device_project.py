"""On-device projection of the closed form's outputs (sm_app_device_project): the select
list of every (e1, e2) match of a device batch, evaluated on the GPU (QuerySelector.processNoGroupBy,
core/query/selector/QuerySelector.java:124-167) instead of returning index pairs for a host gather. The stream is fed
in ragged device batches, so matches whose e1 was carried from an earlier batch read the carried partial's values.
Every output's values and timestamp must equal the oracle's Event.data for the whole stream (doubles bit-exact)."""
import ctypes

import numpy as np
import pytest

from oracle_lib import OracleApp, lib as olib
from test_device_batch import PART, SCHEMA, stock
from test_device_stream import pieces

pytestmark = pytest.mark.gpu

SELECT = ("select e1.symbol as k, e1.price as p1, e2.price as p2, e2.volume - e1.volume as dv, "
          "e1.timestamp as i, e2.timestamp as j, e2.price > 50.0 as hi, e1.price / e2.volume as r")
TYPES = ["INT", "DOUBLE", "DOUBLE", "LONG", "LONG", "LONG", "BOOL", "DOUBLE"]


def text(partitioned=True):
    q = ("@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
         + SELECT + " insert into OutputStream;")
    return SCHEMA.format(kt="int") + (PART.format(q=q) if partitioned else q)


def oracle_outputs(app_text, cols, ts):
    a = OracleApp(app_text)
    a.start()
    cs = [np.ascontiguousarray(c) for c in cols]
    ptrs = (ctypes.c_void_p * len(cs))(*[c.ctypes.data for c in cs])
    err = ctypes.create_string_buffer(512)
    t = np.ascontiguousarray(ts, dtype=np.int64)
    assert olib().cr_send_columns(a.h, a.stream_index("StockStream"), len(t), t.ctypes.data, ptrs, err, 512) == 0
    out = a.outputs()["streams"].get("OutputStream", [])
    a.close()
    return out


def as_python(vals, nulls):
    """Device rows (raw 64-bit words) -> the oracle dump's Python values."""
    rows = []
    for r, nr in zip(vals.tolist(), nulls.tolist()):
        row = []
        for w, isnull, ty in zip(r, nr, TYPES):
            if isnull:
                row.append(None)
            elif ty == "DOUBLE":
                row.append(float(np.array([w], dtype=np.int64).view(np.float64)[0]))
            elif ty == "BOOL":
                row.append(bool(w))
            else:
                row.append(int(w))
        rows.append(row)
    return rows


def run(app_text, cols, ts, ranges, stack):
    import torch
    from siddhi_amd.testing import ProductApp
    app = ProductApp(app_text, fast_stack=stack)
    dev = torch.device("cuda", 0)
    got = []
    for lo, hi in ranges:
        tcols = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        tts = torch.from_numpy(np.ascontiguousarray(ts[lo:hi], dtype=np.int64)).to(dev)
        torch.cuda.synchronize()
        app.process_device_batch("StockStream", tts, tcols, ordinal_base=lo)
        vals, nulls, ots = app.device_project("q")  # the batch's columns are still resident
        torch.cuda.synchronize()
        for row, t in zip(as_python(vals.cpu(), nulls.cpu()), ots.cpu().tolist()):
            got.append([t, row])
    app.close()
    return got


@pytest.mark.parametrize("stack", [1, 2])
@pytest.mark.parametrize("n,K,div,splits", [(20000, 200, 10, [1, 8191, 8193]), (60000, 50, 3, [5000] * 11),
                                            (120000, 3000, 30, [33333])])
def test_projection_equals_oracle(stack, n, K, div, splits):
    cols, ts = stock(n, K, div)
    t = text()
    exp = [[o[0], o[1]] for o in oracle_outputs(t, cols, ts)]
    got = run(t, cols, ts, pieces(n, splits), stack)
    assert len(exp) > 100
    assert got == exp


def test_projection_unpartitioned():
    n = 30000
    cols, _ = stock(n, 10, 1, config=1)
    ts = np.arange(n, dtype=np.int64)
    t = text(partitioned=False)
    exp = [[o[0], o[1]] for o in oracle_outputs(t, cols, ts)]
    got = run(t, cols, ts, pieces(n, [7000, 7001]), 0)
    assert got == exp


def test_projection_of_filter_queries():
    """A filter query's device batch: each kept row's select list (FilterProcessor → QuerySelector on one event)."""
    import torch
    from siddhi_amd.testing import ProductApp
    t = SCHEMA.format(kt="int") + ("@info(name='q') from StockStream[price > 50] select symbol, price * 2 as p2, "
                                   "timestamp insert into O;")
    cols, ts = stock(5000, 5, 1)
    app = ProductApp(t)
    dev = torch.device("cuda", 0)
    tts = torch.from_numpy(ts.astype(np.int64)).to(dev)
    tcols = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]  # read again by the projection
    app.process_device_batch("StockStream", tts, tcols)
    vals, nulls, ots = app.device_project("q")
    app.close()
    sel = np.nonzero(cols[1] > 50)[0]
    v = vals.cpu().numpy()
    assert v.shape[0] == len(sel) and not nulls.any()
    np.testing.assert_array_equal(v[:, 0], cols[0][sel])
    np.testing.assert_array_equal(v[:, 1].view(np.float64), cols[1][sel] * 2)
    np.testing.assert_array_equal(v[:, 2], cols[3][sel])
    np.testing.assert_array_equal(ots.cpu().numpy(), ts[sel])


def test_projection_after_host_events():
    """Host-API events of an app whose queries all take the device-batch path run there (flush_device), so their
    outputs can be projected like a device batch's; a host batch the device path cannot take (a null value) runs on
    the host-staged path and leaves nothing to project."""
    import torch
    from siddhi_amd.testing import EngineError, ProductApp
    app = ProductApp(SCHEMA.format(kt="int") + "@info(name='q') from StockStream[price > 50] select price insert into O;")
    app.start()
    types = ["INT", "DOUBLE", "LONG", "LONG"]
    app.send("StockStream", 1, [1, 60.0, 1, 0], types)
    app.send("StockStream", 2, [1, 40.0, 1, 0], types)
    app.send("StockStream", 3, [1, 70.5, 1, 0], types)
    app.flush()
    vals, nulls, ts = app.device_project("q")
    assert vals[:, 0].cpu().view(torch.float64).tolist() == [60.0, 70.5] and ts.tolist() == [1, 3]
    app.send("StockStream", 4, [1, 80.0, None, 0], types)
    app.flush()
    with pytest.raises(EngineError):
        app.device_project("q")
    app.close()
