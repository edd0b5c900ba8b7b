"""Snapshot / restore of the device matching state (sm_app_snapshot / sm_app_restore), the counterpart of
SiddhiAppRuntime.snapshot() :548 / restore(byte[]) :560 and of the reference's PersistenceTestCase
(modules/siddhi-core/src/test/java/org/wso2/siddhi/core/managment/PersistenceTestCase.java:150-240): a run
split at a snapshot, restored into a fresh runtime of the same app, emits exactly the outputs of the
uninterrupted run (checked against the CPU oracle) — partial matches, count chains, pending `not … for` timers,
partition instances, the playback clock and string values all carry over."""
import numpy as np
import pytest

import synth
from oracle_lib import OracleApp

pytestmark = pytest.mark.gpu

PERSIST_APP = ("define stream Stream1 (symbol string, price float, volume int); "
               "define stream Stream2 (symbol string, price float, volume int); "
               "@info(name = 'query1') from e1=Stream1[price>20] <2:5> -> e2=Stream2[price>20] "
               "select e1[0].price as price1_0, e1[1].price as price1_1, e1[2].price as price1_2, "
               "e1[3].price as price1_3, e2.price as price2 insert into OutputStream ;")
TYPES = ["STRING", "FLOAT", "INT"]


def _product(text):
    from siddhi_amd.testing import ProductApp
    a = ProductApp(text)
    a.start()
    return a


def test_persistence_testcase_count_pattern():
    # PersistenceTestCase.persistenceTest1: three Stream1 events, persist, restart, one Stream2 event
    first = [("Stream1", ["WSO2", 25.6, 100]), ("Stream1", ["GOOG", 47.6, 100]), ("Stream1", ["GOOG", 13.7, 100])]
    second = [("Stream2", ["IBM", 45.7, 100])]
    a = _product(PERSIST_APP)
    for t, (sid, row) in enumerate(first):
        a.send(sid, 100 * t, row, TYPES)
    snap = a.snapshot()
    assert a.outputs()["streams"].get("OutputStream", []) == []
    a.close()
    b = _product(PERSIST_APP)
    b.restore(snap)
    for t, (sid, row) in enumerate(second):
        b.send(sid, 1000 + 100 * t, row, TYPES)
    b.flush()
    out = b.outputs()["streams"]["OutputStream"]
    b.close()
    o = OracleApp(PERSIST_APP)
    o.start()
    for t, (sid, row) in enumerate(first):
        o.send(sid, 100 * t, row, TYPES)
    for t, (sid, row) in enumerate(second):
        o.send(sid, 1000 + 100 * t, row, TYPES)
    o.flush()
    exp = o.outputs()["streams"]["OutputStream"]
    assert len(out) == 1 and out == exp
    assert [round(v, 1) if v is not None else None for v in out[0][1]] == [25.6, 47.6, None, None, 45.7]


@pytest.mark.parametrize("body,split", [
    ("every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 5 sec", 41_111),
    ("every e1=A, e2=B[price>e1.price]<1:3>, (e3=C or e4=D), not E for 1 sec", 50_000),
    ("every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C and e4=D) within 2 sec", 12_345),
])
def test_split_run_equals_uninterrupted(body, split):
    import torch
    sid, cols, ts = synth.gen5(0, 100_000, 2000, 1)
    text = synth.app5(body)
    o = OracleApp(text)
    o.start()
    o.send_interleaved(sid, ts, cols)
    o.flush()
    exp = o.outputs()["streams"].get("Out", [])
    assert len(exp) > 100
    dev = torch.device("cuda", 0)

    def batch(app, lo, hi):
        t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
        app.process_device_events(t(sid[lo:hi]), t(ts[lo:hi]), [t(c[lo:hi]) for c in cols], ordinal_base=lo)

    a = _product(text)
    batch(a, 0, split)
    snap = a.snapshot()
    first = a.outputs()["streams"].get("Out", [])
    a.close()
    b = _product(text)
    b.restore(snap)
    batch(b, split, len(ts))
    b.flush()
    second = b.outputs()["streams"].get("Out", [])
    # restoring into the SAME runtime rewinds it: replaying the second half repeats exactly its outputs
    b.restore(snap)
    batch(b, split, len(ts))
    b.flush()
    again = b.outputs()["streams"].get("Out", [])[len(second):]
    b.close()
    assert first + second == exp
    assert len(first) > 0 and len(second) > 0
    assert again == second


def test_restore_rejects_other_app():
    from siddhi_amd.testing import EngineError
    a = _product(PERSIST_APP)
    snap = a.snapshot()
    a.close()
    b = _product(PERSIST_APP.replace("price>20", "price>21"))
    with pytest.raises(EngineError):
        b.restore(snap)
    with pytest.raises(EngineError):
        b.restore(b"not a snapshot")
    b.close()
