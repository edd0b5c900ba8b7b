"""Query chaining and partition inner streams on the GPU engine against the CPU oracle: a query's output events go
on to the queries reading its stream, depth first, before the next input event (InsertIntoStreamCallback.send →
StreamJunction.sendEvent; OutputRateLimiter.sendToCallBacks :61-92), and an inner stream ('#name') only reaches
the queries of its own partition instance (PartitionRuntime.addQuery :118-142, clonePartition :262-309).
Random event sequences, several flushes; the collect dumps (values, timestamps, order, match ordinals) must be
identical. The reference's own chaining KATs (FilterTestCase1.filterTest1, PatternPartitionTestCase
testPatternPartitionQuery32/33) run in test_product_kat.py."""
import random

import pytest

from oracle_lib import OracleApp

pytestmark = pytest.mark.gpu

S = "define stream S (symbol string, price float, volume int, quantity int); "
S2 = "define stream S2 (symbol string, price float, volume int, quantity int); "
TYPES = ["STRING", "FLOAT", "INT", "INT"]

APPS = {
    "filter_filter": S + "@info(name='q1') from S[70 > price] select symbol, price insert into O1; "
                         "@info(name='q2') from O1[price > 30] select symbol, price * 2 as p2 insert into O2;",
    "pattern_filter": S + "@info(name='q1') from every e1=S[price > 20] -> e2=S[price > e1.price] "
                          "within 40 milliseconds select e1.symbol as s1, e2.price as p insert into M; "
                          "@info(name='q2') from M[p > 60] select s1, p insert into O;",
    "three_levels": S + "@info(name='q1') from S[volume > 10] select symbol, price, volume insert into F; "
                        "@info(name='q2') from every e1=F[price > 30] -> e2=F[price < e1.price] "
                        "select e1.price as a, e2.price as b insert into P; "
                        "@info(name='q3') from P select a, b, a - b as d insert into O;",
    "two_consumers": S + "@info(name='q1') from S[price > 40] select symbol, price, quantity insert into X; "
                         "@info(name='q2') from X[quantity > 2] select symbol, price insert into O1; "
                         "@info(name='q3') from every e1=X -> e2=X[price > e1.price] "
                         "select e1.symbol as a, e2.symbol as b insert into O2;",
    "reads_trigger_stream": S + "@info(name='q1') from S[price > 50] select price, volume insert into X; "
                                "@info(name='q2') from every e1=X -> e2=S[price < e1.price] "
                                "select e1.price as a, e2.price as b insert into O;",
    "inner_filter_pattern": S + S2 + "partition with (quantity of S, quantity of S2) begin "
                                     "@info(name='q2') from S[price > 10] select symbol, price insert into #I; "
                                     "@info(name='q1') from every e1=#I[price > 20] -> e2=S2[price > e1.price] "
                                     "select e1.symbol as a, e2.symbol as b insert into O; end;",
    "inner_pattern_filter": S + S2 + "partition with (quantity of S, quantity of S2) begin "
                                     "@info(name='q1') from every e1=S -> e2=S2[price > e1.price] "
                                     "select e1.symbol as s1, e2.price as p insert into #M; "
                                     "@info(name='q2') from #M[p > 50] select s1, p insert into O; end;",
    # the intermediate streams declared with `define stream` (not only named by `insert into`)
    "declared_intermediate": S + "define stream X (symbol string, price float, quantity int); "
                                 "define stream P (a float, b float); "
                                 "@info(name='q1') from S[price > 40] select symbol, price, quantity insert into X; "
                                 "@info(name='q2') from every e1=X -> e2=X[price > e1.price] "
                                 "select e1.price as a, e2.price as b insert into P; "
                                 "@info(name='q3') from P[b - a > 5] select a, b insert into O;",
    # S2 is not keyed: each S2 event reaches every instance that exists when it arrives (A17)
    "broadcast": S + S2 + "partition with (quantity of S) begin "
                          "@info(name='q1') from every e1=S[price > 50] -> e2=S2[price < e1.price] "
                          "select e1.symbol as a, e2.symbol as b, e1.quantity as k insert into O; end;",
    "broadcast_inner": S + S2 + "partition with (quantity of S) begin "
                                "@info(name='q2') from S[price > 30] select symbol, price, quantity insert into #I; "
                                "@info(name='q1') from every e1=#I -> e2=S2[price < e1.price] "
                                "select e1.symbol as a, e2.symbol as b, e1.quantity as k insert into O; end;",
}


def events(seed, n, streams):
    rnd = random.Random(seed)
    syms = ["IBM", "WSO2", "GOOG", "ORCL", "MSFT"]
    out, ts = [], 1000
    for _ in range(n):
        ts += rnd.choice([0, 1, 3, 7])
        out.append((rnd.choice(streams), ts, [rnd.choice(syms), float(rnd.randint(0, 1000)) / 10.0,
                                              rnd.randint(0, 30), rnd.randint(0, 5)]))
    return out


def drive(factory, text, evs, chunks):
    app = factory(text)
    app.start()
    for k, (sid, ts, row) in enumerate(evs):
        app.send(sid, ts, row, TYPES)
        if k % chunks == chunks - 1:
            app.flush()
    app.flush()
    out = app.outputs()
    app.close()
    return out


@pytest.mark.parametrize("name", sorted(APPS))
@pytest.mark.parametrize("seed,chunks", [(1, 1), (2, 7), (3, 1000)])
def test_chained_queries_equal_oracle(name, seed, chunks):
    from siddhi_amd.testing import ProductApp
    text = APPS[name]
    streams = ["S", "S2"] if "S2" in text else ["S"]
    evs = events(seed, 400, streams)
    want = drive(OracleApp, text, evs, chunks)
    got = drive(ProductApp, text, evs, chunks)
    assert sum(len(v) for v in want["streams"].values()) > 10
    assert got == want


def test_device_batches_refuse_chained_apps():
    import torch
    from siddhi_amd.testing import EngineError, ProductApp
    app = ProductApp(APPS["filter_filter"])
    dev = torch.device("cuda", 0)
    n = 8
    cols = [torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.float32, device=dev),
            torch.zeros(n, dtype=torch.int32, device=dev), torch.zeros(n, dtype=torch.int32, device=dev)]
    with pytest.raises(EngineError):
        app.process_device_batch("S", torch.arange(n, dtype=torch.int64, device=dev), cols)
    app.close()


def test_reader_defined_before_producer_is_refused():
    """A query reading a declared stream that a LATER query inserts into: the reference delivers the inserted
    events after the reader has seen their root event on the shared junction; the product's chaining levels assume
    the other order, so the app is refused (SM_E_UNSUPPORTED) instead of answered in a different order."""
    from siddhi_amd.testing import EngineError, ProductApp
    text = (S + "define stream X (symbol string, price float); "
            "@info(name='q2') from every e1=X -> e2=S[price < e1.price] select e1.price as a, e2.price as b "
            "insert into O; "
            "@info(name='q1') from S[price > 50] select symbol, price insert into X;")
    with pytest.raises(EngineError) as ei:
        ProductApp(text)
    assert ei.value.code == 3
