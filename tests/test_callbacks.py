"""The reference boundary itself: the KATs driven through the Python mirror of SiddhiManager /
SiddhiAppRuntime / InputHandler / StreamCallback / QueryCallback (siddhi_amd/__init__.py over the C ABI), with the
outputs taken from what the callbacks received. Also the delivery contract: one callback call per output chunk
(StreamCallback.receive(Event[]) StreamCallback.java:65-76; QueryCallback.receive(timestamp, in, removed) with the
chunk's last timestamp, QueryCallback.java:52-74), callbacks that send into the same app, partition clones that do
not inherit QueryCallbacks (PatternPartitionTestCase.java:71), and the runtime's error paths (a rejected row, a
batch that fails half-way)."""
import re

import pytest

from kat_runner import drive_only, load_kats, run_kat
from oracle_lib import OracleApp

pytestmark = pytest.mark.gpu

KATS = [k for k in load_kats() if "skip" not in k]


class CallbackApp:
    """kat_runner engine over the public API; outputs() = what the callbacks received, in the dump's shape."""

    def __init__(self, text):
        import siddhi_amd as S
        self.rt = S.SiddhiManager().createSiddhiAppRuntime(text)
        self.streams, self.queries, self.calls = {}, {}, []
        app = self

        class SC(S.StreamCallback):
            def __init__(self, sid):
                self.sid = sid

            def receive(self, events):
                app.calls.append(("stream", self.sid, len(events)))
                app.streams.setdefault(self.sid, []).extend([e.timestamp, e.data] for e in events)

        class QC(S.QueryCallback):
            def __init__(self, name):
                self.name = name

            def receive(self, timestamp, in_events, remove_events):
                app.calls.append(("query", self.name, len(in_events or []), timestamp))
                app.queries.setdefault(self.name, []).append([timestamp, [e.data for e in in_events or []]])

        for sid in sorted(set(re.findall(r"insert\s+into\s+(\w+)", text, re.I))):
            self.rt.addCallback(sid, SC(sid))
        for name in sorted(set(re.findall(r"@info\s*\(\s*name\s*=\s*'([^']+)'", text))):
            self.rt.addCallback(name, QC(name))

    def start(self):
        self.rt.start()

    def send(self, sid, ts, row, types):
        self.rt.getInputHandler(sid).send(ts, row)

    def advance_time(self, ts):
        self.rt.advance_time(ts)

    def advance_wallclock(self, ts):
        self.rt.advance_wallclock(ts)

    def flush(self):
        self.rt.flush()

    def outputs(self):
        return {"streams": {k: [[ts, d, []] for ts, d in v] for k, v in self.streams.items()},
                "queries": dict(self.queries)}

    def close(self):
        self.rt.shutdown()


def _product():
    from siddhi_amd.testing import ProductApp
    return ProductApp


def _values(outs):
    """(stream events as (ts, values), query events flattened per query as (ts, values))."""
    # inner streams ('#name') are visible inside their partition only: no callback can subscribe to them
    st = {k: [(e[0], e[1]) for e in v] for k, v in outs["streams"].items() if v and not k.startswith("#")}
    qs = {k: [ev for call in v for ev in call[1]] for k, v in outs["queries"].items() if v}
    return st, qs


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kat_through_callbacks(kat):
    r = run_kat(CallbackApp, kat)
    if r.startswith("unsupported"):
        pytest.skip(r)
    assert r in ("pass", "error-as-expected")


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_callbacks_equal_outputs(kat):
    """What the callbacks receive equals the ordered outputs (the collect dump, itself equal to the oracle's):
    every event once, in order; a partitioned query's QueryCallback never fires."""
    want = drive_only(_product(), kat)
    got = drive_only(CallbackApp, kat)
    if isinstance(want, tuple):
        assert isinstance(got, tuple) and got[0] == want[0], (want, got)
        return
    assert _values(got) == _values(want)


SCHEMA = "define stream S (symbol string, price double, volume int); "


def _rt(text):
    import siddhi_amd as S
    return S, S.SiddhiManager().createSiddhiAppRuntime(text)


def test_one_call_per_output_chunk():
    """An event that completes several partials emits them as one chunk: one StreamCallback.receive(Event[]) and
    one QueryCallback.receive whose timestamp is the chunk's last event's."""
    S, rt = _rt(SCHEMA + "@info(name='q') from every e1=S[price > 10] -> e2=S[price > e1.price] "
                "select e1.price as p1, e2.price as p2 insert into O;")
    got_s, got_q = [], []

    class SC(S.StreamCallback):
        def receive(self, events):
            got_s.append([(e.timestamp, e.data) for e in events])

    class QC(S.QueryCallback):
        def receive(self, ts, ins, rm):
            got_q.append((ts, [e.data for e in ins]))

    rt.addCallback("O", SC())
    rt.addCallback("q", QC())
    h = rt.getInputHandler("S")
    rt.start()
    for t, p in [(1, 50.0), (2, 40.0), (3, 30.0), (4, 60.0), (5, 70.0)]:
        h.send(t, ["A", p, 1])
    rt.flush()
    # event 4 (60) completes the partials of 50, 40 and 30 (reference order: spawn order); event 5 completes 60's
    assert got_s == [[(4, [50.0, 60.0]), (4, [40.0, 60.0]), (4, [30.0, 60.0])], [(5, [60.0, 70.0])]]
    assert got_q == [(4, [[50.0, 60.0], [40.0, 60.0], [30.0, 60.0]]), (5, [[60.0, 70.0]])]
    rt.shutdown()


@pytest.mark.parametrize("every", ["every ", ""])
def test_query_callback_before_stream_callback(every):
    """Per output chunk the query's QueryCallback runs before the output stream's StreamCallback
    (OutputRateLimiter.sendToCallBacks core/query/output/ratelimit/OutputRateLimiter.java:61-73: query callbacks, then
    the output callback into the stream's junction), on the host API path (closed form with `every`, NFA kernel
    without; a filter query in front of the pattern)."""
    S, rt = _rt(SCHEMA + "@info(name='f') from S[price > 45] select price insert into H; "
                "@info(name='q') from " + every + "e1=S[price > 10] -> e2=S[price > e1.price] "
                "select e1.price as p1, e2.price as p2 insert into O;")
    calls = []

    def sc(tag):
        class SC(S.StreamCallback):
            def receive(self, events):
                calls.append((tag, [e.data for e in events]))
        return SC()

    def qc(tag):
        class QC(S.QueryCallback):
            def receive(self, ts, ins, rm):
                calls.append((tag, [e.data for e in ins]))
        return QC()

    rt.addCallback("O", sc("O"))
    rt.addCallback("H", sc("H"))
    rt.addCallback("q", qc("q"))
    rt.addCallback("f", qc("f"))
    h = rt.getInputHandler("S")
    rt.start()
    for t, p in [(1, 50.0), (2, 40.0), (3, 30.0), (4, 60.0), (5, 70.0)]:
        h.send(t, ["A", p, 1])
    rt.flush()
    rt.shutdown()
    if every:
        q4 = [[50.0, 60.0], [40.0, 60.0], [30.0, 60.0]]
        q5 = [[60.0, 70.0]]
    else:  # one partial (event 1's), completed by event 4
        q4, q5 = [[50.0, 60.0]], None
    want = [("f", [[50.0]]), ("H", [[50.0]]),   # event 1: the filter query's callbacks
            ("f", [[60.0]]), ("H", [[60.0]]), ("q", q4), ("O", q4),  # event 4: filter first, then the pattern
            ("f", [[70.0]]), ("H", [[70.0]])]
    if q5:
        want += [("q", q5), ("O", q5)]
    assert calls == want


def test_callback_may_send_into_the_same_app():
    """A callback that sends into the runtime it is called from (no deadlock); the nested send's outputs are
    delivered inside it, as the reference's synchronous junctions do."""
    S, rt = _rt("define stream S (price double); define stream T (price double); "
                "@info(name='q1') from S[price > 10] select price insert into O1; "
                "@info(name='q2') from T[price > 100] select price insert into O2;")
    seen = []
    hT = rt.getInputHandler("T")

    class C1(S.StreamCallback):
        def receive(self, events):
            for e in events:
                seen.append(("O1", e.data[0]))
                hT.send(e.timestamp, [e.data[0] * 10])
                rt.flush()

    class C2(S.StreamCallback):
        def receive(self, events):
            seen.extend(("O2", e.data[0]) for e in events)

    rt.addCallback("O1", C1())
    rt.addCallback("O2", C2())
    rt.start()
    h = rt.getInputHandler("S")
    for t, p in [(1, 5.0), (2, 12.0), (3, 20.0)]:
        h.send(t, [p])
    rt.flush()
    assert seen == [("O1", 12.0), ("O2", 120.0), ("O1", 20.0), ("O2", 200.0)]
    rt.shutdown()


def test_rejected_row_keeps_columns_aligned():
    """A row with a wrongly typed value is refused (ClassCastException → SiddhiTypeError) without touching the
    staged columns: later rows produce exactly the oracle's outputs."""
    import siddhi_amd as S
    from siddhi_amd.testing import ProductApp
    text = SCHEMA + "@info(name='q') from S[price > 10] select symbol, price, volume insert into O;"
    rows = [(1, ["A", 11.0, 1]), (2, ["B", 12.0, 2]), (3, ["C", 9.0, 3]), (4, ["D", 30.0, 4])]
    outs = []
    for factory in (OracleApp, ProductApp):
        app = factory(text)
        app.start()
        types = ["STRING", "DOUBLE", "INT"]
        for i, (t, r) in enumerate(rows):
            app.send("S", t, r, types)
            if i == 1 and factory is ProductApp:
                with pytest.raises(Exception) as ei:
                    app.send("S", 3, ["X", "not a double", 5], ["STRING", "STRING", "INT"])
                assert getattr(ei.value, "code", None) == 4
        app.flush()
        outs.append(app.outputs())
        app.close()
    assert outs[0] == outs[1]


def test_failed_batch_refuses_further_events_until_reset():
    """A batch that fails half-way (here: the output buffer option set too small) leaves the matching state
    inconsistent; the app then refuses events instead of replaying the batch, until it is reset or restored. (A
    sequence: an `every e1 -> e2` pattern would take the closed form, whose output has no such buffer.)"""
    from siddhi_amd.testing import EngineError, ProductApp
    text = SCHEMA + ("@info(name='q') from every e1=S[price > 10], e2=S[price > e1.price] "
                     "select e1.price as p1, e2.price as p2 insert into O;")
    app = ProductApp(text, output_records=2)
    app.start()
    types = ["STRING", "DOUBLE", "INT"]
    for t, p in enumerate([20.0, 21.0, 22.0, 23.0, 24.0, 25.0]):
        app.send("S", t, ["A", p, 1], types)
    with pytest.raises(EngineError):
        app.flush()
    with pytest.raises(EngineError, match="restore a snapshot or reset"):
        app.send("S", 9, ["A", 30.0, 1], types)
    app.set_option("output_records", 0)
    app.set_option("reset", 1)
    for t, p in enumerate([20.0, 21.0]):
        app.send("S", t, ["A", p, 1], types)
    app.flush()
    assert len(app.outputs()["streams"]["O"]) == 1
    app.close()
