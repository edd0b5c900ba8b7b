"""`having` in the selector and the instanceOf* functions.

Reference: QuerySelector.processNoGroupBy (core/query/selector/QuerySelector.java:124-167) evaluates the output
attributes, then drops the event when the having condition is false (:138-139); SelectorParser.generateHavingExecutor
(:214-228) parses the condition with HAVING_STATE, so a bare name resolves to an output attribute first and, for a
state input, to the input events otherwise (ExpressionParser.parseVariable :1242-1275). instanceOf<T>(x) is
`x instanceof T` (core/executor/function/InstanceOf*FunctionExecutor.java). The reference's own KAT,
CountPatternTestCase.testQuery14 (having over instanceOfFloat of count-state slots), runs in test_oracle_kat.py
and test_product_kat.py; here random streams through several having queries must give identical collect dumps
on the GPU product and the oracle."""
import ctypes
import os
import random
import sys

import pytest

from oracle_lib import EngineError, OracleApp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from siddhi_amd import _lib  # noqa: E402

S = "define stream S (symbol string, price float, volume int, quantity int); "
S2 = "define stream S2 (symbol string, price float, volume int, quantity int); "
S3 = "define stream S3 (sym string, amount float, cnt int, q2 int); "
TYPES = ["STRING", "FLOAT", "INT", "INT"]

APPS = {
    "filter_having_output": S + "@info(name='q1') from S[volume > 3] select symbol, price * 2 as p2, volume "
                                "having p2 > 100 and volume < 25 insert into O;",
    "filter_having_only": S + "@info(name='q1') from S select symbol, price having price < 40 insert into O;",
    "pattern_having": S + "@info(name='q1') from every e1=S[price > 20] -> e2=S[price > e1.price] within 30 milliseconds "
                          "select e1.price as a, e2.price as b having b - a > 10 insert into O;",
    # a bare name the output does not define resolves against the input events (UNKNOWN_STATE fallback)
    "pattern_having_input_attr": S + S3 + "@info(name='q1') from every e1=S[price > 30] -> e2=S3[cnt > 5] "
                                          "select e1.symbol as s, e2.amount as p having quantity > 2 insert into O;",
    # a logical `or` leaves one slot null: instanceOf of a null is false
    "logical_instanceof": S + S2 + S3 + "@info(name='q1') from every e1=S[price > 40] -> e2=S2[price > e1.price] or "
                                        "e3=S3[amount < e1.price] select e1.price as a, e2.price as b, e3.amount as c "
                                        "having instanceOfFloat(b) or c < 20 insert into O;",
    # count slots e1[1], e1[2] exist or not (CountPatternTestCase.testQuery14's shape, one instance per volume)
    "count_instanceof": S + S2 + "partition with (volume of S, volume of S2) begin @info(name='q1') "
                                 "from e1=S[price > 20] <0:5> -> e2=S2[price > e1[0].price] "
                                 "select e1[0].price as p0, e1[1].price as p1, e1[2].price as p2, e2.price as q "
                                 "having instanceOfFloat(e1[1].price) and not instanceOfFloat(p2) insert into O; end;",
    "count_not_instanceof": S + S2 + "partition with (volume of S, volume of S2) begin @info(name='q1') "
                                     "from e1=S[price > 20] <1:3> -> e2=S2[price > e1[0].price] "
                                     "select e1[0].price as p0, e1[1].price as p1, e2.price as q "
                                     "having not instanceOfFloat(p1) insert into O; end;",
    "partition_sequence_having": S + "partition with (symbol of S) begin "
                                     "@info(name='q1') from every e1=S[price > 20], e2=S[price > e1.price] "
                                     "select e1.price as a, e2.price as b, e2.volume as v having v % 2 == 0 "
                                     "insert into O; end;",
    "select_star_having": S + "@info(name='q1') from S[price > 5] select * having quantity == 3 or volume > 20 "
                              "insert into O;",
    "instanceof_in_filter": S + "@info(name='q1') from S[instanceOfFloat(price) and not instanceOfLong(volume)] "
                                "select symbol, instanceOfString(symbol) as isstr insert into O;",
}


def events(seed, n, streams):
    rnd = random.Random(seed)
    syms = ["IBM", "WSO2", "GOOG", "ORCL"]
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


def _dump(text):
    import siddhi_amd
    try:
        return 0, siddhi_amd.compile_dump(text)
    except Exception as e:  # the reference's exception classes
        return 1, str(e)


def _jit(text):
    L = _lib.lib()
    log = ctypes.create_string_buffer(8192)
    size = ctypes.c_size_t()
    rc = L.sm_nfa_jit_compile(text.encode(), 0, log, 8192, ctypes.byref(size))
    return rc, log.value.decode(errors="replace")


def test_parser_dumps_having_and_instanceof():
    rc, js = _dump(APPS["count_instanceof"])
    assert rc == 0, js
    q = js["partitions"][0]["queries"][0]
    h = q["having"]
    assert h["and"][0] == {"instanceof": "FLOAT", "arg": {"var": "price", "ref": "e1", "index": 1}}, h
    assert h["and"][1] == {"not": {"instanceof": "FLOAT", "arg": {"var": "p2"}}}
    rc, js = _dump(APPS["filter_having_only"])
    assert rc == 0 and "having" in js["queries"][0]


def test_parser_rejects_other_functions_and_bad_arity():
    rc, msg = _dump(S + "from S select convert(price, 'string') as c insert into O;")
    assert rc != 0 and "function" in msg
    rc, msg = _dump(S + "from S select instanceOfFloat(price, volume) as c insert into O;")
    assert rc != 0 and "required only 1" in msg
    rc, msg = _dump(S + "from S select symbol group by symbol insert into O;")
    assert rc != 0 and "group by" in msg


@pytest.mark.parametrize("name", ["count_instanceof"])
def test_having_plans_compile_to_specialised_kernels(name):
    rc, log = _jit(APPS[name])
    assert rc == 0, log


def test_single_stream_having_sees_output_attributes_only():
    # MetaStreamEvent + HAVING_STATE: the output definition only (ExpressionParser.parseVariable :1242-1246)
    text = S + "@info(name='q1') from S select symbol, price having volume > 3 insert into O;"
    with pytest.raises(EngineError):
        OracleApp(text)
    rc, log = _jit(S + S2 + "@info(name='q1') from every e1=S -> e2=S2 select e1.price as a having zz > 1 "
                             "insert into O;")
    assert rc != 0


def test_oracle_having_drops_outputs():
    text = APPS["filter_having_only"]
    evs = [("S", 1000 + k, ["IBM", p, 1, 1]) for k, p in enumerate([10.0, 50.0, 39.5, 40.0, 0.5])]
    out = drive(OracleApp, text, evs, 1000)
    got = [o[1][1] for o in out["streams"]["O"]]  # [ts, values, ordinals]
    assert got == [10.0, 39.5, 0.5]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(APPS))
@pytest.mark.parametrize("seed,chunks", [(1, 1), (2, 9), (3, 1000)])
def test_having_equals_oracle(name, seed, chunks):
    from siddhi_amd.testing import ProductApp
    text = APPS[name]
    streams = [x for x in ("S", "S2", "S3") if f"define stream {x} " in text]
    evs = events(seed, 300, streams)
    want = drive(OracleApp, text, evs, chunks)
    got = drive(ProductApp, text, evs, chunks)
    assert sum(len(v) for v in want["streams"].values()) >= 3
    assert got == want


@pytest.mark.gpu
def test_having_removes_some_outputs():
    """The having condition must actually drop outputs on these streams (else the parity test proves little)."""
    text = APPS["pattern_having"]
    no_having = text.replace(" having b - a > 10", "")
    evs = events(5, 300, ["S"])
    from siddhi_amd.testing import ProductApp
    with_h = drive(ProductApp, text, evs, 1000)["streams"]["O"]
    without = drive(ProductApp, no_having, evs, 1000)["streams"]["O"]
    assert 0 < len(with_h) < len(without)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pattern_having", "count_instanceof"])
def test_having_query_specialised_kernel_equals_oracle(name):
    """The same having programs in the query-specialised NFA kernel (option nfa_jit = 1, nfa_jit.cpp)."""
    from siddhi_amd.testing import ProductApp
    text = APPS[name]
    streams = [x for x in ("S", "S2", "S3") if f"define stream {x} " in text]
    evs = events(7, 300, streams)
    want = drive(OracleApp, text, evs, 100)
    got = drive(lambda t: ProductApp(t, nfa_jit=1), text, evs, 100)
    assert sum(len(v) for v in want["streams"].values()) >= 3
    assert got == want
