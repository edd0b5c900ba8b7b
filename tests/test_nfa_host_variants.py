"""The config-5 query and its variants (tests/test_device_events.py VARIANTS) through the device NFA code compiled for
the host (tests/native), against the oracle on the same interleaved stream: the CPU check of the NFA's list-node
operand cache (plan.h DPre.ncache: `B[price > e1.price]` is tried from the pending-list node) and of the lazy removal
of count partials whose next state is filled (CountPreStateProcessor.processAndReturn :58-93). Test infrastructure."""
import os
import subprocess

import numpy as np
import pytest

import synth
from test_device_events import VARIANTS, oracle_out

HERE = os.path.dirname(os.path.abspath(__file__))
EXTRA = {
    # two cached operands, one of them null-able (absent states have no cache; the e1 values are cached)
    "two_operands": "every e1=A -> e2=B[price > e1.price and volume < e1.volume + 500]<1:3> -> e3=C",
    # a stream state whose filter reads an earlier state (PK_STREAM trial with the cache)
    "stream_cached": "every e1=A -> e2=B[price > e1.price] -> e3=C[price < e2.price]",
    # a count state whose filter reads an earlier stream state (cached: e1's chain no longer changes)
    "count_cached": "every e1=A -> e2=B[price > e1.price]<2:4> -> e3=C",
    # not cacheable, the record path: three distinct operands of e1 (at most two are cached) ...
    "three_operands": "every e1=A -> e2=B[price > e1.price and volume < e1.volume + 900 and timestamp > e1.timestamp]"
                      "<1:3> -> e3=C",
    # ... and a filter reading a count state (its chain still grows while the partial waits)
    "count_source": "every e1=A -> e2=B[price > e1.price]<1:3> -> e3=C[price < e2[0].price]",
}


@pytest.fixture(scope="module")
def harness():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
    from host_harness_lib import HostHarnessApp
    return HostHarnessApp


def harness_out(H, text, sid, cols, ts, flush_every=0):
    a = H(text)
    a.start()
    types = ["INT", "DOUBLE", "LONG", "LONG"]
    for i in range(len(ts)):
        s = int(sid[i])
        if s < 0:
            a.advance_time(int(ts[i]))
        else:
            a.send("ABCDE"[s], int(ts[i]), [int(cols[0][i]), float(cols[1][i]), int(cols[2][i]), int(cols[3][i])],
                   types)
        if flush_every and (i + 1) % flush_every == 0:
            a.flush()
    a.flush()
    o = a.outputs()
    a.close()
    return o


@pytest.mark.parametrize("name", sorted(VARIANTS) + sorted(EXTRA))
def test_variant_host_nfa_equals_oracle(harness, name):
    sid, cols, ts = synth.gen5(0, 60_000, 2000, 1)
    if name in VARIANTS:
        text = synth.app5(VARIANTS[name])
    else:
        text = synth.app5(EXTRA[name], select="select e1.timestamp as a, e2[0].timestamp as b, e2[last].timestamp as "
                                               "bl, e3.timestamp as c insert into Out;")
    exp = oracle_out(text, sid, cols, ts)
    got = harness_out(harness, text, sid, cols, ts)
    if name not in ("config5",):
        assert len(exp["streams"].get("Out", [])) > 20
    assert got["streams"].get("Out", []) == exp["streams"].get("Out", [])
    if name not in ("config5",):  # the same stream cut into batches (lane state carried across flushes)
        got = harness_out(harness, text, sid, cols, ts, flush_every=7919)
        assert got["streams"].get("Out", []) == exp["streams"].get("Out", [])


def test_stale_count_partials_stay_bounded(harness, monkeypatch):
    """on the lazy count path a partial whose next state is filled stays pending until a trial
    passes; with prices that keep falling none does, and each A leaves one such partial behind. The reference drops
    them at the next B (CountPreStateProcessor.removeIfNextStateProcessed :95-101), so its memory stays bounded; here
    the collector drops them (Lane::prune_stale). With a 256-word arena per semispace and 3000 A's the key's heap
    overflows (NFA_ERR_ARENA) unless they go."""
    monkeypatch.setenv("SM_HOST_HEAP_HALF", "256")
    text = synth.app5("every e1=A -> e2=B[price > e1.price]<1:3> -> e3=C",
                      select="select e1.timestamp as a, e2[0].timestamp as b, e3.timestamp as c insert into Out;")
    n = 3000
    sid, p = [], []
    for i in range(n):  # A at 1e4 - i, one B just above it (the only B it ever passes), a C that fills e3
        sid += [0, 1, 2]
        p += [1e4 - i, 1e4 - i + 0.5, 1.0]
    m = len(sid)
    cols = [np.full(m, 7, np.int32), np.array(p), (np.arange(m) % 2000).astype(np.int64), np.arange(m, dtype=np.int64)]
    ts = np.arange(m, dtype=np.int64)
    sid = np.array(sid, dtype=np.int32)
    exp = oracle_out(text, sid, cols, ts)
    got = harness_out(harness, text, sid, cols, ts)
    assert len(exp["streams"]["Out"]) == n
    assert got["streams"]["Out"] == exp["streams"]["Out"]
