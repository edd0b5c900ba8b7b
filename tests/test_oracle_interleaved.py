"""The oracle's interleaved entry (cr_send_interleaved, used as the checker of device event batches and as the
config-5 CPU baseline) equals the same events sent one InputHandler.send at a time (cr_send, the path the
reference KATs pin)."""
import synth
from oracle_lib import OracleApp

TYPES = ["INT", "DOUBLE", "LONG", "LONG"]


def test_interleaved_equals_per_event_send():
    sid, cols, ts = synth.gen5(0, 6000, 60, 1)
    text = synth.app5("every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 300 milliseconds")
    a = OracleApp(text)
    a.start()
    a.send_interleaved(sid, ts, cols)
    a.flush()
    b = OracleApp(text)
    b.start()
    for i in range(len(ts)):
        row = [int(cols[0][i]), float(cols[1][i]), int(cols[2][i]), int(cols[3][i])]
        b.send("ABCDE"[sid[i]], int(ts[i]), row, TYPES)
    b.flush()
    oa, ob = a.outputs(), b.outputs()
    assert len(oa["streams"]["Out"]) > 20
    assert oa == ob



def _run(text, sid, ts, cols):
    a = OracleApp(text)
    a.start()
    a.send_interleaved(sid, ts, cols)
    a.flush()
    return [(o[0], tuple(o[1])) for o in a.outputs()["streams"].get("Out", [])]


def test_key_sharded_with_heartbeats_equals_single_app():
    """The multi-threaded CPU baseline's split (bench.cpu_shards, config 5) gives each thread one key shard
    plus the other shards' clock-advance points as heartbeats (stream -1): the union of the shard outputs equals
    the single app's outputs (the values carry the global ordinals). Without the heartbeats, timers due after a
    shard's last own event never fire."""
    import os
    import sys
    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    n, K, div, seed, shards = 6000, 60, 1, 0x5EED0005, 5
    text = synth.app5("every e1=A -> e2=B[price>e1.price]<1:3> -> (e3=C or e4=D) -> not E for 300 milliseconds")
    sid, cols, ts = synth.gen5(0, n, K, div, seed)
    whole = sorted(_run(text, sid, ts, cols))
    assert len(whole) > 20
    split = bench.cpu_shards(5, n, K, div, seed, shards)
    assert [k for k, _ in split] == ["interleaved"] * shards
    got = sorted(r for _, (s, t, c) in split for r in _run(text, s, t, c))
    assert got == whole
    no_hb = []
    for _, (s, t, c) in split:
        own = s >= 0
        no_hb += _run(text, s[own], t[own], [x[own] for x in c])
    assert len(no_hb) < len(whole)
