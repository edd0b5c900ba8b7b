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
