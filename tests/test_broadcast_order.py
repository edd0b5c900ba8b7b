"""The order in which a partition hands an event of a stream it does not key to its instances.

PartitionStreamReceiver.send(ComplexEvent) (core/partition/PartitionStreamReceiver.java:271-275) iterates
cachedStreamJunctionMap.values(), a java.util.concurrent.ConcurrentHashMap<String, StreamJunction> keyed by
streamId + String.valueOf(key) and filled in instance creation order (addStreamJunction :284-300, called by
PartitionRuntime.updatePartitionStreamReceivers :311-315). So the outputs one such event triggers in several
instances come out in that map's iteration order, not in creation order.

The expected orders below are derived by hand from Java 8's ConcurrentHashMap: String.hashCode, spread(h) =
(h ^ h >>> 16) & 0x7fffffff, bin = spread & (table length - 1), a table of 16 bins until the 12th key (load 0.75),
a bin's keys in put order, values() in bin order. `java_chm_order` restates the same rules (plus the resize split)
independently of both engines for the larger random checks."""
import random

import pytest

from oracle_lib import OracleApp

S = ("define stream S (symbol string, price float, volume int, quantity int); "
     "define stream S2 (symbol string, price float, volume int, quantity int); ")
TYPES = ["STRING", "FLOAT", "INT", "INT"]


def app(key):
    return (S + f"partition with ({key} of S) begin "
            "@info(name='q1') from every e1=S[price > 20] -> e2=S2[price < e1.price] "
            "select e1.symbol as a, e2.symbol as b, e1.quantity as k insert into O; end;")


def jhash(s):
    """String.hashCode: h = 31 * h + c over the UTF-16 code units, 32-bit wrap-around."""
    h = 0
    units = s.encode("utf-16-be")
    for i in range(0, len(units), 2):
        h = (31 * h + (units[i] << 8 | units[i + 1])) & 0xFFFFFFFF
    return h


def spread(h):
    return (h ^ (h >> 16)) & 0x7FFFFFFF


def java_chm_order(keys):
    """Java 8 ConcurrentHashMap put (distinct keys, one thread) then values(): insertion indices in iteration
    order. Bins are lists; a bin that reaches 8 nodes first grows a table below 64 bins (tryPresize), else becomes
    a TreeBin whose later puts go to the front; transfer splits every bin by the lastRun rule."""
    n, table, tree, size_ctl, hashes = 16, [[] for _ in range(16)], [False] * 16, 12, []

    def transfer():
        nonlocal n, table, tree, size_ctl
        nt, ntree = [[] for _ in range(2 * n)], [False] * (2 * n)
        for i in range(n):
            f = table[i]
            if not f:
                continue
            if not tree[i]:
                run_bit, last = hashes[f[0]] & n, 0
                for k in range(1, len(f)):
                    if hashes[f[k]] & n != run_bit:
                        run_bit, last = hashes[f[k]] & n, k
                lo, hi = (f[last:], []) if run_bit == 0 else ([], f[last:])
                for k in range(last):
                    (lo if hashes[f[k]] & n == 0 else hi).insert(0, f[k])
            else:
                lo = [x for x in f if hashes[x] & n == 0]
                hi = [x for x in f if hashes[x] & n]
                ntree[i], ntree[i + n] = len(lo) > 6, len(hi) > 6
            nt[i], nt[i + n] = lo, hi
        size_ctl = 2 * n - n // 2
        n, table, tree = 2 * n, nt, ntree

    for idx, key in enumerate(keys):
        h = spread(jhash(key))
        hashes.append(h)
        i = h & (n - 1)
        bin_count = 0
        if not table[i]:
            table[i].append(idx)
        elif not tree[i]:
            bin_count = len(table[i])
            table[i].append(idx)
        else:
            bin_count = 2
            table[i].insert(0, idx)
        if bin_count >= 8:
            if n < 64:
                c = 1
                while c < 2 * n + n + 1:
                    c <<= 1
                while c > size_ctl:
                    transfer()
            else:
                tree[i] = True
        while len(hashes) >= size_ctl:
            transfer()
    return [x for b in table for x in b]


def drive(factory, text, evs):
    a = factory(text)
    a.start()
    for sid, ts, row in evs:
        a.send(sid, ts, row, TYPES)
    a.flush()
    out = a.outputs()["streams"].get("O", [])
    a.close()
    return out


def creating_then_broadcast(keys, key_attr):
    """One S event per key (in the given creation order), then one S2 event every instance's partial matches."""
    evs = []
    for i, k in enumerate(keys):
        row = [k, 50.0, 1, 0] if key_attr == "symbol" else ["x", 50.0, 1, int(k)]
        evs.append(("S", 1000 + i, row))
    evs.append(("S2", 2000, ["B", 10.0, 1, 0]))
    return evs


# hand-derived: "S2IBM".hashCode() = 0x04a973b5 → bin 12, "S2WSO2" 0x908ba05e → 5, "S2GOOG" 0x90844b7f → 11,
# "S2ORCL" 0x9087f84b → 12 (after S2IBM), "S2MSFT" 0x908713b3 → 4
HAND_STR = (["IBM", "WSO2", "GOOG", "ORCL", "MSFT"], ["MSFT", "WSO2", "GOOG", "IBM", "ORCL"])
# "S2" + digit d: hashCode 0x13dd1 + d, spread bin: 0→0, 1→3, 2→2, 3→5, 4→4, 5→7, 6→6, 7→9, 8→8, 9→11
HAND_INT = ([str(d) for d in range(10)], ["0", "2", "1", "4", "3", "6", "5", "8", "7", "9"])


def test_java_chm_model_matches_hand_derivation():
    for keys, want in (HAND_STR, HAND_INT):
        got = java_chm_order(["S2" + k for k in keys])
        assert [keys[i] for i in got] == want


@pytest.mark.parametrize("hand,attr", [(HAND_STR, "symbol"), (HAND_INT, "quantity")])
def test_oracle_broadcast_in_junction_map_order(hand, attr):
    keys, want = hand
    out = drive(OracleApp, app(attr), creating_then_broadcast(keys, attr))
    got = [r[1][0] if attr == "symbol" else str(r[1][2]) for r in out]
    assert got == want


def random_events(seed, n, nkeys):
    rnd = random.Random(seed)
    syms = [f"K{i}" for i in range(nkeys)]
    evs, ts = [], 1000
    for _ in range(n):
        ts += rnd.choice([0, 1, 2])
        sid = "S2" if rnd.random() < 0.15 else "S"
        evs.append((sid, ts, [rnd.choice(syms), float(rnd.randint(0, 1000)) / 10.0, rnd.randint(0, 30),
                              rnd.randint(0, nkeys)]))
    return evs


@pytest.mark.parametrize("attr,nkeys", [("symbol", 40), ("quantity", 70)])
def test_oracle_random_broadcast_follows_model(attr, nkeys):
    """Many instances (table resizes): every S2 event's outputs come out in the model's order of the instances
    existing at that point."""
    evs = random_events(7, 1500, nkeys)
    out = drive(OracleApp, app(attr), evs)
    created = []
    pos = 0
    by_trigger = {}
    for r in out:
        by_trigger.setdefault(r[2][1], []).append(r)
    ordinal = 0
    for sid, ts, row in evs:
        key = str(row[0] if attr == "symbol" else row[3])
        if sid == "S" and key not in created:
            created.append(key)
        if sid == "S2" and ordinal in by_trigger:
            order = [created[i] for i in java_chm_order(["S2" + k for k in created])]
            rank = {k: i for i, k in enumerate(order)}
            rows = by_trigger[ordinal]
            keys_out = [str(r[1][0]) if attr == "symbol" else str(r[1][2]) for r in rows]
            assert [rank[k] for k in keys_out] == sorted(rank[k] for k in keys_out)
            pos += 1
        ordinal += 1
    assert pos > 20


@pytest.mark.gpu
@pytest.mark.parametrize("attr,nkeys,seed", [("symbol", 40, 1), ("quantity", 70, 2), ("symbol", 5, 3)])
def test_product_broadcast_equals_oracle(attr, nkeys, seed):
    from siddhi_amd.testing import ProductApp
    evs = random_events(seed, 1500, nkeys)
    want = drive(OracleApp, app(attr), evs)
    got = drive(ProductApp, app(attr), evs)
    assert len(want) > 100
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("hand,attr", [(HAND_STR, "symbol"), (HAND_INT, "quantity")])
def test_product_broadcast_hand_order(hand, attr):
    from siddhi_amd.testing import ProductApp
    keys, want = hand
    out = drive(ProductApp, app(attr), creating_then_broadcast(keys, attr))
    assert [r[1][0] if attr == "symbol" else str(r[1][2]) for r in out] == want


@pytest.mark.gpu
def test_product_refuses_float_key_broadcast():
    """a partition keyed by a float / double attribute whose query reads an unkeyed stream would order
    its broadcasts by Java 8 Double.toString strings (core/partition/executor/ValuePartitionExecutor.java:34-39), which
    nothing here pins: the product refuses the app (SM_E_UNSUPPORTED) instead of guessing the order. The same app
    keyed by an int or string attribute is accepted."""
    from siddhi_amd import _lib
    from siddhi_amd.testing import EngineError, ProductApp
    with pytest.raises(EngineError) as e:
        ProductApp(app("price"))
    assert e.value.code == _lib.SM_E_UNSUPPORTED and "float / double" in str(e.value)
    ProductApp(app("quantity")).close()
