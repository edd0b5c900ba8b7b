"""Deterministic synthetic StockStream of SURVEY.md §8(d): h(i, f) = splitmix64(seed + 4*i + f);
symbol = h(i,0) % K (from the high 32 bits), price = (h(i,1) >> 11) * 2^-53 * 100, volume = h(i,2) % 2000,
timestamp attribute = i, event time = i // ts_div. numpy here; bench.py carries the same generator in torch."""
import numpy as np

GAMMA = 0x9E3779B97F4A7C15


def seed_for(config):
    return 0x5EED0000 + config


def splitmix(z):
    with np.errstate(over="ignore"):
        z = z + np.uint64(GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def gen_stock(lo, hi, K, ts_div, seed):
    with np.errstate(over="ignore"):
        i = np.arange(lo, hi, dtype=np.uint64)
        base = np.uint64(seed) + np.uint64(4) * i
        h0, h1, h2 = splitmix(base), splitmix(base + np.uint64(1)), splitmix(base + np.uint64(2))
    symbol = ((h0 >> np.uint64(32)) % np.uint64(K)).astype(np.int32)
    price = (h1 >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * 100.0
    volume = ((h2 >> np.uint64(32)) % np.uint64(2000)).astype(np.int64)
    idx = i.astype(np.int64)
    return symbol, price, volume, idx, idx // ts_div


# Config 5: five streams A..E of the StockStream schema, stream id = h(i, 3) % 5.
SCHEMA5 = "(symbol int, price double, volume long, timestamp long)"
PART5 = "partition with (symbol of A, symbol of B, symbol of C, symbol of D, symbol of E) begin "
SELECT5 = ("select e1.timestamp as a, e2[0].timestamp as b0, e2[last].timestamp as bl, e3.timestamp as c, "
           "e4.timestamp as d insert into Out;")
QUERY5 = "every e1=A, e2=B[price>e1.price]<2:5>, (e3=C or e4=D), not E for 5 sec"


def app5(body=QUERY5, partitioned=True, playback=True, select=SELECT5):
    defs = ("@app:playback " if playback else "") + " ".join(f"define stream {s} {SCHEMA5};" for s in "ABCDE")
    q = f"@info(name='q') from {body} {select}"
    return defs + " " + (PART5 + q + " end;" if partitioned else q)


def gen5(lo, hi, K, ts_div, seed=0x5EED0005):
    """Returns (stream index int32, [symbol, price, volume, timestamp], event time)."""
    symbol, price, volume, idx, ts = gen_stock(lo, hi, K, ts_div, seed)
    with np.errstate(over="ignore"):
        i = np.arange(lo, hi, dtype=np.uint64)
        h3 = splitmix(np.uint64(seed) + np.uint64(4) * i + np.uint64(3))
    sid = ((h3 >> np.uint64(32)) % np.uint64(5)).astype(np.int32)
    return sid, [symbol, price, volume, idx], ts
