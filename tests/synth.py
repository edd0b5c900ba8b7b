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
