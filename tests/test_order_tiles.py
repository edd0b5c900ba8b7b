"""Match-dense streams on the bucket-stack pipeline (fast_stack = 1): tiles of 8192 ordinals holding about one match
per ordinal ("rising": every event matches its key's previous one; more than the order kernel's LDS images hold, so
its direct path), j's owning 21 matches each, runs longer than a lane group of the order kernel ("spikes"), and the
two alternating every three tiles ("mixed": image and direct tiles within one order workgroup). Every output is compared with the brute-force closed form
(tests/test_bench_shape.py: the first later event of the key with a higher price inside the window,
StreamPreStateProcessor.processAndReturn :274-327), in (j, i) order."""
import pytest

import bench
from test_bench_shape import closed_form_torch
from test_sparse_keys import run

pytestmark = pytest.mark.gpu


def _stream(kind, n):
    import torch
    d = torch.device("cuda", 0)
    i = torch.arange(n, dtype=torch.int64, device=d)
    if kind == "rising":  # every event matches its key's previous one: about one match per ordinal
        key = ((i // 4) % 997).to(torch.int32)
        price = 21.0 + i.to(torch.float64) * 1e-4
    elif kind == "mixed":  # blocks of 3 x 8192 ordinals alternately rising (tiles past the order kernel's LDS images:
        # its direct path) and random (image tiles), so one workgroup's tiles switch between the two paths
        key = ((i // 4) % 997).to(torch.int32)
        g = torch.Generator(device=d).manual_seed(11)
        rnd = torch.rand(n, dtype=torch.float64, device=d, generator=g) * 50.0  # c1 (price > 20) holds for 60 %
        price = torch.where((i // (3 * 8192)) % 2 == 0, 21.0 + i.to(torch.float64) * 1e-4, rnd)
    else:  # per key, blocks of 61: 20 falling prices, a spike that pops them all (21 matches on one j), 40 rising
        key = (i % 7).to(torch.int32)
        local = i // 7
        m = local % 61
        spike = 101.0 + (local // 61).to(torch.float64) * 1e-3
        price = torch.where(m < 20, 100.0 - m.to(torch.float64), spike + (m - 20).to(torch.float64) * 1e-6)
    ts = i // 1000
    torch.cuda.synchronize()
    return key, price, ts


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind", ["rising", "spikes", "mixed"])
def test_match_dense_tiles_equal_brute_force(kind):
    import torch
    key, price, ts = _stream(kind, 2_000_000)
    got, paths = run(bench.APP, key, price, ts, fast_stack=1)
    assert paths == [3], paths
    ref = closed_form_torch(key.to(torch.int64), price, ts, 1000)
    assert ref.numel() > (1_000_000 if kind == "mixed" else 1_500_000)
    if kind == "mixed":  # tiles of both kinds: past the images (7360 matches) and well inside them
        per_tile = torch.bincount(ref >> 45)  # ref: (j << 32) | i; tiles of 2^13 ordinals of j
        assert (per_tile > 8000).any() and (per_tile < 6000).any()
    assert torch.equal(ref, got)
