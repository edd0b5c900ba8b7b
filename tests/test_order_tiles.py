"""Match-dense streams on the bucket-stack pipeline (fast_stack = 1): tiles of 8192 ordinals holding about one match
per ordinal ("rising": every event matches its key's previous one), and j's owning 21 matches each, runs longer than
a lane group of the order kernel ("spikes"). Every output is compared with the brute-force closed form
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
@pytest.mark.parametrize("kind", ["rising", "spikes"])
def test_match_dense_tiles_equal_brute_force(kind):
    import torch
    key, price, ts = _stream(kind, 2_000_000)
    got, paths = run(bench.APP, key, price, ts, fast_stack=1)
    assert paths == [3], paths
    ref = closed_form_torch(key.to(torch.int64), price, ts, 1000)
    assert ref.numel() > 1_500_000
    assert torch.equal(ref, got)
