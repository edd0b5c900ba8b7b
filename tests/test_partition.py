"""HIP stable partition by owner rank (sm_partition_by_owner), the send side of the multi-GPU key exchange:
identical to a stable sort by owner (key mod world, non-negative) for int32 / int64 keys, negative keys, ragged
sizes and 1/2/4/8-byte columns."""
import pytest
import torch

from siddhi_amd.shard import partition_by_owner

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [0, 1, 4095, 4097, 100_003, 3_000_000])
@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kdt", [torch.int32, torch.int64])
def test_partition_equals_stable_sort(n, world, kdt):
    g = torch.Generator().manual_seed(n * 31 + world)
    keys = torch.randint(-10**6, 10**6, (n,), generator=g, dtype=torch.int64).to(kdt)
    cols = [keys.clone(), torch.rand(n, generator=g, dtype=torch.float64), torch.arange(n, dtype=torch.int64),
            torch.randint(0, 5, (n,), generator=g, dtype=torch.int32), torch.randint(0, 255, (n,), generator=g,
                                                                                    dtype=torch.uint8),
            torch.randint(0, 999, (n,), generator=g, dtype=torch.int16)]
    dev = torch.device("cuda", 0)
    got, counts = partition_by_owner(keys.to(dev), [c.to(dev) for c in cols], world)
    owner = torch.remainder(keys.to(torch.int64), world)
    order = torch.argsort(owner, stable=True)
    assert counts == torch.bincount(owner, minlength=world).tolist()
    for a, c in zip(got, cols):
        assert torch.equal(a.cpu(), c[order])
