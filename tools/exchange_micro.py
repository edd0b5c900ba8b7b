"""Time the on-GPU part of the key exchange (everything but the RCCL transfer) for one rank of a world-8 run of
config 4 (N / 8 events): torch form (int64 argsort + a gather per column) vs the HIP stable partition that
siddhi_amd.shard uses on the GPU (measured round 1: 19.95 ms vs 2.49 ms at 1.25e8 events)."""
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 125_000_000
world = 8
dev = torch.device("cuda", 0)
sym, price, vol, tsa, ts = bench.gen_stock(0, n, 1_000_000, 10_000, dev, bench.seed_for(4))
ords = torch.arange(n, dtype=torch.int64, device=dev)
cols = [sym, price, ts, ords]


def old():
    owner = torch.remainder(sym.to(torch.int64), world)
    order = torch.argsort(owner, stable=True)
    torch.bincount(owner, minlength=world).tolist()
    return [c[order].contiguous() for c in cols]


def new():
    from siddhi_amd.shard import partition_by_owner
    return partition_by_owner(sym, cols, world)[0]


for name, f in (("torch argsort + gathers", old), ("hip partition", new)):
    f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        r = f()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t) / 5 * 1e3:.2f} ms for {n} events", flush=True)
a, b = old(), new()
print("equal:", all(torch.equal(x, y) for x, y in zip(a, b)))
