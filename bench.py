"""Headline benchmark (BASELINE.json metric): input events/sec + % HBM peak for the partitioned pattern query

    partition with (symbol of StockStream) begin
      from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
      select e1.timestamp as i, e2.timestamp as j insert into OutputStream;
    end;

on synthetic StockStream events (K = 1e6 symbols, N = 1e9 events, event time
ts_i = floor(i / 10000) ms), device-resident before the timed region. One step = one pass of the hot path
over the whole batch: (multi-GPU) hash-by-key all-to-all of (symbol, price, ts, ordinal) over RCCL/xGMI,
then the closed-form pattern kernels producing the ordered (e1, e2) match tuples on every rank.

Scaling is strong (N is the whole job at every GPU count). Launch: python bench.py [--gpus N --steps K
--warmup W]; for N > 1 the driver uses torch.distributed.run (one rank per GPU).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

APP = ("define stream StockStream (symbol int, price double, volume long, timestamp long); "
       "partition with (symbol of StockStream) begin "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.timestamp as i, e2.timestamp as j insert into OutputStream; end;")
SEED = 0x5EED0000 + 4
HBM_PEAK = 8.0e12
GAMMA = 0x9E3779B97F4A7C15


def _i64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def splitmix_torch(v):
    """splitmix64 finaliser of (v + gamma) on int64 tensors (wrap-around arithmetic, logical shifts)."""
    import torch
    z = v + _i64(GAMMA)
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _i64(0x94D049BB133111EB)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def gen_stock(lo, hi, K, ts_div, device):
    """Events [lo, hi) of the synthetic stream: h(i,f) = splitmix64(seed + 4i + f)."""
    import torch
    i = torch.arange(lo, hi, dtype=torch.int64, device=device)
    base = SEED + 4 * i
    h0 = splitmix_torch(base)
    symbol = (((h0 >> 32) & 0xFFFFFFFF) % K).to(torch.int32)
    del h0
    h1 = splitmix_torch(base + 1)
    price = ((h1 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (2.0 ** -53) * 100.0
    del h1
    h2 = splitmix_torch(base + 2)
    volume = ((h2 >> 32) & 0xFFFFFFFF) % 2000
    del h2, base
    ts = i // ts_div
    return symbol, price, volume, i, ts


def gen_stock_numpy(lo, hi, K, ts_div):
    import numpy as np
    with np.errstate(over="ignore"):
        i = np.arange(lo, hi, dtype=np.uint64)
        out = []
        for f in range(3):
            z = np.uint64(SEED) + np.uint64(4) * i + np.uint64(f) + np.uint64(GAMMA)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out.append(z ^ (z >> np.uint64(31)))
    symbol = ((out[0] >> np.uint64(32)) % np.uint64(K)).astype(np.int32)
    price = (out[1] >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * 100.0
    volume = ((out[2] >> np.uint64(32)) % np.uint64(2000)).astype(np.int64)
    idx = i.astype(np.int64)
    return symbol, price, volume, idx, idx // ts_div


def cpu_baseline(sample, K, ts_div):
    """The CPU oracle (literal restatement of the reference engine, 1 thread) on the first `sample` events."""
    from oracle_lib import OracleApp, lib
    import numpy as np
    sym, price, vol, ts_attr, ts = gen_stock_numpy(0, sample, K, ts_div)
    app = OracleApp(APP)
    app.set_collect(False)
    cols = [np.ascontiguousarray(c) for c in (sym, price, vol, ts_attr)]
    ptrs = (ctypes.c_void_p * 4)(*[c.ctypes.data for c in cols])
    err = ctypes.create_string_buffer(512)
    t0 = time.perf_counter()
    rc = lib().cr_send_columns(app.h, app.stream_index("StockStream"), sample, ts.ctypes.data, ptrs, err, 512)
    dt = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(err.value.decode())
    m = app.output_count("OutputStream")
    app.close()
    return sample / dt, dt, m


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--events", type=float, default=1e9)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--ts-div", type=int, default=10_000)
    ap.add_argument("--cpu-sample", type=int, default=4_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from siddhi_amd.testing import ProductApp
    from siddhi_amd.shard import exchange_by_key

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    N = int(args.events)
    K = args.keys
    lo, hi = N * rank // world, N * (rank + 1) // world
    symbol, price, volume, tsattr, ts = gen_stock(lo, hi, K, args.ts_div, dev)
    del volume, tsattr  # not referenced by the query: the exchange ships only what the plan reads
    ordinals = torch.arange(lo, hi, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()

    app = ProductApp(APP)
    stream = torch.cuda.current_stream(dev)
    hip_stream = ctypes.c_void_p(stream.cuda_stream)
    n_local = [hi - lo]

    def step():
        if world > 1:
            (s_sym, s_price, s_ts, s_ord), _ = exchange_by_key(symbol, [symbol, price, ts, ordinals], world)
        else:
            s_sym, s_price, s_ts, s_ord = symbol, price, ts, None
        n_local[0] = s_ts.numel()
        # columns: symbol, price, volume, timestamp (volume/timestamp are not read by the plan)
        app.process_device_batch("StockStream", s_ts, [s_sym, s_price, s_price, s_price], ordinals=s_ord,
                                 ordinal_base=0, hip_stream=hip_stream)
        return app.device_matches("q")[1]

    log(f"rank {rank}: {hi - lo} events resident; warmup {args.warmup}")
    for _ in range(args.warmup):
        step()
    # per-launch HIP events inside the library, on the launch stream (a few event records per step)
    app.set_option("fast_timing", 1)
    ktot = {}
    log(f"rank {rank}: timing {args.steps} steps")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nm = 0
    for _ in range(args.steps):
        nm = step()
        for lab in KERNELS:  # the library synchronised its stream before returning: the marks are complete
            c = app.get_stat("kernel_calls:" + lab)
            if c:
                e = ktot.setdefault(lab, [0.0, 0])
                e[0] += app.get_stat("kernel_ms:" + lab)
                e[1] += int(c)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    m = torch.tensor([nm], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(m)
    dt = t.item()
    total_matches = m.item()
    ms_per_step = dt / args.steps * 1e3
    value = N / (dt / args.steps)

    roof = roofline(ktot, n_local[0], nm, args.steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        log(f"cpu baseline on {args.cpu_sample} events")
        v, sec, mm = cpu_baseline(args.cpu_sample, K, args.ts_div)
        cpu = {"value": v, "unit": "events/s", "cores": 1, "kind": "port",
               "sample": f"first {args.cpu_sample} events of the same stream through oracle/cpu_ref "
                         f"(C++ restatement of the reference engine, 1 thread): {sec:.2f} s, {mm} matches"}
    if rank == 0:
        alg_bytes = 20 * N + 8 * total_matches
        line = {
            "metric": "input events/sec + % HBM peak, partitioned pattern query, 1/2/4/8 MI355X",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (counter-based splitmix64 StockStream, device-resident)",
            "config": {"workload": "config 4: partition with (symbol of StockStream) every e1 -> e2 within 1 sec",
                       "events": N, "keys": K, "event_time": f"floor(i/{args.ts_div}) ms",
                       "matches": total_matches, "parallelism": f"key-sharded x{world}",
                       "step_hbm_fraction": alg_bytes / (ms_per_step * 1e-3) / HBM_PEAK},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Kernels of the device pipeline (labels recorded by kernels/fastpath3.hip) and their ALGORITHMIC bytes per
# launch for a batch of n events with m matches: what each launch must read and write at minimum.
KERNELS = ["prep", "key_up", "scan", "key_pass0", "key_pass", "walk", "j_up", "j_pass", "j_pass_last"]


def alg_bytes(label, n, m):
    return {"prep": 20 * n + n // 8,        # key i32 + ts i64 + price f64 (c1 = price > 20) in, c1 bit out
            "key_up": 16 * n,               # pass-1 digits: one 16-B record per event (the key word of each)
            "scan": 0,                      # per-chunk digit counts (O(chunks x 1024), not per event)
            "key_pass0": 20 * n + 16 * n,   # key i32 + price f64 + ts i64 in, 16-B keyed record out
            "key_pass": 16 * n + 16 * n,    # 16-B record in and out
            "walk": 16 * n + 8 * m,         # records in, (j, i) u32 pairs out
            "j_up": 4 * m,
            "j_pass": 16 * m,               # (j, i) in and out
            "j_pass_last": 16 * m}[label]


def roofline(ktot, n, m, steps):
    """Dominant kernel (largest total time over the timed steps): algorithmic bytes per launch / average launch
    duration, against HBM peak. Also the per-kernel breakdown."""
    if not ktot:
        return None
    dom = max(ktot, key=lambda k: ktot[k][0])
    tot_ms, calls = ktot[dom]
    avg_ms = tot_ms / calls
    per_launch = alg_bytes(dom, n, m)
    ach = per_launch / (avg_ms * 1e-3)
    brk = {k: {"avg_ms": v[0] / v[1], "calls_per_step": v[1] / steps,
               "gbps": alg_bytes(k, n, m) / (v[0] / v[1] * 1e-3) / 1e9} for k, v in ktot.items()}
    return {"bound": "hbm", "achieved": ach / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": ach / HBM_PEAK,
            "traffic": None, "kernel": dom, "avg_launch_ms": avg_ms, "alg_bytes_per_launch": per_launch,
            "breakdown": brk}


if __name__ == "__main__":
    main()
