"""Headline benchmark (BASELINE.json metric): input events/sec + % HBM peak for the partitioned pattern query

    partition with (symbol of StockStream) begin
      from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec
      select e1.timestamp as i, e2.timestamp as j insert into OutputStream;
    end;

on synthetic StockStream events (K = 1e6 symbols, N = 1e9 events, event time
ts_i = floor(i / 10000) ms), device-resident before the timed region. One step = one pass of the hot path
over the whole batch: the closed-form pattern kernels producing the ordered (e1, e2) match tuples.

Multi-GPU (--gpus N > 1): the reference ingests ONE stream and routes every event to its key's partition instance
(PartitionStreamReceiver.receive core/partition/PartitionStreamReceiver.java:156-168, PartitionRuntime.cloneIfNotExist
core/partition/PartitionRuntime.java:256-309), with one global output order. bench.py measures exactly that
configuration: every rank ingests a contiguous slice of the one N-event stream, the keys are routed to their owner
rank by a hash-by-key RCCL all-to-all of packed (symbol, price, ts, offset) records over xGMI, each rank matches its
keys, and every match tuple returns to the rank that ingested its e2, ordered there (shard.partitioned_step): strong
scaling, value = N / the slowest rank's step time, config.rccl_world = the size of the RCCL (nccl) group.
`--key-partitions` adds an opt-in side line (`key_partitions`, never `value`): each rank runs its own N-event stream on
its own key range with no data-path collective (weak scaling). Launch: python bench.py [--gpus N --steps K
--warmup W]; for N > 1 under torch.distributed.run (one rank per GPU; WORLD_SIZE must equal N), or without a
launcher, in which case bench.py starts torch.distributed.run with N ranks itself (launch_command).

The other §8(d) configurations are parity/measurement side lines, selected with --config:
  --config 2   filter-only `StockStream[price > 70 and volume < 1000]`, N = 1e9 (bandwidth roofline);
               multi-GPU: contiguous index ranges per rank, no exchange (strong scaling)
  --config 3   non-partitioned `every e1 -> e2 within 1 sec`, N = 1e8, ts_i = i ms; does not shard:
               --gpus N runs N independent replicas (weak scaling, replicas only)
  --config 5   `@app:playback`, five streams A..E, partition with (symbol of A..E),
               `every e1=A, e2=B[price>e1.price]<2:5>, (e3=C or e4=D), not E for 5 sec`, K = 1e6, N = 1e8,
               ts_i = floor(i / 100) ms (about one event per key every 10 s, so `not E for 5 sec` timers fire);
               general NFA kernel over an interleaved device batch; multi-GPU: key exchange + the global
               clock-advance points as heartbeats on every rank (strong scaling)
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

SCHEMA = "define stream StockStream (symbol int, price double, volume long, timestamp long); "
APP = (SCHEMA + "partition with (symbol of StockStream) begin "
       "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
       "select e1.timestamp as i, e2.timestamp as j insert into OutputStream; end;")
APP2 = SCHEMA + "@info(name='q') from StockStream[price > 70 and volume < 1000] select timestamp insert into Out;"
APP3 = (SCHEMA + "@info(name='q') from every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] "
        "within 1 sec select e1.timestamp as i, e2.timestamp as j insert into OutputStream;")
STREAMS5 = "ABCDE"
APP5 = ("@app:playback " + " ".join(f"define stream {x} (symbol int, price double, volume long, timestamp long);"
                                    for x in STREAMS5) +
        " partition with (symbol of A, symbol of B, symbol of C, symbol of D, symbol of E) begin "
        "@info(name='q') from every e1=A, e2=B[price>e1.price]<2:5>, (e3=C or e4=D), not E for 5 sec "
        "select e1.timestamp as a, e2[0].timestamp as b0, e2[last].timestamp as bl, e3.timestamp as c, "
        "e4.timestamp as d insert into Out; end;")
# Config 5 variant that emits: the same streams and conditions as a pattern ('->'), so that
# partials survive the interleaving (the sequence form emits nothing at this scale: CountPostStateProcessor
# re-adds a sequence partial only once n >= min, StateStreamRuntime resets it before the second B)
VARIANTS5 = {
    "pattern_count_not5s": "every e1=A -> e2=B[price>e1.price]<2:5> -> (e3=C or e4=D) -> not E for 5 sec",
}


def app5_variant(body):
    return APP5.replace("every e1=A, e2=B[price>e1.price]<2:5>, (e3=C or e4=D), not E for 5 sec", body)


HBM_PEAK = 8.0e12
GAMMA = 0x9E3779B97F4A7C15
METRIC = "input events/sec + % HBM peak, partitioned pattern query, 1/2/4/8 MI355X"


def seed_for(config):
    return 0x5EED0000 + config


def _i64(x):
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >= (1 << 63) else x


def splitmix_torch(v):
    """splitmix64 finaliser of (v + gamma) on int64 tensors (wrap-around arithmetic, logical shifts)."""
    z = v + _i64(GAMMA)
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _i64(0x94D049BB133111EB)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def gen_stock(lo, hi, K, ts_div, device, seed):
    """Events [lo, hi) of the synthetic stream: h(i,f) = splitmix64(seed + 4i + f)."""
    import torch
    i = torch.arange(lo, hi, dtype=torch.int64, device=device)
    base = seed + 4 * i
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


def gen_stream_idx(lo, hi, device, seed):
    """Config 5 stream of each event: h(i, 3) % 5 (A..E)."""
    import torch
    i = torch.arange(lo, hi, dtype=torch.int64, device=device)
    h3 = splitmix_torch(seed + 4 * i + 3)
    return (((h3 >> 32) & 0xFFFFFFFF) % 5).to(torch.int32)


def gen_stock_numpy(lo, hi, K, ts_div, seed):
    import numpy as np
    with np.errstate(over="ignore"):
        i = np.arange(lo, hi, dtype=np.uint64)
        out = []
        for f in range(3):
            z = np.uint64(seed) + np.uint64(4) * i + np.uint64(f) + np.uint64(GAMMA)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out.append(z ^ (z >> np.uint64(31)))
    symbol = ((out[0] >> np.uint64(32)) % np.uint64(K)).astype(np.int32)
    price = (out[1] >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * 100.0
    volume = ((out[2] >> np.uint64(32)) % np.uint64(2000)).astype(np.int64)
    idx = i.astype(np.int64)
    return symbol, price, volume, idx, idx // ts_div


def cpu_baseline(sample, K, ts_div, app_text, seed, out_stream, config=4):
    """The CPU oracle (literal restatement of the reference engine, 1 thread) on the first `sample` events."""
    if config == 5:
        import numpy as np
        import synth
        from oracle_lib import OracleApp
        sid, cols, ts = synth.gen5(0, sample, K, ts_div, seed)
        app = OracleApp(app_text)
        app.set_collect(False)
        app.start()
        t0 = time.perf_counter()
        app.send_interleaved(sid, ts, cols)
        app.flush()
        dt = time.perf_counter() - t0
        m = app.output_count(out_stream)
        app.close()
        return sample / dt, dt, m
    from oracle_lib import OracleApp, lib
    import numpy as np
    sym, price, vol, ts_attr, ts = gen_stock_numpy(0, sample, K, ts_div, seed)
    app = OracleApp(app_text)
    app.set_collect(False)
    cols = [np.ascontiguousarray(c) for c in (sym, price, vol, ts_attr)]
    ptrs = (ctypes.c_void_p * 4)(*[c.ctypes.data for c in cols])
    err = ctypes.create_string_buffer(512)
    t0 = time.perf_counter()
    rc = lib().cr_send_columns(app.h, app.stream_index("StockStream"), sample, ts.ctypes.data, ptrs, err, 512)
    dt = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(err.value.decode())
    m = app.output_count(out_stream)
    app.close()
    return sample / dt, dt, m


def cpu_shards(config, sample, K, ts_div, seed, threads):
    """The sample split for the multi-threaded CPU baseline (SURVEY.md §8(d) variant (b)): partitioned configs
    (4, 5) by key, `symbol % threads` (keys are independent: PartitionRuntime.java:262-309), so each thread runs
    the oracle app on its own key subset; config 2 by contiguous index range. Config 5 is @app:playback: the
    event-time clock is global, so each thread also replays the other threads' clock-advance points as
    heartbeats (stream -1), exactly as a rank of the multi-GPU path does. Returns a list of per-thread
    (kind, args) ready for the oracle entry points."""
    import numpy as np
    if config == 5:
        import synth
        sid, cols, ts = synth.gen5(0, sample, K, ts_div, seed)
        first = np.ones(sample, dtype=bool)
        first[1:] = ts[1:] > ts[:-1]
        out = []
        for t in range(threads):
            mine = (cols[0] % threads) == t
            keep = mine | first
            s = np.where(mine, sid, -1)[keep].astype(np.int32)
            out.append(("interleaved", (s, ts[keep], [c[keep] for c in cols])))
        return out
    sym, price, vol, ts_attr, ts = gen_stock_numpy(0, sample, K, ts_div, seed)
    cols = [sym, price, vol, ts_attr]
    out = []
    for t in range(threads):
        if config == 2:
            lo, hi = sample * t // threads, sample * (t + 1) // threads
            sel = slice(lo, hi)
        else:
            sel = (sym % threads) == t
        out.append(("columns", (ts[sel], [np.ascontiguousarray(c[sel]) for c in cols])))
    return out


def cpu_baseline_threads(sample, K, ts_div, app_text, seed, out_stream, config, threads):
    """The CPU oracle on `threads` host threads, one app per shard (cpu_shards). The oracle's C entry points
    run without the GIL (ctypes), so the shards run in parallel. Timed from the release of all threads to the
    last one's return; the split itself is not timed (the generous baseline). Returns (events/s, s, matches)."""
    import threading
    import numpy as np
    from oracle_lib import OracleApp, lib
    shards = cpu_shards(config, sample, K, ts_div, seed, threads)
    apps = []
    for _ in shards:
        a = OracleApp(app_text)
        a.set_collect(False)
        a.start()
        apps.append(a)
    errs = []
    go = threading.Barrier(len(shards) + 1)

    def work(app, kind, args):
        go.wait()
        try:
            if kind == "interleaved":
                app.send_interleaved(*args)
            else:
                ts, cols = args
                ptrs = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
                err = ctypes.create_string_buffer(512)
                ts = np.ascontiguousarray(ts)
                rc = lib().cr_send_columns(app.h, app.stream_index("StockStream"), ts.size, ts.ctypes.data, ptrs,
                                           err, 512)
                if rc != 0:
                    raise RuntimeError(err.value.decode())
        except Exception as e:  # noqa: BLE001 — reported after join
            errs.append(e)

    ths = [threading.Thread(target=work, args=(a, k, x)) for a, (k, x) in zip(apps, shards)]
    for th in ths:
        th.start()
    go.wait()
    t0 = time.perf_counter()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    if errs:
        raise errs[0]
    m = sum(a.output_count(out_stream) for a in apps)
    for a in apps:
        a.close()
    return sample / dt, dt, m


def host_threads():
    """Host threads for the multi-threaded baseline: the box's CPU share (OMP_NUM_THREADS is set to it on the
    GPU box; os.cpu_count() there shows the whole machine)."""
    n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get("OMP_NUM_THREADS", n)), 16))


def host_cpu():
    """the host the CPU baseline ran on (lscpu model name, nproc)."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    if model is None:
        try:
            import subprocess
            out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
            for ln in out.splitlines():
                if ln.startswith("Model name"):
                    model = ln.split(":", 1)[1].strip()
        except Exception:  # noqa: BLE001
            pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "threads_allowed": host_threads()}


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


# Per configuration: app, default N, event-time divisor, whether the path shards, whole-job algorithmic bytes
#  and the kernels of its device pipeline.
CONFIGS = {
    2: dict(app=APP2, events=1e9, ts_div=1, out="Out", shards=True, scaling="strong",
            workload="config 2: StockStream[price > 70 and volume < 1000] select timestamp (filter roofline)",
            job_bytes=lambda n, m: 16 * n + 4 * m, cpu_sample=20_000_000),
    3: dict(app=APP3, events=1e8, ts_div=1, out="OutputStream", shards=False, scaling="weak",
            workload="config 3: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 1 sec "
                     "(non-partitioned; replicas only)",
            # the CPU sample is BASELINE configs[0], the reference's own CPU case: this query, 1e7 events
            job_bytes=lambda n, m: 16 * n + 8 * m, cpu_sample=10_000_000),
    4: dict(app=APP, events=1e9, ts_div=10_000, out="OutputStream", shards=True, scaling="strong",
            workload="config 4: partition with (symbol of StockStream) every e1 -> e2 within 1 sec",
            job_bytes=lambda n, m: 20 * n + 8 * m, cpu_sample=4_000_000),
    5: dict(app=APP5, events=1e8, ts_div=100, out="Out", shards=True, scaling="strong",
            workload="config 5: @app:playback partition with (symbol of A..E) every e1=A, e2=B[price>e1.price]<2:5>, "
                     "(e3=C or e4=D), not E for 5 sec",
            # key i32 + price f64 + event time i64 + stream id (1 B) in; 5 ordinals per output event out
            job_bytes=lambda n, m: 21 * n + 40 * m, cpu_sample=60_000,
            # per-key arena of 4096 words per semispace (66 GB for 1e6 keys, of 288 GB): fewer copying collections
            # (NFA kernel 64.4 ms at 1024 words, 55.9 at 2048, 54.9 at 4096; query-specialised kernel)
            options={"heap_words": 4096}),
}


def via_input_handler(cols_dev, n, expect, chunk=None, app_text=APP):
    """Config 4 (and config 3's query: BASELINE configs[0], the reference's own CPU case, is that app through
    SiddhiManager / InputHandler) through the unchanged reference API (VERDICT r03 missing #3): host columns (pageable numpy arrays, as a
    JNI receiver would hand over the Event[] data) -> InputHandler.send(Event[]) in columnar form
    (sm_input_send_columns) -> the device-batch pipelines in chunks, the upload of chunk c + 1 overlapping chunk c ->
    every output Event delivered to a registered StreamCallback that counts them (sm_count_events_callback, the
    reference's performance-sample callback). Timed from the call to its return (H2D, matching, callbacks), best of 2,
    a fresh runtime each time. All four StockStream attributes are sent (36 B per event with the timestamp)."""
    import ctypes as ct
    from siddhi_amd import SiddhiManager, _lib
    L = _lib.lib()
    host = [c[:n].cpu().numpy() for c in cols_dev]
    ts_h, cols_h = host[4], host[:4]
    def one(columns):
        rt = SiddhiManager().createSiddhiAppRuntime(app_text)
        if chunk:
            _lib.check(L.sm_app_set_option(rt._h, b"bulk_chunk", int(chunk)))
        cnt = ct.c_int64(0)
        if columns:  # the Event[] of each callback call as columns (sm_app_add_stream_columns_callback, round 6)
            cb = _lib.COLUMNS_CB(("sm_count_columns_callback", L))
            _lib.check(L.sm_app_add_stream_columns_callback(rt._h, b"OutputStream", cb, ct.byref(cnt)))
        else:
            cb = _lib.STREAM_CB(("sm_count_events_callback", L))
            _lib.check(L.sm_app_add_stream_callback(rt._h, b"OutputStream", cb, ct.byref(cnt)))
        ih = rt.getInputHandler("StockStream")
        best = None
        for _ in range(2):
            _lib.check(L.sm_app_set_option(rt._h, b"reset", 1))
            cnt.value = 0
            t0 = time.perf_counter()
            ih.send_columns(ts_h, cols_h)
            dt = time.perf_counter() - t0
            if cnt.value != expect:
                raise RuntimeError(f"input-handler path delivered {cnt.value} output events, the device batch {expect}")
            best = dt if best is None else min(best, dt)
        path = ct.c_double()
        _lib.check(L.sm_app_get_stat(rt._h, b"fast_path:q", ct.byref(path)))
        phases = {}
        for ph in ("device", "outputs", "deliver", "callbacks", "upload_wait"):  # host time of the last run, per phase
            v = ct.c_double()
            _lib.check(L.sm_app_get_stat(rt._h, f"host_ms:{ph}".encode(), ct.byref(v)))
            phases[ph] = v.value
        rt.shutdown()
        del cb
        return best, int(path.value), phases

    best, path, phases = one(True)
    ev_best, _, ev_phases = one(False)
    return {"events": n, "value": n / best, "unit": "events/s", "ms": best * 1e3, "output_events": expect,
            "fast_path": path, "host_bytes_per_event": 36, "host_ms_last_run": phases,
            "callback": "columns StreamCallback (sm_app_add_stream_columns_callback: each call's Event[] as columns)",
            "events_form": {"value": n / ev_best, "ms": ev_best * 1e3, "host_ms_last_run": ev_phases,
                            "callback": "sm_event StreamCallback (sm_app_add_stream_callback)"},
            "note": "host columns -> sm_input_send_columns (InputHandler.send(Event[])) -> the closed form in "
                    "chunks (H2D of the next chunk overlapped) -> StreamCallback counting every output Event (value: "
                    "the columns form; events_form: Events as sm_event / sm_value records); best of 2, fresh runtime "
                    "each"}


def launch_command(gpus, argv, env, port=None):
    """How `bench.py --gpus N` gets N ranks. Under a launcher (WORLD_SIZE set) the process is one rank: WORLD_SIZE
    must equal N (a mismatch is an error, not a silently smaller run). Without one and N > 1, bench.py starts
    torch.distributed.run itself (one process per GPU, rendezvous on 127.0.0.1) with the same arguments and exits with
    its status: the returned command. None = run here as the only rank (N = 1) or as the launcher's rank."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (the launcher started a different number "
                             "of ranks)")
        return None
    if gpus <= 1:
        return None
    if port is None:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def run_plan(config, world, env=None):
    """How a run of `config` on `world` ranks is laid out (no GPU needed; tests/test_bench_launch.py). A configuration
    that shards (2: index ranges; 4, 5: keys) splits ONE stream of N events over the ranks, and value counts N; config
    3 (non-partitioned) runs `world` replicas and counts N x world. Several ranks always form an RCCL (nccl) group:
    configs 4 and 5 exchange keys over it (hash-by-key all-to-all), config 2 gathers its rows over it.
    SM_BENCH_BACKEND=gloo is a functional rehearsal only (several ranks sharing one GPU, which RCCL refuses; the
    collectives then stage through host memory) and reports rccl_world null."""
    cfg = CONFIGS[config]
    env = os.environ if env is None else env
    return {"shards": bool(cfg["shards"]), "units_factor": 1 if cfg["shards"] else world,
            "backend": env.get("SM_BENCH_BACKEND", "nccl") if world > 1 else None,
            "exchange": config in (4, 5) and world > 1,
            "scaling": cfg["scaling"]}


def key_partitions_line(app, N, K, ts_div, seed, rank, world, dev, hip_stream, steps, warmup):
    """Opt-in side line (`--key-partitions`, never `value`): rank r runs its own N-event stream on keys r*K .. r*K+K-1
    (disjoint PartitionRuntime instances share no state, core/partition/PartitionRuntime.java:256-309) with no
    data-path collective: weak scaling, N x world / the slowest rank's step time."""
    import torch
    import torch.distributed as dist
    symbol, price, _, _, ts = gen_stock(0, N, K, ts_div, dev, seed + 7919 * rank)
    symbol += rank * K

    def step():
        app.set_option("reset", 0)
        app.process_device_batch("StockStream", ts, [symbol, price, price, price], hip_stream=hip_stream)
        return app.device_matches("q")[1]

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item() / steps
    return {"value": N * world / dt, "unit": "events/s", "ms_per_step": dt * 1e3, "scaling": "weak",
            "events_per_rank": N, "keys_per_rank": K,
            "note": "side line: each rank its own stream on its own key range, no data-path collective"}


def build_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4, choices=sorted(CONFIGS))
    ap.add_argument("--events", type=float, default=None)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--ts-div", type=int, default=None)
    ap.add_argument("--cpu-sample", type=int, default=None)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="config 4: skip the end-to-end (H2D-inclusive) variant")
    ap.add_argument("--stack", type=int, default=0, choices=(0, 1, 2),
                    help="device-batch pipeline for configs 3/4: 0 automatic, 1 bucket stack, 2 sort / walk")
    ap.add_argument("--variant", default=None, choices=sorted(VARIANTS5),
                    help="config 5: the named emitting variant of the query")
    ap.add_argument("--query5", default=None,
                    help="config 5 diagnostic: this pattern / sequence body instead of the query (a side line only)")
    ap.add_argument("--select5", default="select e1.timestamp as a",
                    help="config 5 diagnostic: the select clause of --query5")
    ap.add_argument("--ih-events", type=float, default=1e8,
                    help="configs 3 and 4: events of the input-handler variant (host columns through sm_input_send_columns)")
    ap.add_argument("--via-input-handler", action="store_true",
                    help="configs 3 and 4: run the input-handler variant on all --events")
    ap.add_argument("--no-ih", action="store_true", help="configs 3 and 4: skip the input-handler variant")
    ap.add_argument("--ih-chunk", type=float, default=None, help="input-handler variant: option bulk_chunk")
    ap.add_argument("--no-sparse", action="store_true", help="config 4: skip the sparse 64-bit key variant")
    ap.add_argument("--key-partitions", action="store_true",
                    help="config 4 on N > 1 GPUs: also time the opt-in side line `key_partitions` (each rank its own "
                         "N-event stream on its own key range, no data-path collective, weak scaling); the headline "
                         "value is always the one exchanged stream")
    ap.add_argument("--heap-words", type=int, default=None,
                    help="NFA per-key partial-match arena (words per semispace; option heap_words)")
    return ap


def main():
    ap = build_parser()
    args = ap.parse_args()
    # before anything touches the GPU: N > 1 without a launcher starts one (a child process, never an exec)
    cmd = launch_command(args.gpus, sys.argv[1:], os.environ)
    if cmd is not None:
        import subprocess
        log(f"starting {args.gpus} ranks: {' '.join(cmd)}")
        sys.exit(subprocess.call(cmd))
    if os.environ.get("SM_BENCH_PROBE"):  # launcher test: report the rank layout and stop before any GPU call
        sys.stdout.write(json.dumps({"rank": int(os.environ.get("RANK", "0")),
                                     "world": int(os.environ.get("WORLD_SIZE", "1")), "gpus": args.gpus}) + "\n")
        sys.stdout.flush()
        return
    cfg = dict(CONFIGS[args.config])
    if args.variant:
        if args.config != 5:
            ap.error("--variant applies to config 5")
        cfg["app"] = app5_variant(VARIANTS5[args.variant])
        cfg["workload"] = f"config 5 variant {args.variant}: @app:playback partition with (symbol of A..E) " \
                          f"{VARIANTS5[args.variant]}"
        # a pattern keeps every A's partial until it completes (no `within`): a larger per-key arena
        cfg["options"] = {"heap_words": 4096}
    if args.query5:
        if args.config != 5:
            ap.error("--query5 applies to config 5")
        cfg["app"] = app5_variant(args.query5).replace(
            "select e1.timestamp as a, e2[0].timestamp as b0, e2[last].timestamp as bl, e3.timestamp as c, "
            "e4.timestamp as d", args.select5)
        cfg["workload"] = f"config 5 diagnostic query: {args.query5}"
        cfg["options"] = {"heap_words": 4096}

    import torch
    import torch.distributed as dist
    from siddhi_amd.testing import ProductApp
    from siddhi_amd.shard import (clock_ticks, concat_ordered, exchange_with_ordinals, merge_heartbeats,
                                  merge_outputs, partitioned_step, slice_starts)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    plan = run_plan(args.config, world)
    # (modulo the visible devices: a box with fewer GPUs than ranks shares them, a functional check only)
    local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    rccl_world = None
    if world > 1:
        # one process per GPU; the data path (key exchange, match return, output merge) runs over RCCL / xGMI
        if plan["backend"] == "nccl":
            dist.init_process_group("nccl", device_id=dev)
            rccl_world = dist.get_world_size()
        else:
            dist.init_process_group(plan["backend"])
    N = int(args.events if args.events is not None else cfg["events"])
    K = args.keys
    ts_div = args.ts_div if args.ts_div is not None else cfg["ts_div"]
    seed = seed_for(args.config)
    shards = plan["shards"]
    if shards:
        lo, hi = N * rank // world, N * (rank + 1) // world
    else:  # replicas: every rank runs the whole workload
        lo, hi = 0, N
    symbol, price, volume, tsattr, ts = gen_stock(lo, hi, K, ts_div, dev, seed)
    if args.config != 2:
        del volume  # not referenced by the pattern: the exchange ships only what the plan reads
        volume = price
    ordinals = torch.arange(lo, hi, dtype=torch.int64, device=dev) if args.config in (4, 5) else None
    sidx = gen_stream_idx(lo, hi, dev, seed) if args.config == 5 else None
    # multi-GPU constants of the exchange, made once: every slice's first ordinal, the in-slice offsets shipped in
    # the packed records, and the device buffer the per-rank match tuples are copied into for the return exchange
    starts = slice_starts(lo, world, dev) if world > 1 and shards else None
    offsets = torch.arange(hi - lo, dtype=torch.int32, device=dev) if world > 1 and shards else None
    mbuf = [None]
    out_local = [0]
    torch.cuda.synchronize()

    opts = dict(cfg.get("options", {}))
    # test only (tests/test_exchange_gpu.py, tools/rehearse_world4.sh): SM_BENCH_DUMP=<prefix> saves config 5's output
    # records of the last step, this rank's part of the delivery order, to <prefix>.rank<r>.pt (outside the timing)
    dump = os.environ.get("SM_BENCH_DUMP") if args.config == 5 else None
    last_recs = [None]
    if args.config == 5 and (world > 1 or dump):
        opts["keep_outputs"] = 1  # the output records of each batch stay on the device for the cross-rank merge
    if args.heap_words:
        opts["heap_words"] = args.heap_words
    app = ProductApp(cfg["app"], fast_stack=args.stack, **opts)
    # outputs are counted (the reference benchmark counts them in its callback), not collected as JSON
    app.set_collect(False)
    stream = torch.cuda.current_stream(dev)
    hip_stream = ctypes.c_void_p(stream.cuda_stream)
    n_local = [hi - lo]

    def step():
        if args.config == 5:
            # a fresh runtime of the app per step (state dropped, device allocations kept), then the batch
            app.set_option("reset", 1)
            if world > 1:
                # the global clock-advance points (one all-gather), the key exchange, then the heartbeats merged
                # into the received events on the device (shard.py, sm_merge_heartbeats): all inside the step
                ticks = clock_ticks(ts, lo, world)
                (s_sym, s_price, s_ts, s_sid), s_ord, _ = exchange_with_ordinals(
                    symbol, [symbol, price, ts, sidx], world, lo, starts=starts, offsets=offsets)
                s_sid, s_ts, (s_sym, s_price), s_ord = merge_heartbeats(s_sid, s_ts, [s_sym, s_price], s_ord, ticks)
            else:
                s_sym, s_price, s_ts, s_ord, s_sid = symbol, price, ts, ordinals, sidx
            n_local[0] = s_ts.numel()
            # columns: symbol, price, volume (not read: aliased), timestamp attribute = global ordinal
            app.process_device_events(s_sid, s_ts, [s_sym, s_price, s_price, s_ord], ordinals=s_ord,
                                      hip_stream=hip_stream)
            if world > 1:
                # the reference's single output order across ranks (shard.merge_outputs): every output record to the
                # rank that ingested its trigger, ordered there (timers of one clock advance in key creation order)
                merged = merge_outputs(app.copy_device_outputs("q"), starts, N, world)
                out_local[0] = merged.shape[0]
                if dump:
                    last_recs[0] = merged
            elif dump:
                last_recs[0] = app.copy_device_outputs("q")
            return int(app.get_stat("output_events:q"))
        # a fresh runtime of the app per step: the query's open partials (carried across device batches) dropped
        app.set_option("reset", 0)
        if args.config == 4:
            nm = [0]

            def match(cols, ords):
                # this rank's keys in global arrival order (with their global ordinals when sharded)
                s_sym, s_price, s_ts = cols
                n_local[0] = s_ts.numel()
                app.process_device_batch("StockStream", s_ts, [s_sym, s_price, s_price, s_price], ordinals=ords,
                                         hip_stream=hip_stream)
                m = nm[0] = app.device_matches("q")[1]
                if world == 1:
                    return None  # the output stays in the library's device buffer, in reference order
                if mbuf[0] is None or mbuf[0].numel() < m:
                    mbuf[0] = torch.empty(max(m, 1) + (m >> 3), dtype=torch.int64, device=dev)
                app.copy_device_matches("q", mbuf[0])
                return mbuf[0][:m]

            # the reference's single output order across ranks (shard.partitioned_step): key exchange, matching,
            # every tuple returned to the rank that ingested its e2 and ordered there
            mine = partitioned_step(symbol, [symbol, price, ts], world, lo, N, match, starts=starts, offsets=offsets)
            if mine is not None:
                out_local[0] = mine.numel()
            return nm[0]
        s_sym, s_price, s_ts, s_ord = symbol, price, ts, None
        n_local[0] = s_ts.numel()
        # columns: symbol, price, volume, timestamp (attributes the plan does not read are aliased)
        cols = [s_sym, s_price, volume if args.config == 2 else s_price, tsattr if args.config == 2 else s_price]
        app.process_device_batch("StockStream", s_ts, cols, ordinals=s_ord, ordinal_base=lo if args.config == 2 else 0,
                                 hip_stream=hip_stream)
        m = app.device_matches("q")[1]
        if world > 1 and shards:
            # config 2's index-range outputs are concatenated in rank order (shard.concat_ordered)
            if mbuf[0] is None or mbuf[0].numel() < m:
                mbuf[0] = torch.empty(max(m, 1) + (m >> 3), dtype=torch.int32, device=dev)
            app.copy_device_matches("q", mbuf[0])
            out_local[0] = concat_ordered(mbuf[0][:m].to(torch.int64) + lo, world).numel()
        return m

    log(f"rank {rank}: config {args.config}, {hi - lo} events resident; warmup {args.warmup}")
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
    if dump and last_recs[0] is not None:
        torch.save(last_recs[0].cpu(), f"{dump}.rank{rank}.pt")
    path = app.get_stat("fast_path:q")
    nfa_kernel = int(app.get_stat("nfa_kernel:q")) if args.config == 5 else 0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    m = torch.tensor([nm], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if shards:
            dist.all_reduce(m)
    dt = t.item()
    total_matches = m.item()
    ms_per_step = dt / args.steps * 1e3
    units = N * plan["units_factor"]  # sharded: the one stream; replicas: every rank processed a whole stream
    value = units / (dt / args.steps)
    kparts = None
    if args.key_partitions and args.config == 4 and world > 1:
        kparts = key_partitions_line(app, N, K, ts_div, seed, rank, world, dev, hip_stream, args.steps, args.warmup)

    from siddhi_amd import _lib
    build_id = _lib.lib().sm_build_id().decode()
    roof = roofline(ktot, n_local[0], nm, args.steps, args.config, build_id, args.variant)
    e2e = None
    if args.config == 4 and world == 1 and not args.no_e2e:
        # SURVEY.md §8(d) end-to-end variant: the same step with the three columns the plan reads (symbol i32,
        # price f64, event time i64: 20 B/event) copied host -> device first, from pinned host buffers, timed together
        log("e2e variant: pinning the host columns")
        host = [x.cpu().pin_memory() for x in (symbol, price, ts)]
        best = None
        for _ in range(2):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for d, h in zip((symbol, price, ts), host):
                d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            m_e2e = step()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            if m_e2e != nm:
                raise RuntimeError(f"e2e step found {m_e2e} matches, the device-resident steps {nm}")
            if best is None or t3 - t1 < best[1]:
                best = (t2 - t1, t3 - t1)
        del host
        e2e = {"ms_per_step": best[1] * 1e3, "value": N / best[1], "unit": "events/s", "h2d_ms": best[0] * 1e3,
               "h2d_GBps": 20 * N / best[0] / 1e9,
               "note": "H2D of symbol + price + event time from pinned host memory over PCIe, then the step; "
                       "not overlapped (best of 2)"}
    sparse = None
    if args.config == 4 and world == 1 and not args.no_sparse:
        # the same stream keyed by sparse 64-bit ids (splitmix64 of the dense symbol: K ids over the whole int64
        # range), `symbol long`: the keys become dense ids on the device (remap_keys) before key pass 0
        log("sparse-key variant")
        key64 = splitmix_torch(symbol.to(torch.int64) * 7919 + 11)
        app_s = ProductApp(APP.replace("symbol int", "symbol long"), fast_stack=args.stack)
        app_s.set_collect(False)

        def step_s():
            app_s.set_option("reset", 0)
            app_s.process_device_batch("StockStream", ts, [key64, price, price, price], hip_stream=hip_stream)
            return app_s.device_matches("q")[1]

        for _ in range(args.warmup):
            step_s()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            ms_ = step_s()
        torch.cuda.synchronize()
        dts = (time.perf_counter() - t1) / args.steps
        if ms_ != nm:
            raise RuntimeError(f"sparse-key run found {ms_} matches, the dense one {nm}")
        sparse = {"ms_per_step": dts * 1e3, "value": N / dts, "unit": "events/s",
                  "ratio_to_dense": dts * 1e3 / ms_per_step, "fast_path": int(app_s.get_stat("fast_path:q")),
                  "keys": "1e6 splitmix64 ids over the int64 range (symbol long), remapped to dense ids on the device"}
        app_s.close()
        del key64
    ih = None
    if args.config in (3, 4) and world == 1 and not args.no_ih:
        n_ih = N if args.via_input_handler else min(N, int(args.ih_events))
        log(f"input-handler variant on {n_ih} events")
        app.set_option("reset", 0)
        app.process_device_batch("StockStream", ts[:n_ih], [symbol[:n_ih], price[:n_ih], price[:n_ih], price[:n_ih]],
                                 hip_stream=hip_stream)
        expect = app.device_matches("q")[1]
        vol_attr = volume if volume is not price else None
        if vol_attr is None:  # the plan does not read volume: the host columns still carry it, as a caller's would
            vol_attr = torch.zeros(n_ih, dtype=torch.int64, device=dev)
        ih = via_input_handler([symbol, price, vol_attr, tsattr, ts], n_ih, expect,
                               int(args.ih_chunk) if args.ih_chunk else None, cfg["app"])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = args.cpu_sample or cfg["cpu_sample"]
        log(f"cpu baseline on {sample} events")
        v, sec, mm = cpu_baseline(sample, K, ts_div, cfg["app"], seed, cfg["out"], args.config)
        cpu = {"value": v, "unit": "events/s", "cores": 1, "kind": "port", **host_cpu(),
               "sample": f"first {sample} events of the same stream through oracle/cpu_ref "
                         f"(C++ restatement of the reference engine, 1 thread): {sec:.2f} s, {mm} matches"}
        nt = host_threads() if args.config != 3 else 1  # config 3 is one non-partitioned app: no split
        if nt > 1:
            # the generous baseline, the same sample split over host threads
            log(f"cpu baseline on {sample} events, {nt} threads")
            vt, sect, mt = cpu_baseline_threads(sample, K, ts_div, cfg["app"], seed, cfg["out"], args.config, nt)
            if mt != mm:
                raise RuntimeError(f"threaded CPU baseline found {mt} matches, 1 thread {mm}")
            cpu = {"value": vt, "unit": "events/s", "cores": nt, "kind": "port",
                   "sample": f"first {sample} events of the same stream through oracle/cpu_ref on {nt} host threads, "
                             f"one app per {'key shard (symbol % threads)' if args.config in (4, 5) else 'index range'}"
                             f"{' + global clock heartbeats' if args.config == 5 else ''}: {sect:.2f} s, {mt} matches",
                   "single_thread": {"value": v, "cores": 1, "seconds": sec}, **host_cpu()}
    if rank == 0:
        alg = cfg["job_bytes"](N, total_matches) * plan["units_factor"]
        conf = {"workload": cfg["workload"], "config": args.config, "events": N,
                "event_time": f"floor(i/{ts_div}) ms", "matches": total_matches,
                "parallelism": (f"key-sharded x{world} (one stream, hash-by-key RCCL all-to-all)"
                                if args.config in (4, 5) and world > 1 else
                                "single GPU" if world == 1 else
                                f"index-range-sharded x{world}" if cfg["shards"] else f"replicas x{world}"),
                "device_path": (("general NFA (interleaved device events), " +
                                 {1: "query-specialised kernel", 2: "interpreter"}.get(nfa_kernel, "?"))
                                if args.config == 5 else
                                ({1: "general closed form", 2: "sort / walk closed form", 3: "bucket-stack closed form"}
                                 if args.config in (3, 4) else {3: "filter interpreter", 4: "filter typed conjunction"})
                                .get(int(path), str(path))),
                "step_hbm_fraction": alg / (ms_per_step * 1e-3) / HBM_PEAK}
        if args.config in (4, 5):
            conf["keys"] = K
        conf["rccl_world"] = rccl_world
        conf["build_id"] = build_id
        conf["variant"] = args.variant or "literal"
        line = {
            "metric": METRIC if args.config == 4 else f"input events/sec + % HBM peak, {cfg['workload']}",
            "value": value, "unit": "events/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": plan["scaling"], "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (counter-based splitmix64 StockStream, device-resident)",
            "config": conf, "roofline": roof, "cpu_baseline": cpu,
        }
        if e2e:
            line["e2e_with_h2d"] = e2e
        if ih:
            line["via_input_handler"] = ih
        if sparse:
            line["sparse_keys"] = sparse
        if kparts:
            line["key_partitions"] = kparts
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Kernels of the device pipelines (labels recorded by kernels/fastpath3.hip and kernels/filter.hip) and their
# ALGORITHMIC bytes per launch for a batch of n events with m matches: what each launch must read
# and write at minimum.
KERNELS = ["prep", "key_up", "scan", "key_pass0", "key_pass", "walk", "j_count", "j_tile", "j_up", "j_pass",
           "j_pass_last",
           "stack_prep", "stack", "order", "carry_merge", "carry_out",
           "filter_count", "filter_scan", "filter_write",
           "event_index", "nfa_select", "nfa_group", "nfa_setup", "nfa"]


def alg_bytes(label, n, m, config):
    keyed = config == 4
    return {"prep": (12 * n) if keyed else (16 * n + n // 8),  # keyed: key i32 + ts i64 (c1 = price > 20 is
                                                              # evaluated in pass 0); unkeyed: ts + price in,
                                                              # c1 bit out
            "key_up": 16 * n,               # pass-1 digits: one 16-B record per event (the key word of each)
            "scan": 0,                      # per-chunk digit counts (O(chunks x 1024), not per event)
            "key_pass0": 20 * n + 16 * n,   # key i32 + price f64 + ts i64 in, 16-B keyed record out
            "key_pass": 16 * n + 16 * n,    # 16-B record in and out
            "walk": (16 * n + 8 * m) if keyed else (16 * n + n // 8 + 8 * m),  # records (unkeyed: price + ts +
                                                                               # c1 bits) in, (j, i) pairs out
            "stack_prep": 0,                # staging bases (O(kBins))
            "stack": 16 * n + 8 * m,        # bucket records in, staged (j, i) pairs out (bucket order)
            "order": 8 * m + 8 * m,         # staged pairs in, output pairs out (reference order)
            "carry_merge": 16 * m,
            "carry_out": 0,                 # open partials at the end of the batch (O(keys))
            "j_count": 8 * m,               # (j, i) pairs in: pairs per output j-tile
            "j_tile": 16 * m,               # (j, i) in (in i order) and out (in j order), once each
            "j_up": 4 * m,
            "j_pass": 16 * m,               # (j, i) in and out
            "j_pass_last": 16 * m,
            "filter_count": 16 * n + n // 8,  # price f64 + volume i64 in, one mask bit per event out
            "filter_scan": 0,
            "filter_write": n // 8 + 4 * m,   # mask in, u32 row per kept event out
            # config 5 (general NFA over an interleaved batch): index build reads event time + stream id and
            # writes row / ordinal / clock / advance points; the NFA kernel must at least read each event's key
            # position, stream id, event time, price and key (and write the output events)
            "event_index": 8 * n + 4 * n + 8 * 3 * n + 24 * n,
            "nfa_select": 4 * n + 8 * n,
            "nfa_group": 4 * n + 8 * n + 8 * n,
            "nfa_setup": 0,
            "nfa": 8 * n + 4 * n + 8 * n + 8 * n + 4 * n + 40 * m,
            }[label]


def roofline(ktot, n, m, steps, config, build_id=None, variant=None):
    """Dominant kernel (largest total time over the timed steps). `achieved` follows SURVEY.md §8(d): the job's
    algorithmic bytes per event / per match (config 4: 20 B per event + 8 B per match) x the events and matches
    one launch of it processes (the dominant kernel handles the whole batch), / its average launch duration
    (HIP events on the launch stream). The per-kernel breakdown keeps each kernel's own algorithmic bytes
    (alg_bytes) as a diagnostic; traffic_step sums the committed PMC bytes of every kernel of one step."""
    if not ktot:
        return None
    dom = max(ktot, key=lambda k: ktot[k][0])
    tot_ms, calls = ktot[dom]
    avg_ms = tot_ms / calls
    job = CONFIGS[config]["job_bytes"](n, m)
    ach = job / (avg_ms * 1e-3)
    own = alg_bytes(dom, n, m, config)
    brk = {k: {"avg_ms": v[0] / v[1], "calls_per_step": v[1] / steps,
               "gbps": alg_bytes(k, n, m, config) / (v[0] / v[1] * 1e-3) / 1e9} for k, v in ktot.items()}
    doc, why = pmc_doc(config, n, build_id, variant)
    traffic, src = pmc_traffic(doc, dom, config, variant)
    step_traffic = pmc_step_traffic(doc, brk)
    return {"bound": "hbm", "achieved": ach / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": ach / HBM_PEAK,
            "traffic": traffic, "traffic_unit": "HBM bytes per launch", "traffic_source": src or why,
            "kernel": dom, "avg_launch_ms": avg_ms, "alg_bytes_per_launch": job,
            "alg_bytes_basis": "SURVEY.md §8(d) job bytes of the batch the launch processes",
            "kernel_own_alg_bytes": own, "kernel_own_frac": own / (avg_ms * 1e-3) / HBM_PEAK,
            "traffic_step": step_traffic,
            "traffic_step_ratio": (step_traffic / job) if step_traffic else None,
            "breakdown": brk}


def pmc_path(config, variant=None):
    """profiles/pmc_config<C>.json (literal query) or profiles/pmc_config<C>_<variant>.json."""
    return os.path.join(ROOT, "profiles", f"pmc_config{config}" + (f"_{variant}" if variant else "") + ".json")


def pmc_doc(config, n, build_id, variant=None):
    """The committed PMC summary of this configuration (tools/summarize_profile.py, from separate rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this bench) if it describes THIS run: the same event count, the same query
    variant and the same library build (sm_build_id, a hash of the kernel sources and build flags). Otherwise
    (None, why): a profile of another build or variant never reaches the bench line."""
    path = pmc_path(config, variant)
    try:
        doc = json.load(open(path))
    except (OSError, ValueError):
        return None, f"no {os.path.relpath(path, ROOT)}"
    if doc.get("events") != n:
        return None, f"stale: {os.path.basename(path)} profiled {doc.get('events')} events, this run {n}"
    if doc.get("variant", "literal") != (variant or "literal"):
        return None, f"stale: {os.path.basename(path)} profiled variant {doc.get('variant')}"
    if build_id is None or doc.get("build_id") != build_id:
        return None, f"stale: {os.path.basename(path)} profiled build {doc.get('build_id')}, this build {build_id}"
    return doc, None


def pmc_step_traffic(doc, brk):
    """HBM bytes of one step: the committed PMC bytes per launch of every kernel label x its launches per step
    (None unless the summary matches this run and covers every kernel of the step)."""
    if doc is None:
        return None
    labels = doc.get("labels", {})
    tot = 0.0
    for lab, b in brk.items():
        ent = labels.get(lab)
        if ent is None:
            if lab == "scan":
                continue
            return None
        tot += ent.get("hbm_bytes", 0.0) * b["calls_per_step"]
    return tot


def pmc_traffic(doc, label, config, variant=None):
    """HBM bytes per launch of `label` from the matching PMC summary (pmc_doc), else (None, None)."""
    if doc is None:
        return None, None
    ent = doc.get("labels", {}).get(label)
    if not ent or not ent.get("hbm_bytes"):
        return None, None
    return ent["hbm_bytes"], (f"{os.path.relpath(pmc_path(config, variant), ROOT)} ({doc.get('tag')}, build "
                              f"{doc.get('build_id')}: {doc.get('method')})")


if __name__ == "__main__":
    main()
