"""`bench.py --gpus N` means N ranks: without a launcher it starts torch.distributed.run with N
processes itself; under a launcher whose WORLD_SIZE differs from N it fails instead of timing fewer GPUs. The
multi-rank config-4 step (shard.partitioned_step, the code bench.py runs over RCCL) is checked here on CPU with gloo
at world 2: the ranks' outputs in rank order equal the world-1 output, on bench.py's own synthetic stream. The
per-rank matcher is the CPU oracle (this checks the sharding of the step; the kernels are checked in the -m gpu
tests)."""
import ctypes
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, K, DIV = 100_000, 3000, 10


def test_launch_command_rules():
    assert bench.launch_command(1, [], {}) is None
    assert bench.launch_command(8, [], {"WORLD_SIZE": "8"}) is None
    with pytest.raises(SystemExit):
        bench.launch_command(8, [], {"WORLD_SIZE": "1"})
    cmd = bench.launch_command(4, ["--gpus", "4", "--steps", "3"], {}, port=29999)
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd and "--master-port=29999" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(kw)
    return env


@pytest.mark.timeout(300)
def test_bench_starts_its_ranks():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=_env(SM_BENCH_PROBE="1"),
                         capture_output=True, text=True, timeout=280)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 and d["gpus"] == 2 for d in lines)


@pytest.mark.timeout(120)
def test_bench_refuses_world_mismatch():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                         env=_env(WORLD_SIZE="2", RANK="0", SM_BENCH_PROBE="1"), capture_output=True, text=True,
                         timeout=110)
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


def oracle_match(cols, ords):
    """The CPU oracle as a rank's matcher: packed (e2 << 32) | e1 global-ordinal tuples in its output order."""
    from oracle_lib import OracleApp, lib as olib
    sym, price, ts = (c.numpy() for c in cols)
    o = np.arange(len(ts), dtype=np.int64) if ords is None else ords.numpy()
    cs = [np.ascontiguousarray(sym), np.ascontiguousarray(price), np.zeros(len(ts), dtype=np.int64),
          np.ascontiguousarray(o)]
    a = OracleApp(bench.APP)
    a.start()
    ptrs = (ctypes.c_void_p * 4)(*[c.ctypes.data for c in cs])
    err = ctypes.create_string_buffer(512)
    tsa = np.ascontiguousarray(ts, dtype=np.int64)
    rc = olib().cr_send_columns(a.h, a.stream_index("StockStream"), len(tsa), tsa.ctypes.data, ptrs, err, 512)
    assert rc == 0, err.value
    out = a.outputs()["streams"].get("OutputStream", [])
    a.close()
    p = np.array([r[1] for r in out], dtype=np.int64).reshape(-1, 2)  # the selected e1 / e2 timestamp attributes
    return torch.from_numpy((p[:, 1] << 32) | p[:, 0])


def _rank(rank, world, port, outfile):
    from siddhi_amd.shard import partitioned_step
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = N * rank // world, N * (rank + 1) // world
        sym, price, vol, tsa, ts = bench.gen_stock(lo, hi, K, DIV, torch.device("cpu"), bench.seed_for(4))
        mine = partitioned_step(sym, [sym, price, ts], world, lo, N, oracle_match)
        parts = [None] * world
        dist.all_gather_object(parts, mine.tolist())
        if rank == 0:
            with open(outfile, "w") as f:
                json.dump(parts, f)
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_partitioned_step_world2_equals_world1(tmp_path):
    from siddhi_amd.shard import partitioned_step
    out = str(tmp_path / "parts.json")
    mp.start_processes(_rank, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    parts = json.load(open(out))
    sym, price, vol, tsa, ts = bench.gen_stock(0, N, K, DIV, torch.device("cpu"), bench.seed_for(4))
    single = partitioned_step(sym, [sym, price, ts], 1, 0, N, oracle_match)
    assert single.numel() > 0.3 * N
    got = np.concatenate([np.asarray(p, dtype=np.int64) for p in parts])
    np.testing.assert_array_equal(got, single.numpy())


def test_default_multi_gpu_plan_is_the_exchanged_stream():
    """`bench.py --gpus N` (config 4, no flags) measures BASELINE's configuration, one stream of N
    events routed by key over RCCL: value counts N (strong scaling), not N x world."""
    args = bench.build_parser().parse_args(["--gpus", "2"])
    assert args.config == 4 and not args.key_partitions
    plan = bench.run_plan(args.config, 2, env={})
    assert plan == {"shards": True, "units_factor": 1, "backend": "nccl", "exchange": True, "scaling": "strong"}
    for c in (2, 5):
        p = bench.run_plan(c, 8, env={})
        assert p["units_factor"] == 1 and p["backend"] == "nccl"
    assert bench.run_plan(5, 8, env={})["exchange"]
    # config 3 does not shard: replicas, counted per rank
    p3 = bench.run_plan(3, 4, env={})
    assert p3["units_factor"] == 4 and p3["scaling"] == "weak" and not p3["exchange"]
    assert bench.run_plan(4, 1, env={})["backend"] is None
    assert bench.run_plan(4, 2, env={"SM_BENCH_BACKEND": "gloo"})["backend"] == "gloo"


def test_stale_pmc_profile_yields_null_traffic(tmp_path, monkeypatch):
    """the roofline's PMC traffic is reported only when the committed summary names the same
    event count, query variant and library build (sm_build_id) as the running bench."""
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    (tmp_path / "profiles").mkdir()
    n, m = 1000, 400
    ktot = {"stack": [10.0, 5], "order": [2.0, 5]}
    doc = {"config": 4, "events": n, "matches": m, "tag": "t", "build_id": "abcd", "variant": "literal",
           "method": "x", "labels": {"stack": {"hbm_bytes": 5e4}, "order": {"hbm_bytes": 1e4}}}
    (tmp_path / "profiles" / "pmc_config4.json").write_text(json.dumps(doc))
    r = bench.roofline(ktot, n, m, 5, 4, build_id="abcd")
    assert r["traffic"] == 5e4 and r["traffic_step"] == 6e4 and "build abcd" in r["traffic_source"]
    r = bench.roofline(ktot, n, m, 5, 4, build_id="ffff")
    assert r["traffic"] is None and r["traffic_step"] is None and "stale" in r["traffic_source"]
    r = bench.roofline(ktot, n + 1, m, 5, 4, build_id="abcd")
    assert r["traffic"] is None
    # a variant reads its own file; the literal query's profile never stands in for it
    r = bench.roofline(ktot, n, m, 5, 4, build_id="abcd", variant="pattern_count_not5s")
    assert r["traffic"] is None and "no profiles/pmc_config4_pattern_count_not5s.json" in r["traffic_source"]
    doc["variant"] = "pattern_count_not5s"
    (tmp_path / "profiles" / "pmc_config4_pattern_count_not5s.json").write_text(json.dumps(doc))
    assert bench.roofline(ktot, n, m, 5, 4, build_id="abcd", variant="pattern_count_not5s")["traffic"] == 5e4
