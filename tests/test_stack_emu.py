"""The bucket-stack ring kernel (siddhi_amd/csrc/kernels/stack_dev.h, stack4_kernel) run on the CPU under the host
wave emulator (tests/native/stack_emu.cpp: the same device source, one fiber per GPU thread, wave64 operations
through per-wave barriers), against a plain pending-list model of the reference:
StreamPreStateProcessor.processAndReturn (core/query/input/stream/state/StreamPreStateProcessor.java:274-327)
walks a key's pending list oldest first, drops expired partials (isExpired :102-121), emits and removes those c2
accepts, keeps the rest; then the event's own partial is appended if c1 holds (addState :208-221).

Checked per bucket: the staged (j, i) matches in arrival order of j and pending-list order within j, the per-tile
staging offsets (mstart), the match totals, and the carry-out candidates (the partials still pending at the end,
oldest first per key). Test infrastructure: no GPU; `-m "not gpu"`."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
LIB = os.path.join(NATIVE, "build", os.environ.get("SM_STACK_EMU_LIB", "libstack_emu.so"))


def lib():
    src = [os.path.join(NATIVE, "stack_emu.cpp")]
    deps = src + [os.path.join(HERE, "..", "siddhi_amd", "csrc", "kernels", f)
                  for f in ("stack_dev.h", "fastpath_dev.h", "hd.h", "expr.h", "nfa.h")]
    if not os.path.exists(LIB) or any(os.path.getmtime(d) > os.path.getmtime(LIB) for d in deps):
        subprocess.check_call(["make", "-C", NATIVE, "emu"])
    l = ctypes.CDLL(LIB)
    l.sm_stack4_emu.restype = ctypes.c_int
    return l


def consts(l):
    out = (ctypes.c_int * 7)()
    l.sm_stack4_emu_consts(out)
    return dict(zip(["bins", "keys", "tb", "q", "ss", "r", "c"], list(out)))


def vcode(price):
    b = price.view(np.uint64).copy()
    b[price == 0.0] = 0
    neg = (b >> np.uint64(63)) != 0
    m = np.where(neg, ~b, b | np.uint64(1 << 63))
    return (m >> np.uint64(32)).astype(np.uint32)


def model(keys, price, ts, within, c1):
    """Per key pending lists: matches (i, j) in order of j then pending order; pending partials at the end."""
    pend = {}
    last = {}
    matches = []
    for j in range(len(keys)):
        k = int(keys[j])
        lst = pend.setdefault(k, [])
        keep = []
        for i in lst:
            if within >= 0 and ts[j] - ts[i] > within:
                continue
            if price[j] > price[i]:
                matches.append((i, j))
            else:
                keep.append(i)
        if c1[j]:
            keep.append(j)
        pend[k] = keep
        last[k] = ts[j]
    cand = []
    for k, lst in pend.items():
        for i in lst:
            if within < 0 or last[k] - ts[i] <= within:
                cand.append((k, i, int(ts[i]), i))
    return matches, sorted(cand)


def ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def run_case(n, K, div, within=1000, seed=1, grid=2, price=None, keys=None):
    l = lib()
    c = consts(l)
    rng = np.random.default_rng(seed)
    if keys is None:
        keys = rng.integers(0, K, n).astype(np.int64)
    if price is None:
        price = rng.random(n) * 100.0
    ts = (np.arange(n) // div).astype(np.int64)
    c1 = price > 20.0
    bins = c["bins"]
    H = ((K - 1) >> 10) + 1
    d = keys & (bins - 1)
    order = np.argsort(d, kind="stable")
    counts = np.bincount(d, minlength=bins)
    dbase = np.zeros(bins, np.uint32)
    dbase[1:] = np.cumsum(counts)[:-1]
    rec = np.zeros((n, 4), np.uint32)
    rec[:, 0] = (keys | (c1.astype(np.int64) << 31)).astype(np.uint32)
    rec[:, 1] = np.arange(n, dtype=np.uint32)
    rec[:, 2] = vcode(price)
    rec[:, 3] = (ts - ts[0]).astype(np.uint32)
    rec = np.ascontiguousarray(rec[order])
    ntiles = ((n - 1) >> c["tb"]) + 1
    stage = np.full(n, 0xFFFFFFFFFFFFFFFF, np.uint64)
    mstart = np.zeros(bins * (ntiles + 1), np.uint32)
    mtot = np.zeros(bins, np.uint32)
    cap = n + 1024
    cand = np.zeros(4 * cap, np.int64)
    cand_n = np.zeros(1, np.uint32)
    err = np.zeros(1, np.uint32)
    spill = np.zeros(grid * c["keys"] * c["q"] * 4, np.uint32)
    u32, i64, u64, f64 = ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
    rc = l.sm_stack4_emu(ptr(rec, u32), ptr(dbase, u32), u32(n), ctypes.c_int(H), ctypes.c_int32(within),
                         u32(ntiles), ctypes.c_int(grid), ptr(price, f64), i64(0), i64(int(ts[0])), i64(0),
                         ctypes.c_int32(0), None, None, None, None, ptr(dbase, u32), ptr(stage, u64),
                         ptr(mstart, u32), ptr(mtot, u32), ptr(cand, i64), u32(cap), ptr(cand_n, u32),
                         ptr(err, u32), ptr(spill, u32))
    assert rc == 0
    matches, exp_cand = model(keys, price, ts, within, c1)
    return dict(keys=keys, d=d, dbase=dbase, counts=counts, stage=stage, mstart=mstart.reshape(bins, ntiles + 1),
                mtot=mtot, cand=cand[:4 * int(cand_n[0])].reshape(-1, 4), err=int(err[0]), matches=matches,
                exp_cand=exp_cand, ntiles=ntiles, tb=c["tb"], bins=bins)


def check(r):
    assert r["err"] == 0, f"kernel error flags {r['err']:#x}"
    bins, tb = r["bins"], r["tb"]
    per = [[] for _ in range(bins)]
    for i, j in r["matches"]:  # already in order of j, then pending order
        per[int(r["d"][j])].append((j << 32) | i)
    for b in range(bins):
        exp = np.array(per[b], np.uint64)
        assert int(r["mtot"][b]) == len(exp), f"bucket {b}: {int(r['mtot'][b])} matches, expected {len(exp)}"
        got = r["stage"][r["dbase"][b]:r["dbase"][b] + len(exp)]
        assert np.array_equal(got, exp), f"bucket {b}: staged matches differ"
        js = exp >> np.uint64(32)
        t = np.arange(r["ntiles"] + 1, dtype=np.uint64) << np.uint64(tb)
        assert np.array_equal(r["mstart"][b], np.searchsorted(js, t, side="left").astype(np.uint32)), \
            f"bucket {b}: tile offsets differ"
    got_cand = sorted(tuple(int(x) for x in row) for row in r["cand"])
    assert got_cand == r["exp_cand"]


@pytest.mark.parametrize("n,K,div", [(3000, 200, 10), (20000, 200, 10), (20000, 5000, 3), (60000, 3000, 30)])
def test_stack4_emulated_equals_pending_list_model(n, K, div):
    check(run_case(n, K, div))


def test_stack4_emulated_no_within_spills():
    """no `within`: each key's stack grows past its register part (spill ring) on falling runs of 30 events, and the
    rise after each run pops it whole, through the refills of the spilled entries"""
    n = 6000
    i = np.arange(n)
    keys = (i % 50).astype(np.int64)
    price = 99.0 - ((i // 50) % 31) * 2.5
    check(run_case(n, 50, 1, within=-1, price=price, keys=keys))
