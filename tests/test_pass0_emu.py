"""Key pass 0 (siddhi_amd/csrc/kernels/pass0_dev.h, pass0_kernel) run on the CPU under the host wave emulator
(tests/native/pass0_emu.cpp: the same device source, one fiber per GPU thread): its output must be the stable
partition of the 16-byte keyed records by the key's low 10-bit digit, which is what the partitioned key lookup of the
reference (core/partition/PartitionRuntime / PartitionStreamReceiver: events of one key stay in arrival order) needs
of the bucketing. Chunk counts and digit bases are computed as the host does (fastpath3.hip: per = round_up(n/G,
4096), cnt[d*G+g] = records of digit d in chunks before g). Test infrastructure: no GPU; `-m "not gpu"`."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")
LIB = os.path.join(NATIVE, "build", os.environ.get("SM_PASS0_EMU_LIB", "libpass0_emu.so"))
TILE, BINS = 4096, 1024


def lib():
    deps = [os.path.join(NATIVE, "pass0_emu.cpp"), os.path.join(NATIVE, "emu_fibers.h")] + [
        os.path.join(HERE, "..", "siddhi_amd", "csrc", "kernels", f) for f in ("pass0_dev.h", "fastpath_dev.h", "hd.h")]
    if not os.path.exists(LIB) or any(os.path.getmtime(d) > os.path.getmtime(LIB) for d in deps):
        subprocess.check_call(["make", "-C", NATIVE, "pass0emu"])
    return ctypes.CDLL(LIB)


def run(keys, G):
    n = len(keys)
    rng = np.random.default_rng(n)
    rec = np.zeros((n, 4), np.uint32)
    rec[:, 0] = keys.astype(np.uint32) | (rng.integers(0, 2, n).astype(np.uint32) << np.uint32(31))
    rec[:, 1] = np.arange(n, dtype=np.uint32)
    rec[:, 2] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    rec[:, 3] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    per = -(-(-(-n // G)) // TILE) * TILE
    d = rec[:, 0] & (BINS - 1)
    cnt = np.zeros((BINS, G), np.uint32)
    for g in range(G):
        c = np.bincount(d[g * per:(g + 1) * per], minlength=BINS)
        if g + 1 < G:
            cnt[:, g + 1] = cnt[:, g] + c
    tot = np.bincount(d, minlength=BINS)
    dbase = np.zeros(BINS, np.uint32)
    dbase[1:] = np.cumsum(tot)[:-1]
    out = np.full((n, 4), 0xDEADBEEF, np.uint32)
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))
    cnt = np.ascontiguousarray(cnt)
    assert lib().sm_pass0_emu(P(rec), ctypes.c_int64(n), ctypes.c_int64(per), ctypes.c_int(G), P(cnt), P(dbase),
                              P(out)) == 0
    exp = rec[np.argsort(d, kind="stable")]
    assert np.array_equal(out, exp)


@pytest.mark.parametrize("n,K,G", [(1, 1000, 1), (4095, 1 << 20, 1), (4096 * 3 + 17, 5000, 2), (40000, 1 << 20, 3),
                                   (30000, 7, 2), (20000, 1, 1), (9000, 1 << 20, 4)])
def test_pass0_emulated_is_stable_digit_partition(n, K, G):
    keys = np.random.default_rng(K + n).integers(0, K, n)
    run(keys, G)


def test_pass0_emulated_runs_straddle_segments():
    """digit runs of 1..7 records per tile, so most runs end inside a 64-byte segment: exercises the carry"""
    n = 4096 * 5 + 300
    i = np.arange(n)
    keys = (i // 3) % 1400 * 7 % 1024 + ((i * 2654435761) % 5 == 0) * 1024
    run(keys, 2)
