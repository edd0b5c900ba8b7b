"""The bucket-stack pipeline's order kernel (siddhi_amd/csrc/kernels/order_dev.h, order2_kernel) run on the CPU under
the host wave emulator (tests/native/stack_emu.cpp), against a stable sort by j of the staged matches.

The stack kernel stages each bucket's matches in arrival order of j, the pops of one j consecutive and oldest e1
first (StreamPreStateProcessor.processAndReturn, core/query/input/stream/state/StreamPreStateProcessor.java:274-327,
walks the pending list oldest first); a j belongs to one bucket (its key's). The order kernel must emit every
(i, j) in (j, then staging order) — the reference's emission order — across all buckets. Cases: sparse tiles,
long runs of one j (more than a lane group), and tiles denser than the kernel's LDS images (its direct path).
Test infrastructure: no GPU; `-m "not gpu"`."""
import ctypes

import numpy as np
import pytest

from test_stack_emu import lib as emu_lib

BINS = 1024
TB = 13


def staged(ntiles, rate, seed, long_every=0, dense_tiles=()):
    """Random staged matches: every ordinal is owned by a random bucket and has Poisson(rate) matches (rate 1.3
    in dense_tiles; a run of 21 every long_every-th ordinal); i values are random."""
    rng = np.random.default_rng(seed)
    n = ntiles << TB
    owner = rng.integers(0, BINS, n)
    r = np.full(n, rate)
    for t in dense_tiles:
        r[t << TB:(t + 1) << TB] = 1.3
    cnt = rng.poisson(r)
    if long_every:
        cnt[::long_every] = 21
    j = np.repeat(np.arange(n, dtype=np.uint64), cnt)
    d = np.repeat(owner, cnt)
    i = rng.integers(0, 1 << 32, j.size, dtype=np.uint64)
    v = (j << np.uint64(32)) | i
    order = np.argsort(d, kind="stable")  # bucket runs, each in j order (pops of a j consecutive)
    stage = v[order]
    per = np.bincount(d, minlength=BINS).astype(np.int64)
    sbase = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.uint32)
    # mt[t][d]: matches of bucket d with j < t << TB
    jt = (j >> np.uint64(TB)).astype(np.int64)
    mt = np.zeros((ntiles + 1, BINS), np.int64)
    np.add.at(mt, (jt + 1, d), 1)
    mt = np.cumsum(mt, axis=0).astype(np.uint32)
    return stage, sbase, mt, v  # v is already in (j, staging order) order: the expected output


def run_order(stage, sbase, mt):
    l = emu_lib()
    l.sm_order2_emu.restype = ctypes.c_int
    out = np.zeros(stage.size, np.uint64)
    P = ctypes.c_void_p
    cap = l.sm_order2_emu(P(stage.ctypes.data), P(sbase.ctypes.data), P(mt.ctypes.data),
                          ctypes.c_int64(mt.shape[0] - 1), P(out.ctypes.data))
    return out, cap


@pytest.mark.parametrize("ntiles,rate,seed,long_every,dense", [
    (3, 0.7, 1, 0, ()),          # the bench's density: about 5.7k matches per tile
    (35, 0.05, 2, 0, ()),        # two workgroups (32 tiles each), sparse
    (5, 0.3, 3, 97, ()),         # runs of 21 matches of one j: segments longer than a lane group
    (6, 0.7, 4, 0, (1, 4)),      # tiles 1 and 4 outgrow the LDS images: the direct path between image tiles
    (1, 0.0, 5, 0, ()),          # no matches
])
def test_order2_emulated_equals_stable_sort_by_j(ntiles, rate, seed, long_every, dense):
    stage, sbase, mt, want = staged(ntiles, rate, seed, long_every, dense)
    got, cap = run_order(stage, sbase, mt)
    if dense:
        per_tile = np.diff(mt.astype(np.int64).sum(axis=1))
        assert (per_tile[list(dense)] > cap).all() and (np.delete(per_tile, list(dense)) <= cap).all()
    assert np.array_equal(got, want)
