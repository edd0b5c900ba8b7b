"""Key sharding of a partitioned stream across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

The reference runs every partition key in one JVM (PartitionStreamReceiver.receive
core/partition/PartitionStreamReceiver.java:156 → PartitionRuntime.cloneIfNotExist core/partition/PartitionRuntime.java:256):
keys are independent, and for one input event only the runtime of that event's key runs. So a partitioned app
shards by key with ONE exchange step: every rank ingests a contiguous slice of the arrival order, computes the
owner rank of each event's key (`owner_of`: a splitmix64 hash of the key, so structured keys still spread), and
the ranks swap events with one all-to-all-v of packed records (`exchange_with_ordinals`: every event's fields in
one record, so one collective per step whatever the number of columns). Each rank then holds the complete event
sequence of the keys it owns, in global arrival order (stable local order + contiguous rank slices), with the
events' global ordinals, so the per-rank device pipeline returns exactly the reference's match tuples of those
keys.

Output order: every event belongs to one key, hence the matches triggered by one event (one e2) come from one
rank. `return_matches` sends each match tuple back to the rank whose ingest slice holds its e2 (one all-to-all-v;
the per-rank tuples are e2-ordered, so the split points are a binary search) and `order_matches` (HIP) puts the
received runs into the reference's order for that slice: the ranks' outputs concatenated in rank order are the
single-process output. `concat_ordered` is the same idea for index-range shards (the filter of config 2).
"""
import torch
import torch.distributed as dist

# partition keys: 32- or 64-bit integers (the owner hash reads the key's 64-bit two's complement; a narrower key
# would need its signedness passed to the device, so it is widened by the caller instead)
_INT_DTYPES = (torch.int32, torch.int64)
_BY_WIDTH = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def _staged(t: torch.Tensor, group) -> bool:
    """A collective on device tensors over a gloo group (the functional rehearsal of the multi-GPU path with several
    ranks sharing one GPU, where RCCL refuses duplicate devices) goes through host copies; over RCCL the tensors stay
    in HBM and the collective runs over xGMI."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_to_all_single(out, inp, out_splits=None, in_splits=None, group=None):
    if _staged(inp, group):
        h = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
        return
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def _all_gather(outs, t, group=None):
    if _staged(t, group):
        hs = [torch.empty(o.shape, dtype=o.dtype) for o in outs]
        dist.all_gather(hs, t.cpu(), group=group)
        for o, h in zip(outs, hs):
            o.copy_(h)
        return
    dist.all_gather(outs, t, group=group)


def _i64(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def _check_keys(keys: torch.Tensor):
    if keys.dtype not in _INT_DTYPES:
        raise TypeError(f"partition keys must be an int32 or int64 tensor, got {keys.dtype} (widen a narrower "
                        "integer key, hash a non-integer key to an integer first)")
    if keys.dim() != 1:
        raise ValueError("partition keys must be a 1-D tensor")


def owner_of(keys: torch.Tensor, world: int) -> torch.Tensor:
    """Owning rank of each key: hi32(splitmix64 finaliser of the key's 64-bit two's complement) mod world — the
    function kernels/partition.h key_owner computes on the GPU (wrap-around int64 arithmetic, logical shifts)."""
    _check_keys(keys)
    z = keys.to(torch.int64)
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _i64(0x94D049BB133111EB)
    z = z ^ ((z >> 31) & ((1 << 33) - 1))
    return ((z >> 32) & 0xFFFFFFFF) % world


def _launch_partition(keys, world, srcs, dsts, widths, strides):
    import ctypes
    from siddhi_amd import _lib
    k = len(srcs)
    cw = (ctypes.c_int32 * k)(*widths)
    cs = (ctypes.c_int32 * k)(*strides)
    src = (ctypes.c_void_p * k)(*srcs)
    dst = (ctypes.c_void_p * k)(*dsts)
    counts = (ctypes.c_uint64 * world)()
    stream = ctypes.c_void_p(torch.cuda.current_stream(keys.device).cuda_stream)
    rc = _lib.lib().sm_partition_by_owner(keys.data_ptr(), keys.element_size(), keys.numel(), world, k, cw, cs, src,
                                          dst, counts, stream)
    if rc != _lib.SM_OK:
        raise RuntimeError(_lib.lib().sm_last_error().decode(errors="replace"))
    return [int(c) for c in counts]


def _check_columns(keys, columns):
    for c in columns:
        if c.dim() != 1 or c.numel() != keys.numel() or c.device != keys.device or not c.is_contiguous():
            raise ValueError("columns must be contiguous 1-D tensors aligned with the keys, on the keys' device")
        if c.element_size() not in _BY_WIDTH:
            raise ValueError(f"column element size {c.element_size()} not supported")


def partition_by_owner(keys: torch.Tensor, columns, world: int):
    """Stable partition of `columns` by owner rank: (partitioned columns, per-owner counts). On the GPU this is
    the HIP counting sort of the native library (one read of the key + one read and write of each column); host
    tensors (the gloo CPU tests) take the equivalent torch form."""
    _check_keys(keys)
    _check_columns(keys, columns)
    if keys.is_cuda:
        outs = [torch.empty_like(c) for c in columns]
        w = [c.element_size() for c in columns]
        counts = _launch_partition(keys, world, [c.data_ptr() for c in columns], [o.data_ptr() for o in outs], w, w)
        return outs, counts
    owner = owner_of(keys, world)
    order = torch.argsort(owner, stable=True)
    return [c[order] for c in columns], torch.bincount(owner, minlength=world).tolist()


def record_layout(columns):
    """Packed record of one event: fields in decreasing width (so each is aligned to its width), the record
    padded to 8 bytes. Returns ([(offset, width)] in column order, record bytes)."""
    order = sorted(range(len(columns)), key=lambda c: -columns[c].element_size())
    off, lay = 0, [None] * len(columns)
    for c in order:
        w = columns[c].element_size()
        lay[c] = (off, w)
        off += w
    return lay, (off + 7) // 8 * 8


def pack_by_owner(keys: torch.Tensor, columns, world: int):
    """Partition by owner and pack in one pass: an int64 (n, R/8) record tensor grouped by owner rank (arrival
    order within an owner) + per-owner counts. On the GPU the partition kernel writes the records directly
    (sm_partition_by_owner with strides = R)."""
    _check_keys(keys)
    _check_columns(keys, columns)
    lay, R = record_layout(columns)
    n = keys.numel()
    rec = torch.empty((n, R // 8), dtype=torch.int64, device=keys.device)
    if keys.is_cuda:
        base = rec.data_ptr()
        counts = _launch_partition(keys, world, [c.data_ptr() for c in columns], [base + o for o, _ in lay],
                                   [w for _, w in lay], [R] * len(columns))
        return rec, counts, lay
    owner = owner_of(keys, world)
    order = torch.argsort(owner, stable=True)
    for c, (o, w) in zip(columns, lay):
        rec.view(_BY_WIDTH[w]).view(n, R // w)[:, o // w] = c[order].view(_BY_WIDTH[w])
    return rec, torch.bincount(owner, minlength=world).tolist(), lay


def unpack(rec: torch.Tensor, lay, dtypes):
    """Columns (contiguous) of a packed record tensor."""
    m = rec.shape[0]
    R = rec.shape[1] * 8 if rec.dim() == 2 else 8
    out = []
    for (o, w), dt in zip(lay, dtypes):
        out.append(rec.view(_BY_WIDTH[w]).view(m, R // w)[:, o // w].contiguous().view(dt))
    return out


def _all_to_all_counts(send_counts, device, group):
    sc = torch.tensor(send_counts, dtype=torch.int64, device=device)
    rc = torch.empty_like(sc)
    _all_to_all_single(rc, sc, group=group)
    return rc.tolist()


def unpack_with_ordinals(rec: torch.Tensor, lay, dtypes, rc, starts):
    """Received packed records → contiguous columns (all but the last field) + int64 global ordinals from the last
    field (the uint32 offset inside the source rank's slice) and the sources' first ordinals `starts`, the runs given
    by the received counts `rc`. GPU: one pass of the native library (sm_unpack_records); host tensors: unpack +
    torch arithmetic (the same values)."""
    m = rec.shape[0]
    if rec.is_cuda:
        import ctypes
        from siddhi_amd import _lib
        R = rec.shape[1] * 8
        k = len(lay)
        outs = [torch.empty(m, dtype=dt, device=rec.device) for dt in dtypes[:-1]]
        ords = torch.empty(m, dtype=torch.int64, device=rec.device)
        offs = (ctypes.c_int32 * k)(*[o for o, _ in lay])
        wids = (ctypes.c_int32 * k)(*[w for _, w in lay])
        dst = (ctypes.c_void_p * k)(*([t.data_ptr() for t in outs] + [None]))
        cnt = (ctypes.c_uint64 * len(rc))(*[int(x) for x in rc])
        first = (ctypes.c_int64 * len(rc))(*[int(x) for x in starts])
        stream = ctypes.c_void_p(torch.cuda.current_stream(rec.device).cuda_stream)
        r = _lib.lib().sm_unpack_records(rec.data_ptr(), m, R, k, offs, wids, dst, k - 1, len(rc), cnt, first,
                                         ords.data_ptr(), stream)
        if r != _lib.SM_OK:
            raise RuntimeError(_lib.lib().sm_last_error().decode(errors="replace"))
        return outs, ords
    cols = unpack(rec, lay, dtypes)
    base = torch.repeat_interleave(torch.tensor(starts, dtype=torch.int64, device=rec.device),
                                   torch.tensor(rc, dtype=torch.int64, device=rec.device))
    return cols[:-1], base + (cols[-1].to(torch.int64) & 0xFFFFFFFF)


def exchange_by_key(keys: torch.Tensor, columns, world: int, group=None, packed=False):
    """All-to-all-v of `columns` (list of 1-D tensors aligned with `keys`) so that each rank receives the rows
    whose key it owns, as ONE packed record per row through ONE collective. Returns (received columns, received
    counts per source rank). Row order in the result: by source rank, then original order — i.e. global arrival
    order when rank r holds the r-th contiguous slice."""
    _check_keys(keys)
    if world == 1:
        return list(columns), [keys.numel()]
    rec, sc, lay = pack_by_owner(keys, columns, world)
    rc = _all_to_all_counts(sc, keys.device, group)
    buf = torch.empty((sum(rc), rec.shape[1]), dtype=torch.int64, device=keys.device)
    _all_to_all_single(buf, rec, rc, sc, group=group)
    if packed:  # the caller unpacks (exchange_with_ordinals: one pass with the ordinals)
        return (buf, lay), rc
    return unpack(buf, lay, [c.dtype for c in columns]), rc


def slice_starts(lo: int, world: int, device, group=None):
    """First global ordinal of every rank's ingest slice (all-gathered; a list of world ints)."""
    los = torch.tensor([lo], dtype=torch.int64, device=device)
    all_lo = [torch.empty_like(los) for _ in range(world)]
    _all_gather(all_lo, los, group=group)
    return [int(x.item()) for x in all_lo]


def exchange_with_ordinals(keys: torch.Tensor, columns, world: int, lo: int, group=None, starts=None, offsets=None):
    """exchange_by_key plus the global arrival ordinal of every received row. The ordinal is not shipped as an
    int64: each record carries the row's uint32 offset inside its source rank's contiguous slice, and the receiver
    adds the source slice's first ordinal (`starts`, all-gathered once and reusable across steps), saving 4 of the
    bytes per event that cross xGMI. `offsets` (int32 arange of the slice) may be passed to reuse it across steps.
    Returns (received columns, received int64 ordinals, received counts per source rank)."""
    n = keys.numel()
    if world == 1:
        return list(columns), torch.arange(lo, lo + n, dtype=torch.int64, device=keys.device), [n]
    if n >= 2**31:
        raise ValueError("exchange_with_ordinals: more than 2^31 events in one rank's slice")
    off = offsets if offsets is not None else torch.arange(n, dtype=torch.int32, device=keys.device)
    cols = list(columns) + [off]
    (buf, lay), rc = exchange_by_key(keys, cols, world, group=group, packed=True)
    if starts is None:
        starts = slice_starts(lo, world, keys.device, group)
    out, ords = unpack_with_ordinals(buf, lay, [c.dtype for c in cols], rc, starts)
    return out, ords, rc


def pack_pairs(e1: torch.Tensor, e2: torch.Tensor) -> torch.Tensor:
    """(e2 << 32) | uint32(e1) as int64 — the layout of the device match tuples (uint32 e1, e2 interleaved)."""
    return (e2.to(torch.int64) << 32) | (e1.to(torch.int64) & 0xFFFFFFFF)


def unpack_pairs(p: torch.Tensor):
    """(e1, e2) int64 tensors of packed tuples (e1 as signed 32-bit)."""
    e1 = (p & 0xFFFFFFFF)
    e1 = torch.where(e1 >= 1 << 31, e1 - (1 << 32), e1)
    return e1, p >> 32


def order_matches(pairs: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    """Received match tuples (int64 packed, every e2 in [lo, hi); a concatenation of runs each in (e2, e1) order,
    one e2's tuples all in one run) → the reference's output order for that slice. GPU: sm_order_matches (count
    per e2, scan, place: HBM-bound, no comparison sort); host tensors: a stable sort by e2."""
    if pairs.dtype != torch.int64 or pairs.dim() != 1:
        raise TypeError("pairs must be a 1-D int64 tensor of packed (e2 << 32 | e1) tuples")
    if pairs.numel() == 0:
        return pairs.clone()
    if pairs.is_cuda:
        import ctypes
        from siddhi_amd import _lib
        out = torch.empty_like(pairs)
        stream = ctypes.c_void_p(torch.cuda.current_stream(pairs.device).cuda_stream)
        rc = _lib.lib().sm_order_matches(pairs.data_ptr(), pairs.numel(), lo, hi, out.data_ptr(), stream)
        if rc != _lib.SM_OK:
            raise RuntimeError(_lib.lib().sm_last_error().decode(errors="replace"))
        return out
    e2 = pairs >> 32
    if int(e2.min()) < lo or int(e2.max()) >= hi:
        raise ValueError("a match tuple's e2 lies outside the slice")
    return pairs[torch.argsort(e2, stable=True)]


def return_matches(pairs: torch.Tensor, starts, hi_last: int, world: int, group=None) -> torch.Tensor:
    """Send every match tuple (int64 packed, this rank's tuples in reference order for its keys) to the rank whose
    ingest slice holds its e2 (`starts` = slice_starts, the last slice ending at hi_last), then order what this
    rank received (order_matches). One all-to-all-v of 8 bytes per tuple; the split points are a binary search
    since the tuples are e2-ordered. Returns this rank's slice of the global output, in reference order."""
    rank = dist.get_rank(group)
    lo = starts[rank]
    hi = starts[rank + 1] if rank + 1 < world else hi_last
    if world == 1:
        return pairs
    e2 = pairs >> 32
    bnd = torch.searchsorted(e2, torch.tensor(starts[1:], dtype=torch.int64, device=pairs.device))
    cuts = [0] + bnd.tolist() + [pairs.numel()]
    sc = [cuts[r + 1] - cuts[r] for r in range(world)]
    rc = _all_to_all_counts(sc, pairs.device, group)
    buf = torch.empty(sum(rc), dtype=torch.int64, device=pairs.device)
    _all_to_all_single(buf, pairs, rc, sc, group=group)
    return order_matches(buf, lo, hi)


def partitioned_step(keys: torch.Tensor, columns, world: int, lo: int, n_total: int, match, starts=None,
                     offsets=None, group=None) -> torch.Tensor:
    """One step of a key-sharded partitioned pattern (bench.py config 4), from this rank's contiguous ingest slice
    [lo, lo + len) to its slice of the global output: exchange_with_ordinals (one packed record per event, one
    all-to-all-v) → `match(received columns, global ordinals or None)`, which returns this rank's match tuples (int64
    (e2 << 32) | e1, global ordinals, reference order for its keys) → return_matches (each tuple to the rank that
    ingested its e2, ordered there). The ranks' results in rank order are the single-process output. With world 1
    the columns go to `match` unchanged (ordinals None: positions are the global ordinals)."""
    if world == 1:
        return match(list(columns), None)
    recv, ords, _ = exchange_with_ordinals(keys, columns, world, lo, group=group, starts=starts, offsets=offsets)
    if starts is None:
        starts = slice_starts(lo, world, keys.device, group)
    return return_matches(match(recv, ords), starts, n_total, world, group=group)


def concat_ordered(rows: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """Index-range shards (config 2: rank r filtered the r-th contiguous slice of the arrival order): every rank's
    kept rows (global ordinals, ordered) concatenated in rank order = the single-process output order. All-gather
    of the per-rank counts, then of the rows padded to the largest count; every rank gets the whole output."""
    if world == 1:
        return rows
    cnt = torch.tensor([rows.numel()], dtype=torch.int64, device=rows.device)
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    _all_gather(cnts, cnt, group=group)
    cs = [int(c.item()) for c in cnts]
    mx = max(cs)
    pad = torch.zeros(mx, dtype=rows.dtype, device=rows.device)
    pad[:rows.numel()] = rows
    parts = [torch.empty_like(pad) for _ in range(world)]
    _all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, cs)])


def clock_ticks(ts: torch.Tensor, lo: int, world: int, group=None) -> torch.Tensor:
    """Multi-GPU playback (@app:playback partitioned apps, config 5): the clock is global (every event advances it,
    StreamJunction.sendData :232-237) but a rank receives only its keys' events. Each rank finds the clock-advance
    points of its own contiguous ingest slice (the first event of each new event time: global ordinal lo + i), and
    one all-gather (counts, then the padded points) gives every rank all of them, in global ordinal order (the
    slices are contiguous and ranked). Returns an int64 (m, 2) tensor of (global ordinal, clock)."""
    first = torch.ones_like(ts, dtype=torch.bool)
    if ts.numel() > 1:
        first[1:] = ts[1:] > ts[:-1]
    pos = torch.nonzero(first).flatten()
    mine = torch.stack([pos + lo, ts[pos]], 1)
    if world == 1:
        return mine
    cnt = torch.tensor([mine.shape[0]], dtype=torch.int64, device=ts.device)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    _all_gather(cnts, cnt, group=group)
    cs = [int(c.item()) for c in cnts]
    pad = torch.zeros((max(cs), 2), dtype=torch.int64, device=ts.device)
    pad[:mine.shape[0]] = mine
    parts = [torch.empty_like(pad) for _ in range(world)]
    _all_gather(parts, pad, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, cs)])


def merge_heartbeats(sid: torch.Tensor, ts: torch.Tensor, columns, ords: torch.Tensor, ticks: torch.Tensor):
    """A rank's received events (global ordinals `ords` ascending) merged with the global clock-advance points
    (`ticks` from clock_ticks) in ordinal order, as heartbeats (stream index -1, zero attributes, ordinal = that of the
    event that advanced the clock there: the trigger of the timers the heartbeat fires) for
    sm_app_process_device_events; a point at an ordinal this rank holds is dropped (that event advances the clock
    itself). GPU tensors: the HIP merge of the native library (sm_merge_heartbeats: binary-search merge path, no
    sort); host tensors (gloo tests): the same merge with torch.searchsorted. Returns (sid, ts, columns, ords)."""
    tord = ticks[:, 0].contiguous()
    tts = ticks[:, 1].contiguous()
    n, m = ords.numel(), tord.numel()
    for c in columns:
        if c.element_size() not in (4, 8) or c.numel() != n:
            raise ValueError("merge_heartbeats: columns of 4- or 8-byte elements aligned with the events")
    if ords.is_cuda:
        import ctypes
        from siddhi_amd import _lib
        cap = n + m
        o_sid = torch.empty(cap, dtype=torch.int32, device=ords.device)
        o_ts = torch.empty(cap, dtype=torch.int64, device=ords.device)
        o_ord = torch.empty(cap, dtype=torch.int64, device=ords.device)
        cols = [c.contiguous() for c in columns]
        outs = [torch.empty(cap, dtype=c.dtype, device=c.device) for c in cols]
        k = len(cols)
        widths = (ctypes.c_int32 * max(k, 1))(*[c.element_size() for c in cols])
        src = (ctypes.c_void_p * max(k, 1))(*[c.data_ptr() for c in cols])
        dst = (ctypes.c_void_p * max(k, 1))(*[o.data_ptr() for o in outs])
        n_out = ctypes.c_size_t()
        stream = ctypes.c_void_p(torch.cuda.current_stream(ords.device).cuda_stream)
        rc = _lib.lib().sm_merge_heartbeats(n, ords.data_ptr(), sid.contiguous().data_ptr(), ts.contiguous().data_ptr(),
                                            k, widths, src, m, tord.data_ptr(), tts.data_ptr(), o_sid.data_ptr(),
                                            o_ts.data_ptr(), o_ord.data_ptr(), dst, ctypes.byref(n_out), stream)
        if rc != _lib.SM_OK:
            raise RuntimeError(_lib.lib().sm_last_error().decode(errors="replace"))
        L = n_out.value
        return o_sid[:L], o_ts[:L], [o[:L] for o in outs], o_ord[:L]
    lb = torch.searchsorted(ords, tord)
    held = (lb < n) & (ords[lb.clamp(max=max(n - 1, 0))] == tord) if n else torch.zeros(m, dtype=torch.bool)
    keep = ~held
    kt, kts, klb = tord[keep], tts[keep], lb[keep]
    K = kt.numel()
    tick_at = torch.arange(K, dtype=torch.int64) + klb
    ev_at = torch.arange(n, dtype=torch.int64) + torch.searchsorted(kt, ords)
    L = n + K
    o_sid = torch.full((L,), -1, dtype=torch.int32)
    o_ts = torch.empty(L, dtype=torch.int64)
    o_ord = torch.full((L,), -1, dtype=torch.int64)
    o_sid[ev_at] = sid.to(torch.int32)
    o_ts[ev_at] = ts
    o_ts[tick_at] = kts
    o_ord[ev_at] = ords
    o_ord[tick_at] = kt  # a heartbeat carries the ordinal of the event that advanced the clock (its timers' trigger)
    outs = []
    for c in columns:
        o = torch.zeros(L, dtype=c.dtype)
        o[ev_at] = c
        outs.append(o)
    return o_sid, o_ts, outs, o_ord


def route_outputs(recs: torch.Tensor, starts, n_total: int, world: int, group=None) -> torch.Tensor:
    """Multi-GPU config 5: send every output record (int64 rows of the sm_app_copy_device_outputs
    layout, column 0 = the trigger's global ordinal, this rank's records in delivery order, so ascending in column 0)
    to the rank whose ingest slice holds its trigger (one all-to-all-v; split points by binary search). Returns the
    received rows: one run per source rank, in rank order."""
    if world == 1:
        return recs
    W = recs.shape[1]
    trig = recs[:, 0].contiguous()
    bnd = torch.searchsorted(trig, torch.tensor(starts[1:], dtype=torch.int64, device=recs.device))
    cuts = [0] + bnd.tolist() + [recs.shape[0]]
    sc = [(cuts[r + 1] - cuts[r]) * W for r in range(world)]
    rc = _all_to_all_counts(sc, recs.device, group)
    buf = torch.empty(sum(rc), dtype=torch.int64, device=recs.device)
    _all_to_all_single(buf, recs.contiguous().view(-1), rc, sc, group=group)
    return buf.view(-1, W)


def order_outputs(recs: torch.Tensor) -> torch.Tensor:
    """Runs of output records, each in delivery order, into the reference's delivery order for their triggers: one
    JVM calls its callbacks per trigger event in arrival order, the clock advance's timers first, those in scheduler
    listener registration order = partition instance creation order (EventTimeBasedMillisTimestampGenerator
    .setCurrentTimestamp core/util/timestamp/EventTimeBasedMillisTimestampGenerator.java:99-116; instances created in
    PartitionRuntime.cloneIfNotExist core/partition/PartitionRuntime.java:256-309). Stable sorts by the instance
    creation ordinal (column 2), the clock step (column 1), then (trigger ordinal, phase) (column 0, low half of
    column 4): records equal in all of them come from one instance and keep their run order. GPU: sm_order_outputs
    (radix passes); host tensors: the same passes with torch's stable sort."""
    if recs.shape[0] <= 1:
        return recs
    if recs.is_cuda:
        import ctypes
        from siddhi_amd import _lib
        out = torch.empty_like(recs)
        stream = ctypes.c_void_p(torch.cuda.current_stream(recs.device).cuda_stream)
        rc = _lib.lib().sm_order_outputs(recs.data_ptr(), recs.shape[0], recs.shape[1] * 8, out.data_ptr(), stream)
        if rc != _lib.SM_OK:
            raise RuntimeError(_lib.lib().sm_last_error().decode(errors="replace"))
        return out
    idx = torch.arange(recs.shape[0])
    phase = recs[:, 4] & 0xFFFFFFFF
    for key in (recs[:, 2] + 1, recs[:, 1], recs[:, 0] * 2 + phase):  # least significant first
        idx = idx[torch.sort(key[idx], stable=True).indices]
    return recs[idx]


def merge_outputs(recs: torch.Tensor, starts, n_total: int, world: int, group=None) -> torch.Tensor:
    """route_outputs + order_outputs: this rank's slice of the single-process output sequence (the ranks' results
    concatenated in rank order are the one-JVM delivery order)."""
    return order_outputs(route_outputs(recs, starts, n_total, world, group))


def merge_matches(parts):
    """Merge per-rank match tuples (each an (n, 2) int array of global (e1, e2) ordinals in reference order for
    that rank's keys) into the reference's global order: by e2 ordinal; ties (same e2) come from one rank and
    keep that rank's order. Host-side (numpy) helper for tests."""
    import numpy as np
    parts = [np.asarray(p, dtype=np.int64).reshape(-1, 2) for p in parts]
    if not parts:
        return np.zeros((0, 2), dtype=np.int64)
    allp = np.concatenate(parts)
    order = np.argsort(allp[:, 1], kind="stable")
    return allp[order]
