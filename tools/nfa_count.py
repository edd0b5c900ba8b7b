"""Per-event work of the config-5 NFA on a key subsample, from the SM_COUNT_ACCESS build of the host NFA harness
(tests/native, `make count=1`): key-state and heap word accesses, words allocated, words copied by collections,
collections, run records and chain nodes allocated. Diagnostic (CPU only, no GPU): the split of the NFA kernel's
HBM traffic into allocation, collection copy and state that DESIGN.md §4 cites.

Usage: python tools/nfa_count.py [N=1e8] [heap_half=4096] [variant]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import synth  # noqa: E402

N = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
half = sys.argv[2] if len(sys.argv) > 2 else "4096"
variant = sys.argv[3] if len(sys.argv) > 3 else None
os.environ["SM_HOST_HEAP_HALF"] = half
L = ctypes.CDLL(os.path.join(ROOT, "tests", "native", "build", "libnfa_host_count.so"))
import host_harness_lib as hh  # noqa: E402

L.h_create.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_char_p, ctypes.c_size_t]
L.h_send.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(hh.HV)]
L.h_advance.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
L.h_flush.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t]
L.h_start.argtypes = [ctypes.c_void_p]
K, div = 1_000_000, 100
body = synth.QUERY5 if variant is None else dict(synth.VARIANTS5)[variant] if hasattr(synth, "VARIANTS5") else variant
text = synth.app5(body)
h = ctypes.c_void_p()
err = ctypes.create_string_buffer(1024)
assert L.h_create(text.encode(), ctypes.byref(h), err, 1024) == 0, err.value
L.h_start(h)
row = (hh.HV * 4)()
for k, t in enumerate((0, 3, 1, 1)):
    row[k].type = t
sel = lambda sym: sym % 1009 == 5  # noqa: E731
n_ev = n_hb = 0
last_ts = -1
for lo in range(0, N, 10_000_000):
    sid, cols, ts = synth.gen5(lo, min(N, lo + 10_000_000), K, div)
    mine = sel(cols[0])
    adv = np.ones(len(ts), bool)
    adv[1:] = ts[1:] > ts[:-1]
    adv[0] = ts[0] > last_ts
    last_ts = int(ts[-1])
    for i in np.nonzero(mine | adv)[0]:
        if mine[i]:
            row[0].i = int(cols[0][i])
            row[1].d = float(cols[1][i])
            row[2].i = int(cols[2][i])
            row[3].i = int(cols[3][i])
            L.h_send(h, "ABCDE"[sid[i]].encode(), int(ts[i]), row)
            n_ev += 1
        else:
            L.h_advance(h, int(ts[i]), 0)
            n_hb += 1
assert L.h_flush(h, err, 1024) == 0, err.value
c = (ctypes.c_int64 * 8)()
L.h_access(c)
names = ["key-state word accesses", "heap word accesses", "words allocated", "words copied by collections",
         "collections", "events delivered", "run records allocated", "chain nodes allocated"]
print(f"N = {N:.0e}, key subsample sym % 1009 == 5: {n_ev} events, {n_hb} heartbeats, heap_half {half}")
for k, name in enumerate(names):
    print(f"  {name:30s} {c[k]:12d}   {c[k] / max(n_ev, 1):8.2f} per event")
ph = (ctypes.c_int64 * 32)()
L.h_access_phases(ph)
pn = {0: "other", 12: "emit (selector)", 13: "timers (fire_all)", 14: "updateState", 15: "safe point / gc"}
print("  per phase (key-state / heap word accesses per event):")
for k in range(16):
    if ph[k] or ph[16 + k]:
        name = pn.get(k, f"processAndReturn pre {k - 1}")
        print(f"    {name:32s} {ph[k] / max(n_ev, 1):8.2f} {ph[16 + k] / max(n_ev, 1):8.2f}")
