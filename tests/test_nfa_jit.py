"""The query-specialised NFA kernel (siddhi_amd/csrc/nfa_jit.cpp): the NFA interpreter compiled per query plan with
hiprtc for gfx950. CPU: the JIT source compiles for representative plans (no device needed). GPU parity of the
specialised kernel against the oracle is in tests/test_device_events.py (nfa_jit forced on)."""
import ctypes
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from siddhi_amd import _lib  # noqa: E402


def _jit(app, query=0):
    L = _lib.lib()
    log = ctypes.create_string_buffer(8192)
    size = ctypes.c_size_t()
    rc = L.sm_nfa_jit_compile(app.encode(), query, log, 8192, ctypes.byref(size))
    return rc, size.value, log.value.decode(errors="replace")


@pytest.mark.parametrize("app", [bench.APP5, bench.APP], ids=["config5_sequence", "config4_pattern"])
def test_jit_kernel_compiles(app):
    rc, size, log = _jit(app)
    assert rc == 0, log
    assert size > 10000


def test_jit_reports_missing_query():
    rc, size, log = _jit(bench.APP5, query=7)
    assert rc != 0 and "no such query" in log
