"""Every transcribed reference KAT (tests/golden/kats.json) through the device NFA code compiled for the host
(tests/native/nfa_host_harness.cpp over siddhi_amd/csrc/kernels/nfa_impl.h, the same source the GPU kernel and the
query-specialised JIT kernel are built from). A CPU check of the NFA interpreter's semantics that runs without a
GPU; the GPU product runs the same KATs in tests/test_product_kat.py. Test infrastructure."""
import os
import subprocess

import pytest

from kat_runner import load_kats, run_kat

HERE = os.path.dirname(os.path.abspath(__file__))
KATS = [k for k in load_kats() if "skip" not in k]


@pytest.fixture(scope="module", params=[0, 2], ids=["lists", "pending_arrays2"])
def harness(request):
    """pending_arrays2: the build with the query-specialised kernel's LDS pending arrays (nfa_impl.h SM_NFA_PA) of 2
    entries, so that most partials of a longer list go through the HBM part, the refills and the relink"""
    pa = request.param
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")] + ([f"pa={pa}"] if pa else []))
    from host_harness_lib import HostHarnessApp

    class H(HostHarnessApp):
        pass

    H.pa = pa
    return H


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_nfa_host_kat(harness, kat):
    r = run_kat(harness, kat)
    if r.startswith("unsupported"):
        pytest.skip(r)
    assert r in ("pass", "error-as-expected")
