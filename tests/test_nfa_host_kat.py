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


@pytest.fixture(scope="module")
def harness():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
    from host_harness_lib import HostHarnessApp
    return HostHarnessApp


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_nfa_host_kat(harness, kat):
    r = run_kat(harness, kat)
    if r.startswith("unsupported"):
        pytest.skip(r)
    assert r in ("pass", "error-as-expected")
