"""GPU parity on the reference's KATs: the HIP engine (through the C ABI) must (1) satisfy every transcribed
reference expectation and (2) produce exactly the oracle's outputs — values, timestamps, order and the
event-ordinal tuples of every match."""
import pytest

from kat_runner import drive_only, load_kats, run_kat
from oracle_lib import OracleApp

pytestmark = pytest.mark.gpu

KATS = [k for k in load_kats() if "skip" not in k]


def _product():
    from siddhi_amd.testing import ProductApp
    return ProductApp


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_product_kat(kat):
    r = run_kat(_product(), kat)
    if r.startswith("unsupported"):
        pytest.skip(r)
    assert r in ("pass", "error-as-expected")


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_product_equals_oracle(kat):
    want = drive_only(OracleApp, kat)
    got = drive_only(_product(), kat)
    if isinstance(want, tuple):
        assert isinstance(got, tuple) and got[0] == want[0], (want, got)
        return
    assert got == want
