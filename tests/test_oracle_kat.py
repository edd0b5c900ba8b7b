"""The CPU oracle against the reference's own known-answer tests (tests/golden/kats.json,
transcribed from the TestNG suites by tests/golden/make_kats.py). This pins the oracle."""
import pytest

from kat_runner import load_kats, run_kat
from oracle_lib import OracleApp

KATS = [k for k in load_kats() if "skip" not in k]


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_kat(kat):
    r = run_kat(OracleApp, kat)
    if r.startswith("unsupported"):
        pytest.skip(r)
    assert r in ("pass", "error-as-expected")


def test_kat_coverage():
    # every hot-path suite contributes pinned vectors
    suites = {k["name"].split(".")[0] for k in KATS}
    for s in ["EveryPatternTestCase", "WithinPatternTestCase", "CountPatternTestCase", "LogicalPatternTestCase",
              "SequenceTestCase", "PatternPartitionTestCase", "SequencePartitionTestCase", "FilterTestCase1",
              "AbsentPatternTestCase", "EveryAbsentPatternTestCase", "LogicalAbsentSequenceTestCase"]:
        assert s in suites
    assert len(KATS) >= 450
