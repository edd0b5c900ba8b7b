"""Parser known-answer tests, independent of the shared parser: SiddhiQL texts from the
reference's own query-tree tests must parse into the trees the reference's builders construct
(tests/golden/ast_kats.json, transcribed by tests/golden/make_ast_kats.py from siddhi-query-api
PatternQueryTestCase / SequenceQueryTestCase and siddhi-query-compiler AbsentPatternTestCase), or fail with
SiddhiParserException where the reference's compiler does. The compiler's SimpleQueryTestCase (filter queries) and
DefinePartitionTestCase pin the filter-expression trees (FilterProcessor) and the value
partition type; the parts of those texts outside the hot-path subset (windows, aggregations, group by, update,
range partitions) must be refused with OperationNotSupportedException, never mis-parsed. The oracle and the product share the parser, so these
are the checks a parse/binding bug (e.g. `within` attached to the wrong element) cannot pass on both sides.
CPU only: sm_compile_dump parses without a device."""
import json
import os

import pytest

import siddhi_amd

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ast_kats.json")
KATS = json.load(open(GOLDEN))
DEFS = " ".join(f"define stream Stream{k} (symbol string, price float, volume int);" for k in range(1, 5)) + " "
SIMPLE_DEFS = " ".join(f"define stream {s} (symbol string, price float, volume int);"
                       for s in ("StockStream", "AllStockQuotes", "cseEventStream")) + " "


def norm(s):
    """State tree with `->` chains flattened (builders nest them to the right, the grammar to the left; the
    processor chain is the same) unless the nesting carries a `within`."""
    if "next" in s:
        items = []
        for c in s["next"]:
            c = norm(c)
            if "chain" in c and "within" not in c:
                items.extend(c["chain"])
            else:
                items.append(c)
        out = {"chain": items}
    elif "every" in s:
        out = {"every": norm(s["every"])}
    elif "count" in s:
        out = {"count": norm(s["count"]), "min": s["min"], "max": s["max"]}
    elif "and" in s or "or" in s:
        k = "and" if "and" in s else "or"
        out = {k: [norm(c) for c in s[k]]}
    elif "not" in s:
        out = {"not": s["not"]}
        if "for" in s:
            out["for"] = s["for"]
    else:
        out = {"stream": s["stream"], "filters": s["filters"]}
        if s.get("ref"):
            out["ref"] = s["ref"]
    if "within" in s:
        out["within"] = s["within"]
    return out


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_parse_kat(kat):
    if "skip" in kat:
        pytest.skip(kat["skip"])
    if kat["name"].startswith(("compiler.SimpleQueryTestCase", "compiler.DefinePartitionTestCase")):
        return check_filter_or_partition_kat(kat)
    text = DEFS + kat["text"] + " select * insert into OutputStream;"
    if kat.get("expect") == "parse_error":
        with pytest.raises(siddhi_amd.SiddhiParserException):
            siddhi_amd.compile_dump(text)
        return
    q = siddhi_amd.compile_dump(text)["queries"][0]
    assert q["input"] == kat["input"]
    assert norm(q["state"]) == norm(kat["tree"])


def test_within_binds_to_the_element_it_follows():
    """in `every e1 -> e2 within 1 sec` the `within` binds to e2's stream element; on a
    parenthesised chain it binds to the chain (SiddhiQLBaseVisitorImpl.java:815-821, 855-860, 782-788)."""
    q = siddhi_amd.compile_dump(DEFS + "from every e1=Stream1 -> e2=Stream2 within 1 sec select * insert into O;")
    st = q["queries"][0]["state"]
    assert st["next"][1] == {"stream": "Stream2", "ref": "e2", "filters": [], "within": 1000}
    assert "within" not in st
    q = siddhi_amd.compile_dump(DEFS + "from (every e1=Stream1 -> e2=Stream2) within 1 sec select * insert into O;")
    st = q["queries"][0]["state"]
    assert st["within"] == 1000 and "within" not in st["next"][1]


def check_filter_or_partition_kat(kat):
    partition = "DefinePartitionTestCase" in kat["name"]
    if partition:  # the reference compares the partition type only (toString() up to "queryList")
        text = SIMPLE_DEFS + kat["text"] + " begin from cseEventStream select symbol insert into PartOut; end;"
    elif kat.get("expect") == "unsupported":
        text = SIMPLE_DEFS + kat["text"]
    else:
        text = SIMPLE_DEFS + kat["text"] + " select symbol insert into OutStockStream;"
    if kat.get("expect") == "unsupported":
        with pytest.raises(siddhi_amd.OperationNotSupportedException):
            siddhi_amd.compile_dump(text)
        return
    d = siddhi_amd.compile_dump(text)
    if partition:
        assert [p["with"] for p in d["partitions"]] == [kat["with"]]
        return
    q = d["queries"][0]
    assert (q["input"], q["stream"], q["filters"]) == (kat["input"], kat["stream"], kat["filters"])
