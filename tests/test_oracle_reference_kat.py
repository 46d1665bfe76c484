"""Pin the CPU oracle to the reference's own known-answer tests.

tests/golden/reference_kat.json is transcribed from the reference's TestNG suites by
tests/golden/extract_reference_tests.py (queries, events with cumulative-sleep timestamps,
hand-asserted expected rows and counts). Fixtures that use features outside the accelerated path
(having, plain queries) must be rejected at plan time rather than mis-executed.""" 
import json
import os

import pytest

from harness import App, parse_literal, values_equal
from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_kat.json")))
OUT_OF_SCOPE = {
    "CountPatternTestCase.testQuery14": "having",
    "IsNullTestCase.isNullTest1": "plain stream query (runs as a one-state pattern in test_filter_kat.py)",
}


def run_fixture(fx, engine_factory=None):
    app = App(fx["app"], engine_factory)
    for ev in fx["events"]:
        app.send(ev["stream"], [[parse_literal(t) for t in ev["data"]]], [ev["ts"]])
    if fx["callback_kind"] == "QueryCallback":
        return app, app.rows_for_query(fx["callback"])
    return app, app.rows_for_stream(fx["callback"])


def check_rows(fx, rows):
    if fx["expected_count"] is not None:
        assert len(rows) == fx["expected_count"], f"{len(rows)} matches, reference expects {fx['expected_count']}"
    if fx["event_arrived"] is False:
        assert not rows
    for r in fx["expected_rows"]:
        if r["case"] is None:
            targets = rows
        else:
            assert r["case"] <= len(rows), f"missing match #{r['case']}"
            targets = [rows[r["case"] - 1]]
        for row in targets:
            assert len(row) == len(r["row"]) and all(values_equal(e, a) for e, a in zip(r["row"], row)), \
                f"row {row} != expected {r['row']} (case {r['case']})"


@pytest.mark.parametrize("fx", KAT["fixtures"], ids=[f["id"] for f in KAT["fixtures"]])
def test_reference_kat(fx):
    if fx["id"] in OUT_OF_SCOPE:
        with pytest.raises((SiddhiParserException, SiddhiAppCreationException)):
            run_fixture(fx)
        return
    _, rows = run_fixture(fx)
    check_rows(fx, rows)


def test_kat_coverage():
    # every in-scope reference suite contributes fixtures
    suites = {f["id"].split(".")[0] for f in KAT["fixtures"]}
    assert suites == {"EveryPatternTestCase", "WithinPatternTestCase", "CountPatternTestCase",
                      "LogicalPatternTestCase", "ComplexPatternTestCase", "SequenceTestCase",
                      "PatternPartitionTestCase", "SequencePartitionTestCase", "IsNullTestCase"}
    assert len(KAT["fixtures"]) >= 130
