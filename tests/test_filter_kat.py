"""Typed predicate semantics pinned by the reference's own filter tests
(FilterTestCase1/2, IsNullTestCase; transcribed by tests/golden/extract_filter_tests.py).

Each filter query ``from S[cond]`` runs as the one-state pattern ``from every e1=S[cond]``: the same
events pass. The oracle must emit exactly the number of events the reference test asserts
(``assertEquals(N, count.get())``) or waits for (``waitForEvents(.., N, count, ..)``), and must reject
the apps the reference rejects at creation. The GPU engine (``-m gpu``) must emit the oracle's match
tuples -- which name the passing events by sequence number -- on every fixture, on the planned path
and forced onto K_gen."""
import json
import os

import pytest

from harness import App, parse_literal
from siddhi_amd.ql import SiddhiAppCreationException

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "reference_filter_kat.json")))
FIXTURES = KAT["fixtures"]
RUNNABLE = [f for f in FIXTURES if not f.get("expect_creation_error")]
TS0 = 1_500_000_000_000


def pattern_app(fx):
    import re
    attrs = [a.split()[0] for a in fx["define"].split("(", 1)[1].rsplit(")", 1)[0].split(",")]
    cond = fx["condition"]
    # inside a pattern a bare name before `is null` resolves as a stream reference (the
    # reference's null_check grammar), so an attribute there is qualified with the state alias
    cond = re.sub(r"\b(" + "|".join(attrs) + r")\s+is\s+null", r"e1.\1 is null", cond)
    return (f"{fx['define']} @info(name = 'query1') from every e1={fx['stream']}[{cond}] "
            f"select e1.{attrs[0]} as a insert into OutputStream;")


def run(fx, engine_factory=None):
    app = App(pattern_app(fx), engine_factory)
    for i, ev in enumerate(fx["events"]):
        app.send(fx["stream"], [[parse_literal(t) for t in ev]], [TS0 + i])
    return app


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_filter_kat_oracle(fx):
    if fx.get("expect_creation_error"):
        with pytest.raises(SiddhiAppCreationException):
            App(pattern_app(fx))
        return
    app = run(fx)
    assert len(app.matches) == fx["expected_count"], \
        f"{len(app.matches)} events pass `{fx['condition']}`, the reference test expects {fx['expected_count']}"


def test_filter_kat_coverage():
    suites = {f["id"].split(".")[0] for f in FIXTURES}
    assert suites == {"FilterTestCase1", "FilterTestCase2", "IsNullTestCase"}
    assert len(RUNNABLE) >= 90


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, 4], ids=["planned", "force_gen"])
@pytest.mark.parametrize("fx", RUNNABLE, ids=[f["id"] for f in RUNNABLE])
def test_filter_kat_gpu(fx, flags):
    o = run(fx)
    probe = App(pattern_app(fx), engine_factory=lambda blob: None)
    types = [s.attr_types for s in probe.ir.streams]

    def make(blob):
        from siddhi_amd.engine import HipEngine
        return HipEngine(blob, stream_types=types, flags=flags)
    g = run(fx, engine_factory=make)
    assert g.matches == o.matches
    assert len(g.matches) == fx["expected_count"]
