"""Pin the CPU oracle's absent-pattern semantics (`not S for T`) to the reference's
own known-answer tests.

tests/golden/reference_absent_kat.json is transcribed from the reference's eight absent suites by
tests/golden/extract_absent_tests.py: each fixture is the app, the timeline after
siddhiAppRuntime.start() (events at their send times, the ends of the test's sleeps, and the
asserted in-event counts at each check), and the callback's ordered expected rows. The runtime
starts at ts0 (playback apps: at 0, TimestampGeneratorImpl's initial time); time passes with the
sleeps (a live runtime's schedulers fire meanwhile) or, in playback, with the events alone.

Logical absent states (`e1=A and not B`, `not A for T or e2=B`: AbsentLogicalPre/PostStateProcessor)
and absent states inside a partition (per-key clones with their own schedulers, never start()ed)
are in scope. Playback apps with a heartbeat (`@app:playback(idle.time=.., increment=..)`: event
time advancing with the wall clock while idle) run as plain playback: their timelines assert right
after the last send, so no heartbeat can fire (the wall clock never idles for `idle.time`)."""
import json
import os

import pytest

from harness import App, parse_literal, values_equal
from siddhi_amd.ql import SiddhiAppCreationException, SiddhiParserException

ABSENT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_absent_kat.json")))
FIXTURES = ABSENT["fixtures"]


def out_of_scope(fx) -> str:
    """Why a fixture is outside the accelerated path ('' if it is in scope)."""
    try:
        App(fx["app"])
    except SiddhiParserException as ex:
        if "logical absent" in str(ex):
            return "logical absent"
        raise
    except SiddhiAppCreationException as ex:
        if "inside a partition" in str(ex):
            return "partitioned absent"
        raise
    return ""


def rows_of(app, fx):
    if fx["callback_kind"] == "query":
        return app.rows_for_query(fx["callback"])
    return app.rows_for_stream(fx["callback"])


def run_absent_fixture(fx, engine_factory=None, start=True):
    """Run one fixture's timeline; returns (app, rows, [(asserted count, rows at that point)])."""
    app = App(fx["app"], engine_factory)
    if start:
        app.start(0 if fx["playback"] else ABSENT["ts0"])
    checks = []
    for a in fx["actions"]:
        if "send" in a:
            app.send(a["send"], [[parse_literal(t) for t in a["data"]]], [a["ts"]])
        elif "advance" in a:
            app.advance_time(a["advance"])
        else:
            checks.append((a["check"], len(rows_of(app, fx))))
    return app, rows_of(app, fx), checks


def check_absent_rows(fx, rows, checks):
    for want, got in checks:
        assert got == want, f"{got} matches at a check, reference expects {want}"
    if fx["event_arrived"] is False:
        assert not rows
    if fx["event_arrived"] is True:
        assert rows
    # TestQueryCallback compares each arriving in-event with the expected row of its position (missing
    # ones show in the asserted counts)
    for k, exp in enumerate(fx["expected_rows"][:len(rows)]):
        row = rows[k]
        assert len(row) == len(exp) and all(values_equal(e, a) for e, a in zip(exp, row)), \
            f"row {row} != expected {exp} (#{k + 1})"


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["id"] for f in FIXTURES])
def test_absent_kat_on_oracle(fx):
    why = out_of_scope(fx)
    if why:
        with pytest.raises((SiddhiParserException, SiddhiAppCreationException)):
            App(fx["app"])
        return
    _, rows, checks = run_absent_fixture(fx)
    check_absent_rows(fx, rows, checks)


def test_absent_kat_coverage():
    suites = {f["id"].split(".")[0] for f in FIXTURES}
    assert len(suites) == 8 and len(FIXTURES) >= 300
    in_scope = [f for f in FIXTURES if not out_of_scope(f)]
    assert len(in_scope) == len(FIXTURES) == 303
