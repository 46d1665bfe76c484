"""f4 (snapshot / restore of the device partial-match state) pinned by the reference's own
persistence test: PersistenceTestCase.persistenceTest2 (PersistenceTestCase.java:145-235) persists a
count pattern's pending state, restarts the app, restores the last revision and expects exactly one
match {25.6f, 47.6f, null, null, 45.7f}. Here: events -> sdh_engine_snapshot -> a NEW engine ->
sdh_engine_restore -> events, on every plan that can run the query (planned and K_gen), and the same
stream on the oracle without a restart gives the same matches."""
import json
import os

import pytest

from harness import App, parse_literal
from test_oracle_reference_kat import check_rows

pytestmark = pytest.mark.gpu

FX = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "reference_persistence_kat.json")))["fixtures"]
SDH_FLAG_FORCE_GEN = 4


def _gpu_app(src, flags):
    from siddhi_amd.engine import HipEngine
    app = App(src, engine_factory=lambda blob: None)
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], flags=flags)
    return app


def _send(app, evs):
    for ev in evs:
        app.send(ev["stream"], [[parse_literal(t) for t in ev["data"]]], [ev["ts"]])


@pytest.mark.parametrize("flags", [0, SDH_FLAG_FORCE_GEN], ids=["planned", "force_gen"])
@pytest.mark.parametrize("fx", FX, ids=[f["id"] for f in FX])
def test_persist_restore_kat(fx, flags):
    a = _gpu_app(fx["app"], flags)
    _send(a, fx["before_persist"])
    assert len(a.rows_for_query(fx["callback"])) == fx["count_before_persist"]
    snap = a.engine.snapshot()
    a.engine.close()
    b = _gpu_app(fx["app"], flags)  # the restarted runtime
    b.engine.restore(snap)
    b.log = a.log  # the host's event log (the events the restored partials refer to by sequence number)
    _send(b, fx["after_restore"])
    check_rows(fx, b.rows_for_query(fx["callback"]))
    o = App(fx["app"])  # the oracle over the whole stream without a restart
    _send(o, fx["before_persist"] + fx["after_restore"])
    assert b.matches == o.matches
