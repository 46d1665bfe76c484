"""GPU parity of a stream the partition does not key (PatternPartitionTestCase query 30's shape):
every event reaches every known key's clones in the order of the reference's ConcurrentHashMap of
"streamId + key" junctions (PartitionStreamReceiver.java:277-281; the engine's chm_order.h against
the oracle's own restatement). The device runs those queries as K_gen fan-out sweeps, and the match
table orders their matches by (partition rank, key's map position, query rank, emission)."""
import numpy as np
import pytest

from fuzz_apps import fanout_app, fanout_events
from harness import App

pytestmark = pytest.mark.gpu


def hip_app(src, **kw):
    app = App(src, engine_factory=lambda blob: None)
    from siddhi_amd.engine import HipEngine
    app.engine = HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], **kw)
    return app


def _send(apps, ev, batch):
    i = 0
    while i < len(ev):
        j = i + 1
        while batch and j < len(ev) and ev[j][0] == ev[i][0] and j - i < 64:
            j += 1
        for a in apps:
            a.send(ev[i][0], [r for _, r, _ in ev[i:j]], [t for _, _, t in ev[i:j]])
        i = j


@pytest.mark.parametrize("batch", [False, True], ids=["per_event", "batched"])
@pytest.mark.parametrize("key_type", ["int", "long", "bool", "string", "float", "double"])
@pytest.mark.parametrize("seed", range(6))
def test_fanout_on_gpu(seed, key_type, batch):
    src = fanout_app(seed, key_type)
    o, g = App(src), hip_app(src)
    _send([o, g], fanout_events(seed, keys=20 + 8 * seed, key_type=key_type), batch)
    assert len(o.matches) > 20
    assert g.matches == o.matches


def test_fanout_many_keys_and_snapshot():
    """150 keys (the junction map resizes to 256 bins), pushed in batches; a snapshot taken midway
    restores the key creation order into a fresh engine that continues identically."""
    src = fanout_app(3)
    ev = fanout_events(11, n=2000, keys=150)
    o, g = App(src), hip_app(src)
    _send([o, g], ev[:1000], True)
    snap = g.engine.snapshot()
    g2 = hip_app(src)
    g2.engine.restore(snap)
    o.matches.clear()
    g.matches.clear()
    _send([o, g, g2], ev[1000:], True)
    assert len(o.matches) > 100
    assert g.matches == o.matches
    assert g2.matches == o.matches


def test_fanout_refused_with_key_shards():
    from siddhi_amd.engine import EngineError, HipEngine
    app = App(fanout_app(0), engine_factory=lambda blob: None)
    with pytest.raises(EngineError):
        HipEngine(app.blob, stream_types=[s.attr_types for s in app.ir.streams], shard_rank=0, shard_world=2)


def test_unregistered_string_key_fails_the_push_cleanly():
    """A fan-out push that reaches a string key whose text hash was never registered
    (sdh_engine_set_strings; e.g. after a restore) fails with SDH_E_INVALID before any kernel runs:
    the engine stays usable, and once the strings are registered the same push goes through and the
    run equals the oracle."""
    from siddhi_amd.engine import EngineError
    from siddhi_amd.events import encode_rows
    src = fanout_app(3, "string")
    ev = fanout_events(5, n=800, keys=30, key_type="string")
    o, g = App(src), hip_app(src)
    _send([o], ev, True)
    n_slots = lambda q: len(g.ir.queries[q].states)  # noqa: E731
    got, refused = [], 0
    i = 0
    while i < len(ev):
        j = i + 1
        while j < len(ev) and ev[j][0] == ev[i][0] and j - i < 64:
            j += 1
        si = g.ir.stream_index(ev[i][0])
        vals, nulls = encode_rows([r for _, r, _ in ev[i:j]], g.ir.streams[si].attr_types, g.dictionary)
        ts = [t for _, _, t in ev[i:j]]
        try:
            g.engine.send(si, ts, vals, nulls)
        except EngineError as ex:
            assert ex.code == -1 and "sdh_engine_set_strings" in str(ex)
            refused += 1
            ids = list(range(len(g.dictionary)))
            g.engine.set_strings(ids, [g.dictionary.lookup(k) for k in ids])
            g.engine.send(si, ts, vals, nulls)
        got.extend(g.engine.take_matches(n_slots))
        i = j
    assert refused >= 1  # (each new string key refuses one push until it is registered)
    assert len(o.matches) > 20
    assert got == o.matches
