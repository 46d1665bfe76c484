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
