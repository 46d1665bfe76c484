"""K_slab on the GPU (nfa_slab.hip: distinct-stream patterns on sparse per-partial entries, the C5
family's plan) against the CPU oracle: random apps of the class (stream / count / logical elements,
cross-references, within, every / non-every, nulls), pushed per event run and in large batches; the
same with the LDS staging area and the slab so small that pushes fail and are rolled back, slabs
grow and sub-rings are reclaimed; the C5 family; snapshot / restore."""
import os

import numpy as np
import pytest

from fuzz_apps import random_slab_app, random_slab_events
from harness import App
from siddhi_amd.ir import T_FLOAT, T_INT, T_STRING

pytestmark = pytest.mark.gpu

SLAB_TYPES = [[T_INT, T_FLOAT, T_INT, T_STRING]] * 6


class Tracked:
    """HipEngine factory that records whether K_slab ran (stats.last_slab_items after each push)."""

    def __init__(self, types, **kw):
        self.types, self.kw, self.slab_items, self.engines = types, kw, 0, []

    def __call__(self, blob):
        from siddhi_amd.engine import HipEngine
        eng = HipEngine(blob, stream_types=self.types, **self.kw)
        orig = eng.send

        def send(*a, **k):
            orig(*a, **k)
            self.slab_items += eng.stats().last_slab_items
        eng.send = send
        self.engines.append(eng)
        return eng


def _run(src, events, batch, factory=None):
    app = App(src, factory)
    run = []
    for ev in events + [(None, None, None)]:
        if run and (ev[0] != run[0][0] or len(run) >= batch):
            app.send(run[0][0], [r for _, r, _ in run], [t for _, _, t in run])
            run = []
        if ev[0] is not None:
            run.append(ev)
    return app


@pytest.mark.parametrize("seed", range(40))
@pytest.mark.parametrize("batch", [3, 10 ** 6])
def test_slab_fuzz_equals_oracle(seed, batch):
    src = random_slab_app(seed)
    ev = random_slab_events(seed, n=500, keys=3 + seed % 4)
    o = _run(src, ev, batch)
    f = Tracked(SLAB_TYPES)
    g = _run(src, ev, batch, f)
    assert f.slab_items > 0
    assert g.matches == o.matches


@pytest.mark.parametrize("seed", range(12))
def test_slab_rollback_growth_and_reclaim(seed, monkeypatch):
    """A 64-word LDS staging area and 64-word sub-rings: pushes overflow both, are undone (journal)
    and re-run at doubled capacity; sub-rings fill with superseded blocks and are reclaimed."""
    monkeypatch.setenv("SIDDHI_HIP_DEBUG", "SDH_SLAB_LDS_WORDS=64;SDH_SLAB_SUB_WORDS=64")
    src = random_slab_app(seed + 100)
    ev = random_slab_events(seed + 100, n=800, keys=2)
    o = _run(src, ev, 50)
    g = _run(src, ev, 50, Tracked(SLAB_TYPES))
    assert g.matches == o.matches and len(o.matches) > 0


@pytest.mark.parametrize("batch", [2000, 333])
def test_c5_family_on_slab(batch):
    from c5_family import run_c5
    from siddhi_amd.engine import HipEngine
    from siddhi_amd.ir import T_FLOAT, T_INT
    o = run_c5(128, 2000, 8000, batch)
    engines = []

    def fac(blob):
        engines.append(HipEngine(blob, stream_types=[[T_INT, T_FLOAT, T_INT]] * 4))
        return engines[-1]
    g = run_c5(128, 2000, 8000, batch, engine_factory=fac)
    st = engines[0].stats()
    assert st.last_slab_items > 0 and st.last_gen_items == 0 and st.last_part_items == 0
    assert g.matches == o.matches and len(o.matches) > 1000
    assert st.live_partials > 0


def test_slab_snapshot_restore():
    """persist() mid-stream, then a new engine restores it and sees the rest of the stream: the
    matches equal the uninterrupted run's (PersistenceTestCase for the sparse state)."""
    from siddhi_amd.engine import HipEngine
    src = random_slab_app(7)
    ev = random_slab_events(7, n=900, keys=5)
    half = 450
    a = _run(src, ev[:half], 20, lambda b: HipEngine(b, stream_types=SLAB_TYPES))
    blob = a.engine.snapshot()
    n0 = len(a.matches)
    for stream, row, t in ev[half:]:
        a.send(stream, [row], [t])
    b = App(src, lambda bl: HipEngine(bl, stream_types=SLAB_TYPES))
    b.engine.restore(blob)
    b.dictionary = a.dictionary  # the same string ids as the run that was persisted
    for stream, row, t in ev[half:]:
        b.send(stream, [row], [t])
    assert b.matches == a.matches[n0:] and len(a.matches) > n0
