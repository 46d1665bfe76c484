"""K_slab restatement (siddhi_amd/csrc/slab.h) on the host against the CPU oracle: the per-partial
entries, list positions and emission order of the device kernel's lanes reproduce the reference's
object graph for distinct-stream patterns (random apps: stream / count / logical elements, cross-
references into earlier slots, count chains read at [0] / [last], within, every / non-every, nulls).
CPU only; the GPU kernel is checked in test_gpu_slab.py."""
import pytest

from fuzz_apps import random_slab_app, random_slab_events
from harness import App
from slab_host import SlabHostEngine


def _run(src, events, batch):
    o, h = App(src), App(src, SlabHostEngine)
    run = []
    for ev in events + [(None, None, None)]:
        if run and (ev[0] != run[0][0] or len(run) >= batch):
            for app in (o, h):
                app.send(run[0][0], [r for _, r, _ in run], [t for _, _, t in run])
            run = []
        if ev[0] is not None:
            run.append(ev)
    return o, h


@pytest.mark.parametrize("seed", range(120))
def test_slab_host_equals_oracle(seed):
    src = random_slab_app(seed)
    o, h = _run(src, random_slab_events(seed, n=500, keys=3 + seed % 4), batch=1 + seed % 7)
    assert h.matches == o.matches


def test_slab_host_c5_family():
    from siddhi_amd.workloads import c5_app
    import c5_family
    o = c5_family.run_c5(64, 200, 4000, 1000)
    h = c5_family.run_c5(64, 200, 4000, 1000, engine_factory=SlabHostEngine)
    assert h.matches == o.matches and len(o.matches) > 100
