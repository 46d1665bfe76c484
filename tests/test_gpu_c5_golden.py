"""GPU parity of C5 at its configured size (BASELINE.json configs[4]): 100,000 mixed patterns over four
joined streams in one `partition with (acct of ...)`, `within 1 hour`, on K_slab's sparse per-partial
state, against the oracle goldens of tests/golden/make_c5_golden.py:

  c5      the streams' first 24,576 events each over the whole 1,000,000-account key space (~93K
          accounts seen, most once or twice): the key-table / sparse-state scale case;
  c5deep  the same streams restricted to accounts with acct % 512 == 0 (1,954 accounts) over their
          first 16M events each, so every account sees dozens of events per stream across hours of
          event time (`within` expiry, count chains, logical partners, every re-arming).

The engine gets the pushes in the generator's order (per batch: Card, Login, Transfer, Device), each
polled through the C-ABI (R18 order), and must reproduce the golden's digest and samples exactly."""
import os

import numpy as np
import pytest

from harness import App
from large_golden import Digest, golden_path, load

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _pushes(g):
    import sys
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_c5_golden import pushes
    return pushes({"events": g["prefix_events_per_stream"], "batch": g["batch"], "key_mod": g["key_mod"]})


_APPS = {}


def _app(patterns):
    """c5 and c5deep run the same 100K-pattern app: plan it once per session."""
    from siddhi_amd.workloads import c5_app
    if patterns not in _APPS:
        _APPS[patterns] = App(c5_app(patterns), engine_factory=lambda blob: None)
    return _APPS[patterns]


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("name", ["c5", "c5deep"])
def test_c5_golden_full_config(name):
    if not os.path.exists(golden_path(name)):
        pytest.skip(f"{golden_path(name)} not generated")
    from siddhi_amd.engine import HipEngine, columns_from_words
    from siddhi_amd.ir import T_FLOAT, T_INT
    g = load(name)
    app = _app(g["patterns"])
    types = [[T_INT, T_FLOAT, T_INT]] * 4
    eng = HipEngine(app.blob, stream_types=types, gen_max_keys=1 << 20)
    dig = Digest(g["sample_stride"])
    n_ev = 0
    for si, ts, vals in _pushes(g):
        if len(ts) == 0:
            continue
        eng.push_columns(si, ts, columns_from_words(vals, types[si]))
        n_ev += len(ts)
        dig.update(*eng.poll())
    assert n_ev == g["pushed_events"]
    assert dig.n == g["n_matches"], f"{name}: {dig.n} matches, golden {g['n_matches']}"
    assert dig.first == g["sample_first"]
    assert dig.strided == g["sample_strided"]
    assert dig.n_words == g["n_words"]
    assert dig.hexdigest() == g["digest"]
    assert eng.stats().live_partials > 0
