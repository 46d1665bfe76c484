"""Shared driver of the C5-family parity tests (BASELINE.json configs[4], reduced): four joined
streams pushed in alternating per-stream batches through one engine (test infrastructure)."""
import numpy as np

from harness import App
from siddhi_amd.workloads import C5_STREAMS, c5_app, c5_events


def run_c5(n_patterns, n_accounts, n_per_stream, batch, engine_factory=None, first=0):
    app = App(c5_app(n_patterns, first=first), engine_factory)
    for lo in range(0, n_per_stream, batch):
        n = min(batch, n_per_stream - lo)
        for si, name in enumerate(C5_STREAMS):
            ts, acct, amount, code = c5_events(si, lo, n, n_accounts)
            vals = np.stack([acct.astype(np.int64), amount.view(np.uint32).astype(np.int64),
                             code.astype(np.int64)], 1)
            app.engine.send(app.ir.stream_index(name), ts, vals, None)
            app.matches.extend(app.engine.take_matches(lambda q: len(app.ir.queries[q].states)))
    return app
