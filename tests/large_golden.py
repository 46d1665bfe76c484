"""Large-stream golden vectors of SURVEY.md §8(c): each BASELINE config at its pattern count over a
seeded synthetic stream, pinned as (seed, config, digest of the R18-ordered match stream) plus an
explicit sample of matches.

Test infrastructure only. The digest is chunk-independent: the R18 delivery order is a
property of the whole stream, so the matches of consecutive polls concatenate to the same sequence
however the stream is cut into pushes. Five running SHA-256s cover the concatenated columns of the
ABI's sdh_matches (query, key, ts, per-match word count, words) as little-endian int64; the digest is
the SHA-256 of their hex digests.

Configs (BASELINE.json configs; workloads.py generators, event seed 42, pattern
seed 7):
  c1: 1 pattern (`every e1[price>20] -> e2[price>e1.price] within 10 sec`) x 1M events, 100 symbols
  c2: 1,000 C2 patterns x 1M events, 100 symbols
  c3: 1,000 C3 patterns (count <2:5>, logical and / or) x 200K events, partition over 10K symbols
  c4: 10,000 C4 fraud sequences x 200K Txn events, 100K accounts
  c2h: the headline configuration itself -- 10,000 C2 patterns (the metric's 10K) x 200K events,
       ~860M matches (tests/test_gpu_golden.py pushes it in 100K-event batches and in one 200K push)
  c2x: 10,000 patterns of the C2 family with an event-only conjunct on e2 (`volume > V_p`) x 200K events
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CONFIGS = {
    "c1": dict(patterns=1, events=1_000_000, keys=100, batch=1 << 16, stream="stock", sample_stride=2_000),
    "c2": dict(patterns=1000, events=1_000_000, keys=100, batch=1 << 16, stream="stock", sample_stride=1_000_000),
    "c3": dict(patterns=1000, events=200_000, keys=10_000, batch=1 << 15, stream="stock", sample_stride=50_000),
    "c4": dict(patterns=10_000, events=200_000, keys=100_000, batch=1 << 15, stream="txn", sample_stride=200_000),
    "c2h": dict(patterns=10_000, events=200_000, keys=100, batch=1 << 13, stream="stock", sample_stride=2_000_000),
    # the C2 family with an event-only conjunct on e2 (workloads.c2x_app), off K_ratchet
    "c2x": dict(patterns=10_000, events=200_000, keys=100, batch=1 << 13, stream="stock", sample_stride=2_000_000),
}
SAMPLE_FIRST = 500
SAMPLE_MAX_STRIDED = 500


def app_source(cfg_name: str, n_patterns: int, first: int = 0) -> str:
    from siddhi_amd.workloads import c1_app, c2_app, c2x_app, c3_app, c4_app
    if cfg_name == "c1":
        assert first == 0 and n_patterns == 1
        return c1_app()
    return {"c2": c2_app, "c2h": c2_app, "c2x": c2x_app, "c3": c3_app, "c4": c4_app}[cfg_name](n_patterns, first=first)


def events(cfg_name: str, start: int, n: int):
    """(ts, [col0, col1, col2] native-width columns, raw-word values [n, 3]) of the config's stream."""
    from siddhi_amd.workloads import stock_events, txn_events
    cfg = CONFIGS[cfg_name]
    gen = txn_events if cfg["stream"] == "txn" else stock_events
    ts, a, b, c = gen(start, n, cfg["keys"])
    cols = [a, b.view(np.uint32), c]
    vals = np.stack([a.astype(np.int64), b.view(np.uint32).astype(np.int64), c.astype(np.int64)], 1)
    return ts, cols, vals


class Digest:
    """Running digest + sample of an R18-ordered match stream given as ABI column arrays."""

    def __init__(self, stride: int):
        self.h = [hashlib.sha256() for _ in range(5)]
        self.n = 0
        self.n_words = 0
        self.stride = stride
        self.first = []
        self.strided = []

    def update(self, q, k, ts, off, words):
        n = len(q)
        if n == 0:
            return
        q = np.ascontiguousarray(q, dtype=np.int64)
        k = np.ascontiguousarray(k, dtype=np.int64)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        off = np.asarray(off, dtype=np.int64)
        assert off[0] == 0
        words = np.ascontiguousarray(words[:off[n]], dtype=np.int64)
        lens = np.ascontiguousarray(np.diff(off[:n + 1]), dtype=np.int64)
        for h, a in zip(self.h, (q, k, ts, lens, words)):
            h.update(a.tobytes())
        base = self.n
        take = [i for i in range(min(n, max(0, SAMPLE_FIRST - base)))]
        lo = (-base) % self.stride
        strided = list(range(lo, n, self.stride)) if len(self.strided) < SAMPLE_MAX_STRIDED else []
        for i in take:
            self.first.append(self._row(i, q, k, ts, off, words))
        for i in strided:
            if len(self.strided) >= SAMPLE_MAX_STRIDED:
                break
            self.strided.append([base + i] + self._row(i, q, k, ts, off, words))
        self.n += n
        self.n_words += int(off[n])

    @staticmethod
    def _row(i, q, k, ts, off, words):
        return [int(q[i]), int(k[i]), int(ts[i]), [int(x) for x in words[off[i]:off[i + 1]]]]

    def hexdigest(self) -> str:
        return hashlib.sha256("".join(h.hexdigest() for h in self.h).encode()).hexdigest()

    def summary(self) -> dict:
        return {"digest": self.hexdigest(), "n_matches": self.n, "n_words": self.n_words,
                "sample_first": self.first, "sample_stride": self.stride, "sample_strided": self.strided}


def golden_path(cfg_name: str) -> str:
    return os.path.join(GOLDEN_DIR, f"large_{cfg_name}.json")


def load(cfg_name: str) -> dict:
    with open(golden_path(cfg_name)) as f:
        return json.load(f)
