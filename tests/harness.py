"""Test harness: runs a SiddhiQL app on the CPU oracle (oracle/liboracle.so) or on the HIP engine
and projects the matches like the reference's QueryCallback would see them.

Test infrastructure only (it loads the oracle)."""
from __future__ import annotations

import ctypes
import os
import struct
import subprocess
from typing import Dict, List, Optional, Sequence

import numpy as np

from siddhi_amd import ql
from siddhi_amd.events import EventLog, StringDictionary, encode_rows
from siddhi_amd.ir import T_BOOL, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_STRING
from siddhi_amd.planner import plan
from siddhi_amd.selector import project, stream_rows

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")

_lib = None


def oracle_lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle")])
        lib = ctypes.CDLL(ORACLE_SO)
        P, I64, VP = ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p
        lib.oracle_create.argtypes = [VP, ctypes.c_size_t, ctypes.POINTER(P)]
        lib.oracle_send.argtypes = [P, ctypes.c_int32, I64, VP, VP, VP, ctypes.c_int]
        lib.oracle_num_matches.argtypes = [P]
        lib.oracle_num_matches.restype = I64
        lib.oracle_match_words.argtypes = [P]
        lib.oracle_match_words.restype = I64
        lib.oracle_get_matches.argtypes = [P, VP, VP, VP, VP, VP]
        lib.oracle_clear_matches.argtypes = [P]
        lib.oracle_get_match_meta.argtypes = [P, VP, VP]
        lib.oracle_live_partials.argtypes = [P]
        lib.oracle_live_partials.restype = I64
        lib.oracle_error.argtypes = [P]
        lib.oracle_error.restype = ctypes.c_char_p
        lib.oracle_destroy.argtypes = [P]
        lib.oracle_start.argtypes = [P, I64]
        lib.oracle_advance_time.argtypes = [P, I64]
        lib.oracle_set_playback.argtypes = [P, ctypes.c_int]
        lib.oracle_set_strings.argtypes = [P, I64, VP, VP, VP]
        _lib = lib
    return _lib


class OracleError(RuntimeError):
    pass


def decode_matches(n, q, k, ts, off, words, n_slots_of):
    out = []
    for i in range(n):
        w = words[off[i]:off[i + 1]]
        slots = []
        j = 0
        for _ in range(n_slots_of(int(q[i]))):
            c = int(w[j])
            slots.append(tuple(int(x) for x in w[j + 1:j + 1 + c]))
            j += 1 + c
        out.append((int(q[i]), int(k[i]), int(ts[i]), tuple(slots)))
    return out


class OracleEngine:
    """Thin ctypes wrapper over liboracle.so."""

    def __init__(self, blob: bytes):
        self.lib = oracle_lib()
        self.h = ctypes.c_void_p()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        rc = self.lib.oracle_create(self._blob, len(blob), ctypes.byref(self.h))
        if rc != 0:
            raise OracleError("oracle_create failed (bad IR)")

    def send(self, stream: int, ts, vals: np.ndarray, nulls: Optional[np.ndarray], as_chunk=False):
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        nl = None if nulls is None else np.ascontiguousarray(nulls, dtype=np.uint8)
        rc = self.lib.oracle_send(self.h, stream, len(ts), ts.ctypes.data, vals.ctypes.data,
                                  None if nl is None else nl.ctypes.data, int(as_chunk))
        if rc != 0:
            raise OracleError(self.lib.oracle_error(self.h).decode())

    def set_playback(self, on: bool):
        self.lib.oracle_set_playback(self.h, int(on))

    def set_strings(self, ids, texts):
        from siddhi_amd.planner import java_string_hash
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        h = np.array([java_string_hash(t) for t in texts], dtype=np.int32)
        ln = np.array([len(t.encode("utf-16-le")) // 2 for t in texts], dtype=np.int32)
        self.lib.oracle_set_strings(self.h, len(ids), ids.ctypes.data, h.ctypes.data, ln.ctypes.data)

    def start(self, t: int):
        if self.lib.oracle_start(self.h, int(t)) != 0:
            raise OracleError(self.lib.oracle_error(self.h).decode())

    def advance_time(self, t: int):
        if self.lib.oracle_advance_time(self.h, int(t)) != 0:
            raise OracleError(self.lib.oracle_error(self.h).decode())

    def take_matches(self, n_slots_of, meta=None):
        """Decoded matches (and, when `meta` is a list, (trigger seq, timer tiebreak) per match
        appended to it), clearing them."""
        n = self.lib.oracle_num_matches(self.h)
        nw = self.lib.oracle_match_words(self.h)
        q = np.zeros(n, np.int64)
        k = np.zeros(n, np.int64)
        ts = np.zeros(n, np.int64)
        off = np.zeros(n + 1, np.int64)
        words = np.zeros(max(nw, 1), np.int64)
        self.lib.oracle_get_matches(self.h, q.ctypes.data, k.ctypes.data, ts.ctypes.data,
                                    off.ctypes.data, words.ctypes.data)
        if meta is not None:
            seq = np.zeros(max(n, 1), np.int64)
            tb = np.zeros(max(n, 1), np.int64)
            self.lib.oracle_get_match_meta(self.h, seq.ctypes.data, tb.ctypes.data)
            meta.extend(zip(seq[:n].tolist(), tb[:n].tolist()))
        self.lib.oracle_clear_matches(self.h)
        return decode_matches(n, q, k, ts, off, words, n_slots_of)

    def __del__(self):
        if getattr(self, "h", None) and self.h:
            self.lib.oracle_destroy(self.h)
            self.h = None


def parse_literal(tok: str, attr_type: Optional[int] = None):
    """Fixture literal (extract_reference_tests._literal) -> Python value."""
    if tok == "null":
        return None
    kind, v = tok.split(":", 1)
    if kind == "s":
        return v
    if kind == "b":
        return v == "true"
    if kind == "f":
        return np.float32(float(v))
    if kind in ("d",):
        return float(v)
    return int(v)


class App:
    """Compile an app and feed it to an engine (default: the oracle)."""

    def __init__(self, src: str, engine_factory=None):
        self.ast = ql.parse(src)
        self.ir = plan(self.ast)
        self.dictionary = StringDictionary()
        self.string_ids = [self.dictionary.intern(s) for s in self.ir.strings]
        self.blob = self.ir.serialize(self.string_ids)
        self.engine = (engine_factory or OracleEngine)(self.blob)
        self.playback = bool(self.ast.annotations.get("app:playback"))
        if self.playback and hasattr(self.engine, "set_playback"):
            self.engine.set_playback(True)   # (the HIP engine takes SDH_FLAG_PLAYBACK at create)
        self.log = EventLog()
        self._strings_sent = 0  # dictionary ids whose text the engine has (set_strings)
        self.matches: List[tuple] = []
        self.meta: List[tuple] = []  # per match (trigger seq, timer tiebreak) when the engine has them

    def stream_types(self, name: str) -> List[int]:
        return self.ir.streams[self.ir.stream_index(name)].attr_types

    def send(self, stream: str, rows: Sequence[Sequence], ts: Sequence[int], as_chunk=False):
        si = self.ir.stream_index(stream)
        vals, nulls = encode_rows(rows, self.ir.streams[si].attr_types, self.dictionary)
        self.log.append(si, ts, vals, nulls)
        n = len(self.dictionary)
        if n > self._strings_sent and hasattr(self.engine, "set_strings"):
            ids = list(range(self._strings_sent, n))
            self.engine.set_strings(ids, [self.dictionary.lookup(i) for i in ids])
            self._strings_sent = n
        self.engine.send(si, ts, vals, nulls, as_chunk)
        self._take()

    def start(self, t: int):
        """SiddhiAppRuntime.start at time t (absent patterns schedule from it)."""
        self.engine.start(t)

    def advance_time(self, t: int):
        """Time passes to t with no event: absent patterns' schedulers fire what falls due."""
        self.engine.advance_time(t)
        self._take()

    def _take(self):
        n_slots = lambda q: len(self.ir.queries[q].states)  # noqa: E731
        if isinstance(self.engine, OracleEngine):
            self.matches.extend(self.engine.take_matches(n_slots, self.meta))
        else:
            self.matches.extend(self.engine.take_matches(n_slots))

    def rows_for_query(self, qname: str):
        qi = self.ir.query_index(qname)
        q = self.ir.queries[qi]
        return [project(q, m[3], self.log, None, self.dictionary, self.ir.strings)
                for m in self.matches if m[0] == qi]

    def rows_for_stream(self, stream: str):
        return stream_rows(self.ir, self.matches, self.log, self.dictionary, self.ir.strings, stream)


def values_equal(expected_tok: str, actual) -> bool:
    e = parse_literal(expected_tok)
    if e is None or actual is None:
        return e is None and actual is None
    if isinstance(e, np.float32):
        return isinstance(actual, (np.float32, float)) and np.float32(actual) == e
    if isinstance(e, float):
        return float(actual) == e
    if isinstance(e, bool):
        return isinstance(actual, (bool, np.bool_)) and bool(actual) == e
    if isinstance(e, int):
        return not isinstance(actual, (bool, np.bool_, float, np.floating)) and int(actual) == e
    return e == actual
