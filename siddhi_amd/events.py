"""Host-side event encoding shared by the runtime mirror and the tests.

Events cross the C-ABI as columns of raw 64-bit attribute words (``int``/``long`` sign-extended,
``float`` as its IEEE-754 binary32 pattern, ``double`` as its binary64 pattern, ``bool`` 0/1,
``string`` as a dictionary id) plus an optional null mask. Strings only support ``==``/``!=`` on
this path (R16), so dictionary ids compare exactly like ``String.equals``.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence

import numpy as np

from .ir import T_BOOL, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_STRING


class StringDictionary:
    """Process-wide string interning (id = order of first appearance)."""

    def __init__(self):
        self._ids: Dict[str, int] = {}
        self._strs: List[str] = []

    def intern(self, s: str) -> int:
        i = self._ids.get(s)
        if i is None:
            i = len(self._strs)
            self._ids[s] = i
            self._strs.append(s)
        return i

    def lookup(self, i: int) -> str:
        return self._strs[i]

    def __len__(self):
        return len(self._strs)


def encode_value(v, t: int, dictionary: StringDictionary) -> (int, int):
    """Python value -> (raw int64 word, is_null)."""
    if v is None:
        return 0, 1
    if t == T_INT:
        return int(np.int32(v)), 0
    if t == T_LONG:
        return int(np.int64(v)), 0
    if t == T_FLOAT:
        return struct.unpack("<I", struct.pack("<f", float(v)))[0], 0
    if t == T_DOUBLE:
        return struct.unpack("<q", struct.pack("<d", float(v)))[0], 0
    if t == T_BOOL:
        return (1 if v else 0), 0
    if t == T_STRING:
        return dictionary.intern(str(v)), 0
    raise TypeError(f"unsupported attribute type {t}")


def decode_value(raw: int, t: int, dictionary: StringDictionary):
    if t == T_INT:
        return int(np.int64(raw).astype(np.int32))
    if t == T_LONG:
        return int(raw)
    if t == T_FLOAT:
        return np.float32(struct.unpack("<f", struct.pack("<I", raw & 0xFFFFFFFF))[0])
    if t == T_DOUBLE:
        return struct.unpack("<d", struct.pack("<q", raw))[0]
    if t == T_BOOL:
        return bool(raw)
    if t == T_STRING:
        return dictionary.lookup(int(raw))
    raise TypeError(t)


def encode_rows(rows: Sequence[Sequence], types: Sequence[int], dictionary: StringDictionary):
    """Rows of Python values -> (vals int64[n, a], nulls uint8[n, a])."""
    n, a = len(rows), len(types)
    vals = np.zeros((n, a), dtype=np.int64)
    nulls = np.zeros((n, a), dtype=np.uint8)
    for i, row in enumerate(rows):
        if len(row) != a:
            raise ValueError(f"event has {len(row)} attributes, stream defines {a}")
        for j, (v, t) in enumerate(zip(row, types)):
            vals[i, j], nulls[i, j] = encode_value(v, t, dictionary)
    return vals, nulls


class EventLog:
    """Values of every event seen so far, indexed by global sequence number (host-side mirror
    used to project match tuples into output rows)."""

    def __init__(self):
        self.stream: List[int] = []
        self.ts: List[int] = []
        self.vals: List[np.ndarray] = []
        self.nulls: List[np.ndarray] = []

    def append(self, stream: int, ts: Sequence[int], vals: np.ndarray, nulls: Optional[np.ndarray]):
        for k in range(len(ts)):
            self.stream.append(stream)
            self.ts.append(int(ts[k]))
            self.vals.append(vals[k])
            self.nulls.append(nulls[k] if nulls is not None else np.zeros(vals.shape[1], np.uint8))

    def __len__(self):
        return len(self.ts)
