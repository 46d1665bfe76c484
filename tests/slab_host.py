"""ctypes wrapper of tests/native/libslab_host.so: the K_slab per-partial semantics (slab.h) run on
the host (test infrastructure only; see tests/native/slab_host.cpp)."""
import ctypes
import os
import subprocess

import numpy as np

from harness import decode_matches

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "libslab_host.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native"), "libslab_host.so"])
        L = ctypes.CDLL(SO)
        P, I64, VP = ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p
        L.slh_create.argtypes = [VP, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
        L.slh_create.restype = P
        L.slh_send.argtypes = [P, ctypes.c_int, I64, I64, VP, VP, VP]
        L.slh_num_matches.argtypes = [P]
        L.slh_num_matches.restype = I64
        L.slh_match_words.argtypes = [P]
        L.slh_match_words.restype = I64
        L.slh_live.argtypes = [P]
        L.slh_live.restype = I64
        L.slh_get_matches.argtypes = [P, VP, VP, VP, VP, VP]
        L.slh_clear.argtypes = [P]
        L.slh_error.argtypes = [P]
        L.slh_error.restype = ctypes.c_char_p
        L.slh_destroy.argtypes = [P]
        _lib = L
    return _lib


class SlabHostEngine:
    def __init__(self, blob):
        self.lib = lib()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        why = ctypes.create_string_buffer(256)
        self.h = self.lib.slh_create(self._blob, len(blob), why, 256)
        if not self.h:
            raise RuntimeError("not a K_slab app: " + why.value.decode())
        self.seq = 0

    def send(self, stream, ts, vals, nulls, as_chunk=False):
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        nl = None if nulls is None else np.ascontiguousarray(nulls, dtype=np.uint8)
        rc = self.lib.slh_send(self.h, stream, len(ts), self.seq, ts.ctypes.data, vals.ctypes.data,
                               None if nl is None else nl.ctypes.data)
        self.seq += len(ts)
        if rc != 0:
            raise RuntimeError(self.lib.slh_error(self.h).decode())

    def live(self):
        return self.lib.slh_live(self.h)

    def take_matches(self, n_slots_of):
        n = self.lib.slh_num_matches(self.h)
        nw = self.lib.slh_match_words(self.h)
        q, k, ts = (np.zeros(n, np.int64) for _ in range(3))
        off = np.zeros(n + 1, np.int64)
        words = np.zeros(max(nw, 1), np.int64)
        self.lib.slh_get_matches(self.h, q.ctypes.data, k.ctypes.data, ts.ctypes.data, off.ctypes.data,
                                 words.ctypes.data)
        self.lib.slh_clear(self.h)
        return decode_matches(n, q, k, ts, off, words, n_slots_of)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.slh_destroy(self.h)
            self.h = None
