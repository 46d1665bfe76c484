"""ctypes wrapper of tests/native/libkgen_host.so: the K_gen interpreter body compiled for the host
(test infrastructure only; see tests/native/kgen_host.cpp)."""
import ctypes
import os
import subprocess

import numpy as np

from harness import decode_matches

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "libkgen_host.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
        L = ctypes.CDLL(SO)
        P, I64, VP = ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p
        L.kgh_create.argtypes = [VP, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.kgh_create.restype = P
        L.kgh_send.argtypes = [P, ctypes.c_int, I64, I64, VP, VP, VP]
        L.kgh_num_matches.argtypes = [P]
        L.kgh_num_matches.restype = I64
        L.kgh_match_words.argtypes = [P]
        L.kgh_match_words.restype = I64
        L.kgh_get_matches.argtypes = [P, VP, VP, VP, VP, VP]
        L.kgh_clear.argtypes = [P]
        L.kgh_set_chunk.argtypes = [P, I64]
        L.kgh_set_window.argtypes = [P, ctypes.c_int]
        L.kgh_error.argtypes = [P]
        L.kgh_error.restype = ctypes.c_char_p
        L.kgh_destroy.argtypes = [P]
        L.kgh_start.argtypes = [P, I64]
        L.kgh_set_playback.argtypes = [P, ctypes.c_int]
        L.kgh_advance.argtypes = [P, I64, I64]
        _lib = L
    return _lib


class KGenHostEngine:
    def __init__(self, blob, R=0, N=0, LC=0, chunk_len=0, window=False):
        self.lib = lib()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        self.h = self.lib.kgh_create(self._blob, len(blob), R, N, LC)
        if not self.h:
            raise RuntimeError("K_gen lowering failed")
        self.lib.kgh_set_chunk(self.h, chunk_len)
        self.lib.kgh_set_window(self.h, int(window))
        self.seq = 0

    def send(self, stream, ts, vals, nulls, as_chunk=False):
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        vals = np.ascontiguousarray(vals, dtype=np.int64)
        nl = None if nulls is None else np.ascontiguousarray(nulls, dtype=np.uint8)
        rc = self.lib.kgh_send(self.h, stream, len(ts), self.seq, ts.ctypes.data, vals.ctypes.data,
                               None if nl is None else nl.ctypes.data)
        self.seq += len(ts)
        if rc != 0:
            raise RuntimeError(self.lib.kgh_error(self.h).decode())

    def set_playback(self, on: bool):
        self.lib.kgh_set_playback(self.h, int(on))

    def start(self, t: int):
        self.lib.kgh_start(self.h, int(t))

    def advance_time(self, t: int):
        if self.lib.kgh_advance(self.h, int(t), self.seq) != 0:
            raise RuntimeError(self.lib.kgh_error(self.h).decode())

    def take_matches(self, n_slots_of):
        n = self.lib.kgh_num_matches(self.h)
        nw = self.lib.kgh_match_words(self.h)
        q, k, ts = (np.zeros(n, np.int64) for _ in range(3))
        off = np.zeros(n + 1, np.int64)
        words = np.zeros(max(nw, 1), np.int64)
        self.lib.kgh_get_matches(self.h, q.ctypes.data, k.ctypes.data, ts.ctypes.data, off.ctypes.data,
                                 words.ctypes.data)
        self.lib.kgh_clear(self.h)
        return decode_matches(n, q, k, ts, off, words, n_slots_of)

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.kgh_destroy(self.h)
            self.h = None
