"""ctypes binding of libsiddhi_hip.so (include/siddhi_hip.h).

This is the product path: it loads the in-tree HIP library and fails loudly when it is missing or
when no GPU is visible -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence

import numpy as np

from .ir import T_BOOL, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_STRING

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libsiddhi_hip.so")

SDH_OK = 0
SDH_FLAG_DEVICE_MATCHES = 1
SDH_FLAG_NO_RATCHET = 2
SDH_FLAG_FORCE_GEN = 4
SDH_FLAG_PLAYBACK = 8  # @app:playback timer semantics (include/siddhi_hip.h)
ERRORS = {-1: "SDH_E_INVALID", -2: "SDH_E_UNSUPPORTED", -3: "SDH_E_DEVICE", -4: "SDH_E_CAPACITY",
          -5: "SDH_E_REFERENCE"}


class SdhConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("shard_rank", ctypes.c_int32),
                ("shard_world", ctypes.c_int32), ("partials_per_inst", ctypes.c_int32),
                ("max_batch", ctypes.c_int64), ("match_capacity", ctypes.c_int64),
                ("chunk_events", ctypes.c_int32), ("flags", ctypes.c_int32),
                ("gen_pool_states", ctypes.c_int32), ("gen_pool_nodes", ctypes.c_int32),
                ("gen_list_cap", ctypes.c_int32), ("gen_pad", ctypes.c_int32),
                ("gen_max_keys", ctypes.c_int64), ("debug", ctypes.c_char_p)]


def debug_string(debug) -> Optional[bytes]:
    """sdh_config.debug from a {NAME: VALUE} dict or a "NAME=VALUE;..." string. The test / bench harness
    may also pass knobs through SIDDHI_HIP_DEBUG (the library itself reads no environment)."""
    parts = []
    env = os.environ.get("SIDDHI_HIP_DEBUG")
    if env:
        parts.append(env)
    if isinstance(debug, dict):
        parts.append(";".join(f"{k}={v}" for k, v in debug.items()))
    elif debug:
        parts.append(str(debug))
    return ";".join(parts).encode() if parts else None


class SdhRecords(ctypes.Structure):
    """sdh_records (include/siddhi_hip.h): the last push's device records, three parts."""
    _fields_ = [("n", ctypes.c_int64), ("seq_base", ctypes.c_int64), ("n_events", ctypes.c_int64),
                ("r_n", ctypes.c_int64), ("r_blocks", ctypes.c_int64), ("r_bytes", ctypes.c_int64),
                ("r_base", ctypes.c_void_p), ("r_count", ctypes.c_void_p), ("r_side", ctypes.c_void_p),
                ("r_group", ctypes.c_void_p), ("r_lane_query", ctypes.c_void_p),
                ("r_format", ctypes.c_int32), ("r_blk_bytes", ctypes.c_int32),
                ("f_n", ctypes.c_int64), ("f_words", ctypes.c_int64), ("f_base", ctypes.c_void_p),
                ("f_query_keys", ctypes.c_void_p),
                ("c_n", ctypes.c_int64), ("c_items", ctypes.c_int64), ("c_words", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("c_base", ctypes.c_void_p), ("c_off", ctypes.c_void_p),
                ("c_count", ctypes.c_void_p)]


SDH_REC_NONE, SDH_REC_8, SDH_REC_16, SDH_REC_4 = 0, 1, 2, 3


class SdhBatch(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("ts", ctypes.c_void_p), ("cols", ctypes.POINTER(ctypes.c_void_p)),
                ("nulls", ctypes.POINTER(ctypes.c_void_p)), ("n_cols", ctypes.c_int32),
                ("on_device", ctypes.c_int32), ("chunk", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class SdhMatches(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("query", ctypes.POINTER(ctypes.c_int64)),
                ("key", ctypes.POINTER(ctypes.c_int64)), ("ts", ctypes.POINTER(ctypes.c_int64)),
                ("off", ctypes.POINTER(ctypes.c_int64)), ("words", ctypes.POINTER(ctypes.c_int64)),
                ("seq", ctypes.POINTER(ctypes.c_int64)), ("tb", ctypes.POINTER(ctypes.c_int64))]


class SdhMatchesCompact(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("seq_base", ctypes.c_int64), ("width", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("rows", ctypes.POINTER(ctypes.c_int32))]


class SdhMatchesCompactEx(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("seq_base", ctypes.c_int64), ("width", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("rows", ctypes.POINTER(ctypes.c_int32)),
                ("key", ctypes.POINTER(ctypes.c_int64)), ("tb", ctypes.POINTER(ctypes.c_int64)),
                ("n_chain", ctypes.c_int64), ("chain", ctypes.POINTER(ctypes.c_int32))]


class SdhStats(ctypes.Structure):
    _fields_ = [("events", ctypes.c_int64), ("pattern_events", ctypes.c_int64),
                ("matches", ctypes.c_int64), ("live_partials", ctypes.c_int64),
                ("last_kernel_ms", ctypes.c_double), ("last_kernel_bytes", ctypes.c_double),
                ("last_gen_items", ctypes.c_int64), ("last_seq_items", ctypes.c_int64),
                ("last_part_items", ctypes.c_int64), ("last_ingest_ms", ctypes.c_double),
                ("ingest_bytes", ctypes.c_int64), ("spec_kernels", ctypes.c_int64),
                ("pool_regrows", ctypes.c_int64), ("last_slab_items", ctypes.c_int64),
                ("placed_pushes", ctypes.c_int64), ("plan_queries", ctypes.c_int64 * 8)]

PLANS = ("K_ratchet", "K_gate", "K_chain", "K_part", "K_slab", "K_seq", "K_gen")


EXPORTS = ["sdh_engine_create", "sdh_engine_push", "sdh_engine_flush", "sdh_engine_poll", "sdh_engine_poll_device",
           "sdh_engine_poll_compact", "sdh_engine_poll_compact_ex",
           "sdh_engine_pending_matches", "sdh_engine_start", "sdh_engine_advance_time", "sdh_engine_stats",
           "sdh_engine_snapshot", "sdh_engine_state_bytes",
           "sdh_engine_restore", "sdh_free", "sdh_engine_destroy", "sdh_last_error", "sdh_version",
           "sdh_engine_debug_digest", "sdh_engine_set_strings", "sdh_calibrate_hbm", "sdh_build_info",
           "sdh_engine_push_stats", "sdh_comm_get_id", "sdh_comm_create", "sdh_comm_create_local",
           "sdh_comm_destroy", "sdh_comm_last_error", "sdh_engine_set_comm", "sdh_engine_push_bcast",
           "sdh_engine_gather", "sdh_engine_reserve", "sdh_engine_reserve_keys", "sdh_engine_poll_records",
           "sdh_engine_records_compact"]
SDH_COMM_ID_BYTES = 128

_lib = None


def load_library(path: str = LIB_PATH):
    """Load libsiddhi_hip.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("SIDDHI_HIP_LIB", path)  # alternative builds (kernel tuning experiments)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(the HIP engine has no CPU fallback)")
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    lib.sdh_engine_create.argtypes = [P, ctypes.c_size_t, ctypes.POINTER(SdhConfig), ctypes.POINTER(P)]
    lib.sdh_engine_push.argtypes = [P, ctypes.c_int32, ctypes.POINTER(SdhBatch)]
    lib.sdh_engine_flush.argtypes = [P]
    lib.sdh_engine_poll.argtypes = [P, ctypes.POINTER(SdhMatches)]
    lib.sdh_engine_poll_device.argtypes = [P, ctypes.POINTER(SdhMatches)]
    lib.sdh_engine_poll_compact.argtypes = [P, ctypes.c_int32, ctypes.POINTER(SdhMatchesCompact)]
    lib.sdh_engine_poll_compact_ex.argtypes = [P, ctypes.c_int32, ctypes.POINTER(SdhMatchesCompactEx)]
    lib.sdh_engine_pending_matches.argtypes = [P, ctypes.POINTER(ctypes.c_int64)]
    lib.sdh_engine_poll_records.argtypes = [P, ctypes.POINTER(SdhRecords)]
    lib.sdh_engine_records_compact.argtypes = [P, P, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64)]
    lib.sdh_engine_start.argtypes = [P, ctypes.c_int64]
    lib.sdh_engine_advance_time.argtypes = [P, ctypes.c_int64]
    lib.sdh_engine_stats.argtypes = [P, ctypes.POINTER(SdhStats)]
    I64P = ctypes.POINTER(ctypes.c_int64)
    lib.sdh_engine_state_bytes.argtypes = [P, I64P, I64P, I64P]
    lib.sdh_engine_reserve.argtypes = [P, ctypes.c_int64]
    lib.sdh_engine_reserve_keys.argtypes = [P, ctypes.c_int64]
    lib.sdh_engine_snapshot.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
    lib.sdh_engine_restore.argtypes = [P, ctypes.c_void_p, ctypes.c_size_t]
    lib.sdh_free.argtypes = [P]
    lib.sdh_engine_destroy.argtypes = [P]
    lib.sdh_last_error.argtypes = [P]
    lib.sdh_last_error.restype = ctypes.c_char_p
    lib.sdh_version.restype = ctypes.c_char_p
    lib.sdh_build_info.restype = ctypes.c_char_p
    lib.sdh_engine_push_stats.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
    lib.sdh_engine_debug_digest.argtypes = [P, ctypes.POINTER(ctypes.c_uint64)]
    lib.sdh_engine_set_strings.argtypes = [P, ctypes.c_int64, P, P, P]
    D = ctypes.POINTER(ctypes.c_double)
    lib.sdh_calibrate_hbm.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int32, D, D]
    lib.sdh_comm_get_id.argtypes = [P, ctypes.c_size_t]
    lib.sdh_comm_create.argtypes = [P, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.POINTER(P)]
    lib.sdh_comm_create_local.argtypes = [ctypes.c_int32, P, ctypes.POINTER(P)]
    lib.sdh_comm_destroy.argtypes = [P]
    lib.sdh_comm_last_error.restype = ctypes.c_char_p
    lib.sdh_engine_set_comm.argtypes = [P, P]
    lib.sdh_engine_push_bcast.argtypes = [P, ctypes.c_int32, ctypes.POINTER(SdhBatch), ctypes.c_int32]
    lib.sdh_engine_gather.argtypes = [P, ctypes.c_int32, ctypes.POINTER(SdhMatches)]
    _lib = lib
    return lib


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def _matches_to_arrays(m: SdhMatches, with_seq: bool):
    """Host sdh_matches -> (query, key, ts, off, words[, seq, tb]) numpy copies."""
    n = m.n
    if n == 0:
        z = np.zeros(0, np.int64)
        return (z, z, z, np.zeros(1, np.int64), z) + ((z, z) if with_seq else ())
    q = np.ctypeslib.as_array(m.query, shape=(n,)).copy()
    k = np.ctypeslib.as_array(m.key, shape=(n,)).copy()
    ts = np.ctypeslib.as_array(m.ts, shape=(n,)).copy()
    off = np.ctypeslib.as_array(m.off, shape=(n + 1,)).copy()
    words = np.ctypeslib.as_array(m.words, shape=(int(off[-1]),)).copy() if off[-1] else np.zeros(0, np.int64)
    if with_seq:
        return (q, k, ts, off, words, np.ctypeslib.as_array(m.seq, shape=(n,)).copy(),
                np.ctypeslib.as_array(m.tb, shape=(n,)).copy())
    return q, k, ts, off, words


_NP_OF = {T_INT: np.int32, T_LONG: np.int64, T_FLOAT: np.uint32, T_DOUBLE: np.int64, T_BOOL: np.uint8,
          T_STRING: np.int32}


def columns_from_words(vals: np.ndarray, types: Sequence[int]) -> List[np.ndarray]:
    """Raw 64-bit attribute words [n, a] -> native-width columns (see sdh_batch)."""
    cols = []
    for j, t in enumerate(types):
        w = vals[:, j]
        if t in (T_FLOAT,):
            cols.append(np.ascontiguousarray((w & 0xFFFFFFFF).astype(np.uint32)))
        elif t in (T_INT, T_STRING):
            cols.append(np.ascontiguousarray(w.astype(np.int64).astype(np.int32)))
        elif t == T_BOOL:
            cols.append(np.ascontiguousarray(w.astype(np.uint8)))
        else:
            cols.append(np.ascontiguousarray(w.astype(np.int64)))
    return cols


class HipEngine:
    """One engine instance on one GPU."""

    def __init__(self, blob: bytes, device: int = 0, partials: int = 128, shard_rank: int = 0,
                 shard_world: int = 1, chunk_events: int = 0, stream_types=None, flags: int = 0,
                 gen_pool_states: int = 0, gen_pool_nodes: int = 0, gen_list_cap: int = 0,
                 gen_max_keys: int = 0, debug=None):
        self.lib = load_library()
        self._debug = debug_string(debug)
        cfg = SdhConfig(device=device, shard_rank=shard_rank, shard_world=shard_world,
                        partials_per_inst=partials, max_batch=0, match_capacity=0,
                        chunk_events=chunk_events, flags=flags, gen_pool_states=gen_pool_states,
                        gen_pool_nodes=gen_pool_nodes, gen_list_cap=gen_list_cap, gen_pad=0,
                        gen_max_keys=gen_max_keys, debug=self._debug)
        self.h = ctypes.c_void_p()
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        rc = self.lib.sdh_engine_create(self._blob, len(blob), ctypes.byref(cfg), ctypes.byref(self.h))
        if rc != SDH_OK:
            raise EngineError(rc, self.lib.sdh_last_error(None).decode())
        self.stream_types = stream_types

    def _check(self, rc):
        if rc != SDH_OK:
            raise EngineError(rc, self.lib.sdh_last_error(self.h).decode())

    def push_columns(self, stream: int, ts: np.ndarray, cols: Sequence[np.ndarray],
                     nulls: Optional[Sequence[Optional[np.ndarray]]] = None, chunk: bool = False):
        """Push host columns: n single-event sends, or (chunk) one ``InputHandler.send(Event[])``."""
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        keep = [ts] + list(cols)
        cp = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        nptr = None
        if nulls is not None:
            nl = [None if x is None else np.ascontiguousarray(x, dtype=np.uint8) for x in nulls]
            keep += [x for x in nl if x is not None]
            nptr = (ctypes.c_void_p * len(cols))(*[0 if x is None else x.ctypes.data for x in nl])
        b = SdhBatch(n=len(ts), ts=ts.ctypes.data, cols=cp, nulls=nptr, n_cols=len(cols), on_device=0,
                     chunk=int(chunk))
        self._check(self.lib.sdh_engine_push(self.h, stream, ctypes.byref(b)))
        del keep

    def push_device(self, stream: int, n: int, ts_ptr: int, col_ptrs: Sequence[int], chunk: bool = False):
        """Push a batch whose columns are already resident in HBM (e.g. torch CUDA tensors)."""
        cp = (ctypes.c_void_p * len(col_ptrs))(*col_ptrs)
        b = SdhBatch(n=n, ts=ts_ptr, cols=cp, nulls=None, n_cols=len(col_ptrs), on_device=1, chunk=int(chunk))
        self._check(self.lib.sdh_engine_push(self.h, stream, ctypes.byref(b)))

    # interface used by tests/harness.App -------------------------------------------------------
    def send(self, stream: int, ts, vals: np.ndarray, nulls: Optional[np.ndarray], as_chunk=False):
        types = self.stream_types[stream]
        cols = columns_from_words(np.asarray(vals, dtype=np.int64).reshape(len(ts), len(types)), types)
        nl = None
        if nulls is not None and np.any(nulls):
            nl = [np.ascontiguousarray(nulls[:, j]) for j in range(len(types))]
        self.push_columns(stream, np.asarray(ts, dtype=np.int64), cols, nl, chunk=as_chunk)

    def poll(self, with_seq: bool = False):
        """R18-ordered matches since the last poll as arrays (query, key, ts, off, words[, seq, tb])."""
        m = SdhMatches()
        self._check(self.lib.sdh_engine_poll(self.h, ctypes.byref(m)))
        return _matches_to_arrays(m, with_seq)

    def set_comm(self, comm: Optional["Comm"]):
        """Attach a communicator (sdh_engine_set_comm); the engine does not own it."""
        self._comm = comm
        self._check(self.lib.sdh_engine_set_comm(self.h, comm.h if comm is not None else None))

    def push_bcast_device(self, stream: int, n: int, ts_ptr: int, col_ptrs: Sequence[int], root: int = 0,
                          chunk: bool = False):
        """Collective push (sdh_engine_push_bcast): the root's batch, resident in HBM, reaches every
        rank; the other ranks call push_bcast_recv."""
        cp = (ctypes.c_void_p * len(col_ptrs))(*col_ptrs)
        b = SdhBatch(n=n, ts=ts_ptr, cols=cp, nulls=None, n_cols=len(col_ptrs), on_device=1, chunk=int(chunk))
        self._check(self.lib.sdh_engine_push_bcast(self.h, stream, ctypes.byref(b), root))

    def push_bcast_columns(self, stream: int, ts: np.ndarray, cols: Sequence[np.ndarray],
                           nulls: Optional[Sequence[Optional[np.ndarray]]] = None, root: int = 0, chunk: bool = False):
        """Collective push from the root's host columns."""
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        cp = (ctypes.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
        nptr, keep = None, []
        if nulls is not None:
            nl = [None if x is None else np.ascontiguousarray(x, dtype=np.uint8) for x in nulls]
            keep = [x for x in nl if x is not None]
            nptr = (ctypes.c_void_p * len(cols))(*[0 if x is None else x.ctypes.data for x in nl])
        b = SdhBatch(n=len(ts), ts=ts.ctypes.data, cols=cp, nulls=nptr, n_cols=len(cols), on_device=0,
                     chunk=int(chunk))
        self._check(self.lib.sdh_engine_push_bcast(self.h, stream, ctypes.byref(b), root))
        del keep

    def push_bcast_recv(self, root: int = 0):
        """A non-root rank's side of push_bcast_*: the batch comes from the root."""
        self._check(self.lib.sdh_engine_push_bcast(self.h, 0, None, root))

    def send_bcast(self, stream: int, ts, vals: np.ndarray, nulls: Optional[np.ndarray], root: int = 0,
                   as_chunk=False):
        """tests/harness.App interface, as send() but through the broadcast (root side)."""
        types = self.stream_types[stream]
        cols = columns_from_words(np.asarray(vals, dtype=np.int64).reshape(len(ts), len(types)), types)
        nl = None
        if nulls is not None and np.any(nulls):
            nl = [np.ascontiguousarray(nulls[:, j]) for j in range(len(types))]
        self.push_bcast_columns(stream, np.asarray(ts, dtype=np.int64), cols, nl, root=root, chunk=as_chunk)

    def gather(self, device: bool = False):
        """Collective poll (sdh_engine_gather). Host: (query, key, ts, off, words, seq, tb) arrays
        on rank 0 (empty elsewhere); device: the SdhMatches struct of HBM pointers."""
        m = SdhMatches()
        self._check(self.lib.sdh_engine_gather(self.h, int(device), ctypes.byref(m)))
        if device:
            return m
        return _matches_to_arrays(m, True)

    def poll_device(self) -> SdhMatches:
        """R18-sorted matches since the last poll, left in HBM: the SdhMatches fields are device
        pointers (valid until the next push / poll)."""
        m = SdhMatches()
        self._check(self.lib.sdh_engine_poll_device(self.h, ctypes.byref(m)))
        return m

    def poll_compact(self, device: bool = False):
        """The same matches as compact int32 rows (sdh_engine_poll_compact): (seq_base, rows[n, width])
        on the host, or the SdhMatchesCompact struct (rows a device pointer) when device is set."""
        m = SdhMatchesCompact()
        self._check(self.lib.sdh_engine_poll_compact(self.h, int(device), ctypes.byref(m)))
        if device:
            return m
        if m.n == 0:
            return m.seq_base, np.zeros((0, m.width), np.int32)
        return m.seq_base, np.ctypeslib.as_array(m.rows, shape=(m.n, m.width)).copy()

    def poll_compact_ex(self, device: bool = False):
        """Compact rows for every match (sdh_engine_poll_compact_ex): host arrays (seq_base, rows[n, width],
        key or None, tb or None, chain), or the SdhMatchesCompactEx struct of HBM pointers (device)."""
        m = SdhMatchesCompactEx()
        self._check(self.lib.sdh_engine_poll_compact_ex(self.h, int(device), ctypes.byref(m)))
        if device:
            return m
        n, w = m.n, m.width
        rows = np.ctypeslib.as_array(m.rows, shape=(n, w)).copy() if n else np.zeros((0, w), np.int32)
        key = np.ctypeslib.as_array(m.key, shape=(n,)).copy() if (m.key and n) else (np.zeros(0, np.int64) if m.key else None)
        tb = np.ctypeslib.as_array(m.tb, shape=(n,)).copy() if (m.tb and n) else (np.zeros(0, np.int64) if m.tb else None)
        chain = np.ctypeslib.as_array(m.chain, shape=(m.n_chain,)).copy() if m.n_chain else np.zeros(0, np.int32)
        return m.seq_base, rows, key, tb, chain

    def poll_records(self) -> SdhRecords:
        """The last push's device records (sdh_engine_poll_records; SDH_FLAG_DEVICE_MATCHES): the
        SdhRecords struct of HBM pointers, formats in include/siddhi_hip.h."""
        r = SdhRecords()
        self._check(self.lib.sdh_engine_poll_records(self.h, ctypes.byref(r)))
        return r

    def records_compact(self, rows_ptr: int = 0, cap: int = 0, width: int = 4) -> int:
        """Decode the K_ratchet part of the last push's device records into compact rows at the device
        pointer rows_ptr (sdh_engine_records_compact); rows_ptr 0: only the row count."""
        n = ctypes.c_int64()
        self._check(self.lib.sdh_engine_records_compact(self.h, rows_ptr or None, int(cap), int(width),
                                                        ctypes.byref(n)))
        return n.value

    def take_matches(self, n_slots_of):
        q, k, ts, off, words = self.poll()
        out = []
        for i in range(len(q)):
            w = words[off[i]:off[i + 1]]
            slots, j = [], 0
            for _ in range(n_slots_of(int(q[i]))):
                c = int(w[j])
                slots.append(tuple(int(x) for x in w[j + 1:j + 1 + c]))
                j += 1 + c
            out.append((int(q[i]), int(k[i]), int(ts[i]), tuple(slots)))
        return out

    def set_strings(self, ids, texts):
        """The String.hashCode and UTF-16 length of each dictionary id's text (sdh_engine_set_strings)."""
        from .planner import java_string_hash
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        h = np.array([java_string_hash(t) for t in texts], dtype=np.int32)
        ln = np.array([len(t.encode("utf-16-le")) // 2 for t in texts], dtype=np.int32)
        self._check(self.lib.sdh_engine_set_strings(self.h, len(ids), ids.ctypes.data, h.ctypes.data, ln.ctypes.data))

    def start(self, t: int):
        """SiddhiAppRuntime.start at time t (absent states schedule their first checks from it)."""
        self._check(self.lib.sdh_engine_start(self.h, int(t)))

    def advance_time(self, t: int):
        """Time passes to t with no event: absent states' schedulers fire what falls due."""
        self._check(self.lib.sdh_engine_advance_time(self.h, int(t)))

    def pending_matches(self) -> int:
        n = ctypes.c_int64()
        self._check(self.lib.sdh_engine_pending_matches(self.h, ctypes.byref(n)))
        return n.value

    def stats(self) -> SdhStats:
        s = SdhStats()
        self._check(self.lib.sdh_engine_stats(self.h, ctypes.byref(s)))
        return s

    def push_stats(self):
        """(last_kernel_ms, last_kernel_bytes) of the last push, with no device work
        (sdh_engine_push_stats: stats() also counts the live partials on the device)."""
        ms, by = ctypes.c_double(), ctypes.c_double()
        self._check(self.lib.sdh_engine_push_stats(self.h, ctypes.byref(ms), ctypes.byref(by)))
        return ms.value, by.value

    def debug_digest(self):
        """(records, order-independent hash) of the last push's K_ratchet records as written, in either
        output mode (sdh_engine_debug_digest)."""
        out = (ctypes.c_uint64 * 2)()
        self._check(self.lib.sdh_engine_debug_digest(self.h, out))
        return int(out[0]), int(out[1])

    def state_bytes(self):
        """(live, reserved, directory) bytes of the sparse K_slab state (sdh_engine_state_bytes)."""
        a, b, c = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.sdh_engine_state_bytes(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    def reserve(self, nbytes: int):
        """Pre-allocate HBM for the sparse K_slab state (sdh_engine_reserve)."""
        self._check(self.lib.sdh_engine_reserve(self.h, int(nbytes)))

    def reserve_keys(self, keys: int):
        """Size the partitioned state for `keys` partition keys now (sdh_engine_reserve_keys)."""
        self._check(self.lib.sdh_engine_reserve_keys(self.h, int(keys)))

    def snapshot(self) -> bytes:
        p = ctypes.c_void_p()
        n = ctypes.c_size_t()
        self._check(self.lib.sdh_engine_snapshot(self.h, ctypes.byref(p), ctypes.byref(n)))
        data = bytes((ctypes.c_char * n.value).from_address(p.value)) if n.value else b""  # (> 2 GiB too)
        self.lib.sdh_free(p)
        return data

    def restore(self, blob: bytes):
        buf = ctypes.create_string_buffer(blob, len(blob))
        self._check(self.lib.sdh_engine_restore(self.h, buf, len(blob)))

    def close(self):
        if getattr(self, "h", None) and self.h:
            self.lib.sdh_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Comm:
    """A communicator of libsiddhi_hip.so (include/siddhi_hip.h sdh_comm_*): RCCL between processes
    (one per GPU), or `world` in-process ranks (Comm.local) for engines driven by one process."""

    def __init__(self, handle: ctypes.c_void_p, rank: int, world: int, group=None):
        self.lib = load_library()
        self.h, self.rank, self.world = handle, rank, world
        self._group = group  # (local ranks share their group; destroyed together)

    @staticmethod
    def unique_id() -> bytes:
        """ncclGetUniqueId on this rank (sdh_comm_get_id): SDH_COMM_ID_BYTES to hand to every rank."""
        lib = load_library()
        buf = ctypes.create_string_buffer(SDH_COMM_ID_BYTES)
        rc = lib.sdh_comm_get_id(buf, SDH_COMM_ID_BYTES)
        if rc != SDH_OK:
            raise EngineError(rc, lib.sdh_comm_last_error().decode())
        return buf.raw

    @classmethod
    def rccl(cls, uid: bytes, rank: int, world: int, device: int = 0) -> "Comm":
        """ncclCommInitRank (collective: every rank calls it with the same id)."""
        lib = load_library()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, len(uid))
        rc = lib.sdh_comm_create(buf, len(uid), rank, world, device, ctypes.byref(h))
        if rc != SDH_OK:
            raise EngineError(rc, lib.sdh_comm_last_error().decode())
        return cls(h, rank, world)

    @classmethod
    def local(cls, world: int, devices: Optional[Sequence[int]] = None) -> List["Comm"]:
        """`world` ranks in this process (sdh_comm_create_local)."""
        lib = load_library()
        hs = (ctypes.c_void_p * world)()
        dv = (ctypes.c_int32 * world)(*(devices or [0] * world))
        rc = lib.sdh_comm_create_local(world, dv, hs)
        if rc != SDH_OK:
            raise EngineError(rc, lib.sdh_comm_last_error().decode())
        group: list = []
        group.extend(cls(ctypes.c_void_p(hs[r]), r, world, group) for r in range(world))
        return group

    def close(self):
        if getattr(self, "h", None) and self.h:
            self.lib.sdh_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def calibrate_hbm(device: int = 0, nbytes: int = 4 << 30, iters: int = 5):
    """(copy GB/s, read GB/s): the measured HBM ceiling (sdh_calibrate_hbm)."""
    lib = load_library()
    c, r = ctypes.c_double(), ctypes.c_double()
    rc = lib.sdh_calibrate_hbm(device, nbytes, iters, ctypes.byref(c), ctypes.byref(r))
    if rc != SDH_OK:
        raise EngineError(rc, "sdh_calibrate_hbm failed")
    return c.value, r.value
