"""Match -> output row projection (the ``QuerySelector`` step).

A match is the tuple the engine returns: output timestamp plus, per state slot, the chain of event
sequence numbers the slot held when the reference would have called
``QuerySelector.process`` (``core/query/selector/QuerySelector.java:76-169``). Output attributes are
evaluated with the same typed bytecode as filters; the selector's default chain index is 0 (the
first event of a count chain, ``SelectorParser.java:193-195``) and ``eK[last]`` is the last one.
Arithmetic follows ``core/executor/math/**`` (binary32 via numpy, null on /0 and %0).
"""
from __future__ import annotations

import math
import struct
from typing import List, Sequence

import numpy as np

from .events import EventLog, StringDictionary, decode_value
from .ir import (AR_ADD, AR_DIV, AR_MOD, AR_MUL, AR_SUB, CMP_EQ, CMP_GE, CMP_GT, CMP_LE, CMP_LT,
                 CMP_NE, OP_AND, OP_ARITH, OP_ATTR, OP_CMP, OP_CONST, OP_IS_NULL, OP_NOT, OP_OR,
                 OP_STREAM_IS_NULL, T_BOOL, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_STRING, Insn)


def _chain_at(chain: Sequence[int], idx: int):
    """StateEvent.getStreamEvent(int[]) on a chain given as a list of event seqs."""
    if not chain:
        return None
    if idx >= 0:
        return chain[idx] if idx < len(chain) else None
    if idx == -1:
        return chain[-1]
    if idx == -2:
        return chain[-2] if len(chain) >= 2 else None
    k = len(chain) + idx
    return chain[k] if k >= 0 else None


def _to_f32(v, t):
    return np.float32(v) if t != T_FLOAT else v


def _cmp(op, a, b):
    return {CMP_EQ: a == b, CMP_NE: a != b, CMP_GT: a > b, CMP_GE: a >= b, CMP_LT: a < b,
            CMP_LE: a <= b}[op]


def typed_compare(op, lv, lt, rv, rt) -> bool:
    if lt in (T_STRING, T_BOOL):
        return (lv == rv) if op == CMP_EQ else (lv != rv)
    if T_DOUBLE in (lt, rt):
        return bool(_cmp(op, float(lv), float(rv)))
    if T_FLOAT in (lt, rt):
        if op in (CMP_EQ, CMP_NE) and T_LONG in (lt, rt):
            return bool(_cmp(op, float(lv), float(rv)))
        return bool(_cmp(op, np.float32(lv), np.float32(rv)))
    return bool(_cmp(op, int(lv), int(rv)))


def _wrap(v, bits):
    m = 1 << bits
    v &= m - 1
    return v - m if v >= (m >> 1) else v


def arith(op, res, lv, rv):
    if lv is None or rv is None:
        return None
    if res in (T_INT, T_LONG):
        bits = 32 if res == T_INT else 64
        a, b = int(lv), int(rv)
        if op == AR_ADD:
            return _wrap(a + b, bits)
        if op == AR_SUB:
            return _wrap(a - b, bits)
        if op == AR_MUL:
            return _wrap(a * b, bits)
        if b == 0:
            return None
        q = abs(a) // abs(b) * (1 if (a >= 0) == (b >= 0) else -1)   # Java truncation
        if op == AR_DIV:
            return _wrap(q, bits)
        return _wrap(a - q * b, bits)
    if res == T_FLOAT:
        a, b = np.float32(lv), np.float32(rv)
        with np.errstate(all="ignore"):
            if op == AR_ADD:
                return np.float32(a + b)
            if op == AR_SUB:
                return np.float32(a - b)
            if op == AR_MUL:
                return np.float32(a * b)
            if b == 0:
                return None
            if op == AR_DIV:
                return np.float32(a / b)
            return np.float32(np.fmod(a, b))
    a, b = float(lv), float(rv)
    if op == AR_ADD:
        return a + b
    if op == AR_SUB:
        return a - b
    if op == AR_MUL:
        return a * b
    if b == 0:
        return None
    if op == AR_DIV:
        try:
            return a / b
        except ZeroDivisionError:
            return None
    return math.fmod(a, b)


def _const(ins: Insn, dictionary: StringDictionary, strings: List[str]):
    t = ins.restype
    if t == T_FLOAT:
        return np.float32(struct.unpack("<f", struct.pack("<I", ins.imm & 0xFFFFFFFF))[0])
    if t == T_DOUBLE:
        return struct.unpack("<d", struct.pack("<q", ins.imm))[0]
    if t == T_BOOL:
        return bool(ins.imm)
    if t == T_STRING:
        return strings[ins.imm]
    return int(ins.imm)


def evaluate(code: List[Insn], slots: Sequence[Sequence[int]], log: EventLog, stream_types,
             dictionary: StringDictionary, strings: List[str]):
    """Evaluate output bytecode over one match. Returns a Python value or None."""
    st = []   # (value, type)
    for ins in code:
        op = ins.op
        if op == OP_CONST:
            st.append((_const(ins, dictionary, strings), ins.restype))
        elif op == OP_ATTR:
            seq = _chain_at(slots[ins.a], ins.b)
            # seq -1: the empty event an absent logical side borrows (StreamEventPool.borrowEvent:
            # every attribute null)
            if seq is None or seq < 0 or log.nulls[seq][ins.imm]:
                st.append((None, ins.restype))
            else:
                st.append((decode_value(int(log.vals[seq][ins.imm]), ins.restype, dictionary), ins.restype))
        elif op == OP_STREAM_IS_NULL:
            st.append((_chain_at(slots[ins.a], ins.b) is None, T_BOOL))
        elif op == OP_IS_NULL:
            v, _ = st.pop()
            st.append((v is None, T_BOOL))
        elif op == OP_NOT:
            v, _ = st.pop()
            st.append((not (v is True), T_BOOL))
        elif op in (OP_AND, OP_OR):
            r, _ = st.pop()
            l, _ = st.pop()
            lb, rb = l is True, r is True
            st.append(((lb and rb) if op == OP_AND else (lb or rb), T_BOOL))
        elif op == OP_CMP:
            r, rt = st.pop()
            l, lt = st.pop()
            st.append((l is not None and r is not None and typed_compare(ins.imm, l, lt, r, rt), T_BOOL))
        elif op == OP_ARITH:
            r, rt = st.pop()
            l, lt = st.pop()
            st.append((arith(ins.imm, ins.restype, l, r), ins.restype))
        else:
            raise ValueError(f"bad opcode {op}")
    v, t = st[-1]
    return v


def project(query_ir, match_slots, log: EventLog, stream_types, dictionary, strings):
    return [evaluate(o.code, match_slots, log, stream_types, dictionary, strings)
            for o in query_ir.outputs]


def stream_rows(ir, matches, log: EventLog, dictionary, strings, stream: str) -> List[list]:
    """Rows arriving on `stream` in delivery order: each match's projected row goes to its query's
    output stream when the match is delivered (R18 order), and through every selector chain reading
    that stream (ir.chains: plain queries over a pattern's inner-stream output, in definition order
    -- the subscription order of StreamJunction.sendEvent:185-205), whose filters and projections see
    the row as a one-event #X stream."""
    from .events import encode_rows
    by_input = {}
    for c in getattr(ir, "chains", []):
        by_input.setdefault(c.input, []).append(c)
    out: List[list] = []

    def deliver(row, types, target):
        if target == stream:
            out.append(row)
        for c in by_input.get(target, []):
            vals, nulls = encode_rows([row], types, dictionary)
            one = EventLog()
            one.append(-1, [0], vals, nulls)
            if not all(evaluate(f, [[0]], one, None, dictionary, strings) is True for f in c.filters):
                continue
            if c.outputs:
                deliver([evaluate(o.code, [[0]], one, None, dictionary, strings) for o in c.outputs],
                        [o.type for o in c.outputs], c.output_stream)
            else:
                deliver(list(row), types, c.output_stream)

    for m in matches:
        q = ir.queries[m[0]]
        deliver(project(q, m[3], log, None, dictionary, strings), [o.type for o in q.outputs], q.output_stream)
    return out
