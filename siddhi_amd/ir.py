"""Pattern IR: the processor-graph description shared by every consumer of a compiled app.

The IR is the serialized form of the object graph ``StateInputStreamParser`` builds
(``core/util/parser/StateInputStreamParser.java:77-398``): one pre/post state-processor pair per
state id, their next / next-every / within-every / partner / callback links, the per-stream
receivers with their processor registration order, and the inner-state-runtime tree that drives
``init``/``reset``/``update``.  Filters and selector outputs are typed postfix bytecode.

Binary layout (little-endian int64 words; the C-ABI's specification is ``include/siddhi_hip_ir.h``),
consumed by the engine (``siddhi_amd/csrc/engine.hip`` ``read_ir`` and ``siddhi_amd/csrc/gen_lower.h``
``kg::read_program``) and by the CPU oracle (``oracle/oracle.cpp``)::

    'SDHIR001' version
    n_streams  { n_attrs attr_type* }
    n_strings  { n_bytes bytes(padded to 8) }
    n_queries  { query }
    n_partitions { n_keys { stream_idx n_insn insn* } n_query_idx query_idx* }

    query := type within_ms n_states partition_idx selector_present
             state*            (indexed by state id)
             n_start start_id*
             n_receivers { stream_idx kind n_procs proc_state_id* }
             n_nodes node*     (runtime tree, node 0 is the root)
             n_outputs { n_insn insn* }
    state := kind stream_idx is_start min max logical_type partner next_pre next_every_pre
             within_every_pre callback_pre this_last_post has_selector waiting_ms
             n_filters { n_insn insn* }
             (waiting_ms: the 'for' time of an absent state or absent logical side; -2 for an
              absent logical side without 'for'; -1 otherwise)
    node  := node_type a b pre
    insn  := w0 a b imm     w0 = op | ltype<<8 | rtype<<16 | restype<<24
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import List

MAGIC = b"SDHIR001"
VERSION = 2

# attribute / value types
T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STRING = range(6)
TYPE_CODE = {"int": T_INT, "long": T_LONG, "float": T_FLOAT, "double": T_DOUBLE, "bool": T_BOOL,
             "string": T_STRING}
TYPE_NAME = {v: k for k, v in TYPE_CODE.items()}

# bytecode ops
OP_CONST, OP_ATTR, OP_IS_NULL, OP_STREAM_IS_NULL, OP_CMP, OP_AND, OP_OR, OP_NOT, OP_ARITH = range(1, 10)
CMP_EQ, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE = range(6)
CMP_CODE = {"==": CMP_EQ, "!=": CMP_NE, ">": CMP_GT, ">=": CMP_GE, "<": CMP_LT, "<=": CMP_LE}
AR_ADD, AR_SUB, AR_MUL, AR_DIV, AR_MOD = range(5)
AR_CODE = {"+": AR_ADD, "-": AR_SUB, "*": AR_MUL, "/": AR_DIV, "%": AR_MOD}

# chain index encoding (SiddhiConstants.CURRENT = -1, LAST = -2, deeper = size + idx)
IDX_CURRENT = -1
IDX_LAST = -2

# state kinds / logical types / query types / receivers / runtime nodes
K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT = range(4)  # K_ABSENT: AbsentStreamPre/PostStateProcessor
L_AND, L_OR = range(2)
Q_PATTERN, Q_SEQUENCE = range(2)
R_SINGLE, R_MULTI = range(2)
N_STREAM, N_NEXT, N_EVERY, N_LOGICAL, N_COUNT = range(5)

INT_MAX = 2 ** 31 - 1


@dataclass
class Insn:
    op: int
    ltype: int = 0
    rtype: int = 0
    restype: int = 0
    a: int = 0
    b: int = 0
    imm: int = 0

    def words(self):
        w0 = self.op | (self.ltype << 8) | (self.rtype << 16) | (self.restype << 24)
        return [w0, self.a, self.b, self.imm]


@dataclass
class StateIR:
    kind: int
    stream_idx: int
    is_start: bool
    min: int = 0
    max: int = 0
    logical_type: int = 0
    partner: int = -1
    next_pre: int = -1
    next_every_pre: int = -1
    within_every_pre: int = -1
    callback_pre: int = -1
    this_last_post: int = -1
    has_selector: bool = False
    waiting_ms: int = -1
    filters: List[List[Insn]] = field(default_factory=list)
    alias: str = ""


@dataclass
class ReceiverIR:
    stream_idx: int
    kind: int
    procs: List[int]


@dataclass
class NodeIR:
    type: int
    a: int = -1
    b: int = -1
    pre: int = -1


@dataclass
class OutputIR:
    name: str
    type: int
    code: List[Insn]


@dataclass
class QueryIR:
    name: str
    type: int
    within_ms: int
    states: List[StateIR]
    start_ids: List[int]
    receivers: List[ReceiverIR]
    nodes: List[NodeIR]
    outputs: List[OutputIR]
    partition_idx: int = -1
    output_stream: str = ""


@dataclass
class PartitionKeyIR:
    stream_idx: int
    code: List[Insn]
    type: int


@dataclass
class PartitionIR:
    keys: List[PartitionKeyIR]
    query_idx: List[int]
    # streams its queries read but no key covers: (stream, String.hashCode of the stream id, id
    # length) -- every event reaches every key's instance (the order: PartitionStreamReceiver.send)
    fanout: List[tuple] = field(default_factory=list)


@dataclass
class StreamIR:
    name: str
    attr_names: List[str]
    attr_types: List[int]


@dataclass
class ChainIR:
    """A plain query over a pattern query's inner-stream output (``from #X[f] select ... insert into
    Y`` inside the partition): part of the host selector (selector.stream_rows), not of the device
    program. Its expressions read the one-event row of #X (slot 0)."""
    name: str
    input: str                  # '#X'
    input_types: List[int]      # #X's schema: the producing query's output types
    filters: List[List[Insn]]
    outputs: List[OutputIR]     # empty: select *
    output_stream: str


@dataclass
class ProgramIR:
    name: str
    streams: List[StreamIR]
    strings: List[str]
    queries: List[QueryIR]
    partitions: List[PartitionIR]
    chains: List[ChainIR] = field(default_factory=list)

    def stream_index(self, name: str) -> int:
        for i, s in enumerate(self.streams):
            if s.name == name:
                return i
        raise KeyError(name)

    def query_index(self, name: str) -> int:
        for i, q in enumerate(self.queries):
            if q.name == name:
                return i
        raise KeyError(name)

    # -------------------------------------------------------------------------------------------
    def serialize(self, string_ids=None) -> bytes:
        """``string_ids[k]`` is the dictionary id of program string constant ``k`` (identity if
        omitted); string CONST instructions carry that id so the engine compares ids only."""
        w: List[int] = []
        sid = list(range(len(self.strings))) if string_ids is None else list(string_ids)

        def code(insns):
            w.append(len(insns))
            for ins in insns:
                ws = ins.words()
                if ins.op == OP_CONST and ins.restype == T_STRING:
                    ws[3] = sid[ins.imm]
                w.extend(ws)

        w.append(VERSION)
        w.append(len(self.streams))
        for s in self.streams:
            w.append(len(s.attr_types))
            w.extend(s.attr_types)
        w.append(len(self.strings))
        tail_strings = []
        for st in self.strings:
            b = st.encode("utf-8")
            w.append(len(b))
            pad = b + b"\0" * ((-len(b)) % 8)
            for k in range(0, len(pad), 8):
                w.append(struct.unpack("<q", pad[k:k + 8])[0])
            tail_strings.append(b)
        w.append(len(self.queries))
        for q in self.queries:
            w.extend([q.type, q.within_ms, len(q.states), q.partition_idx, 1 if q.outputs else 0])
            for s in q.states:
                w.extend([s.kind, s.stream_idx, int(s.is_start), s.min, s.max, s.logical_type, s.partner,
                          s.next_pre, s.next_every_pre, s.within_every_pre, s.callback_pre,
                          s.this_last_post, int(s.has_selector), s.waiting_ms, len(s.filters)])
                for f in s.filters:
                    code(f)
            w.append(len(q.start_ids))
            w.extend(q.start_ids)
            w.append(len(q.receivers))
            for r in q.receivers:
                w.extend([r.stream_idx, r.kind, len(r.procs)])
                w.extend(r.procs)
            w.append(len(q.nodes))
            for n in q.nodes:
                w.extend([n.type, n.a, n.b, n.pre])
            w.append(len(q.outputs))
            for o in q.outputs:
                code(o.code)
        w.append(len(self.partitions))
        for p in self.partitions:
            w.append(len(p.keys))
            for k in p.keys:
                w.append(k.stream_idx)
                code(k.code)
            w.append(len(p.query_idx))
            w.extend(p.query_idx)
        # trailer (readers that predate it stop before it): per partition its fan-out streams
        for p in self.partitions:
            w.append(len(p.fanout))
            for f in p.fanout:
                w.extend(f)
        return MAGIC + struct.pack(f"<{len(w)}q", *w)
