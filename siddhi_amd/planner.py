"""Planner: SiddhiQL AST -> pattern IR.

A restatement of how the reference builds the pattern processor graph, so that every consumer of
the IR (the HIP engine and the CPU oracle) sees the same wiring the Java engine would build:

* state ids in ``SingleInputStreamParser`` registration order; logical element 2 is parsed BEFORE
  element 1 (``StateInputStreamParser.java:161-216,339-351``)                               -- R1
* start states: first element of the chain, inherited by logical sides and every/count wrappers;
  the successor of a Next gets ``false`` (``StateInputStreamParser.java:221-233``)            -- R2
* Next: ``current.last.setNextStatePreProcessor(next.first)`` (``:235-236``), with the logical
  (``LogicalPostStateProcessor.java:134-137``) and count (``CountPostStateProcessor.java:87-95``)
  overrides
* Every: ``last.setNextEveryStatePreProcessor(first)`` and ``withinEveryPreStateProcessor`` on all
  inner pre processors, outer scopes overriding inner ones (``StateInputStreamParser.java:252-278``)
* Count: ``<min:max>`` with ANY -> 0 / ``Integer.MAX_VALUE`` (``:370-393``)
* within: ``startStateIds`` + ``withinTime`` on every pre processor (``:126-138``)
* the query's first pre processor checks the query's LAST post processor for emission
  (``:139-140``), every other pre checks its own post
* selector attachment (``StreamInnerStateRuntime.setQuerySelector``, ``NextInnerStateRuntime``,
  ``LogicalInnerStateRuntime.java:50-53``)
* one receiver per stream id, single vs multi by ``StateInputStream.getStreamCount``
  (``StateInputStreamParser.java:94-113``); processors register in ``init`` order
* partitioned queries are per-key clones; clones do NOT carry ``withinEveryPreStateProcessor``
  (``StreamPreStateProcessor.cloneProperties``, ``StreamPreStateProcessor.java:190-200``)

Predicates lower to typed postfix bytecode following ``ExpressionParser.parseExpression``
(``ExpressionParser.java:231-529``) and ``parseVariable`` (``:1225-1380``).
"""
from __future__ import annotations

import struct
from typing import List, Optional

from . import chm, ql
from .ir import (AR_CODE, CMP_CODE, INT_MAX, K_ABSENT, K_COUNT, K_LOGICAL, K_STREAM, L_AND, L_OR, N_COUNT,
                 N_EVERY, N_LOGICAL, N_NEXT, N_STREAM, OP_AND, OP_ARITH, OP_ATTR, OP_CMP, OP_CONST,
                 OP_IS_NULL, OP_NOT, OP_OR, OP_STREAM_IS_NULL, Q_PATTERN, Q_SEQUENCE, R_MULTI,
                 R_SINGLE, T_BOOL, T_DOUBLE, T_FLOAT, T_INT, T_LONG, T_STRING, TYPE_CODE, Insn,
                 ChainIR, NodeIR, OutputIR, PartitionIR, PartitionKeyIR, ProgramIR, QueryIR, ReceiverIR,
                 StateIR, StreamIR)
from .ql import SiddhiAppCreationException

UNKNOWN_STATE = -1
CURRENT = -1
LAST = -2

_NUMERIC = (T_INT, T_LONG, T_FLOAT, T_DOUBLE)


def _f32_bits(v: float) -> int:
    return struct.unpack("<I", struct.pack("<f", v))[0]


def _f64_bits(v: float) -> int:
    return struct.unpack("<q", struct.pack("<d", v))[0]


class _ExprCompiler:
    """Typed bytecode emission for one expression context (filter of state k, or the selector)."""

    def __init__(self, program: "_ProgramBuilder", meta, current_state: int, default_index: int):
        self.p = program
        self.meta = meta                   # list of (alias, StreamDef) in state-id order
        self.current_state = current_state
        self.default_index = default_index

    def compile(self, e) -> (List[Insn], int):
        code: List[Insn] = []
        t = self._emit(e, code)
        return code, t

    # --------------------------------------------------------------------------------------
    def _emit(self, e, code) -> int:
        if isinstance(e, ql.Const):
            t = TYPE_CODE[e.type]
            if t == T_STRING:
                imm = self.p.intern(e.value)
            elif t == T_FLOAT:
                imm = _f32_bits(e.value)
            elif t == T_DOUBLE:
                imm = _f64_bits(e.value)
            elif t == T_BOOL:
                imm = 1 if e.value else 0
            else:
                imm = int(e.value)
            code.append(Insn(OP_CONST, restype=t, imm=imm))
            return t
        if isinstance(e, ql.Var):
            slot, idx, attr_i, t = self._resolve(e)
            code.append(Insn(OP_ATTR, restype=t, a=slot, b=idx, imm=attr_i))
            return t
        if isinstance(e, ql.StreamIsNull):
            slot, idx = self._resolve_stream(e.stream_ref, e.index)
            code.append(Insn(OP_STREAM_IS_NULL, restype=T_BOOL, a=slot, b=idx))
            return T_BOOL
        if isinstance(e, ql.IsNull):
            self._emit(e.expr, code)
            code.append(Insn(OP_IS_NULL, restype=T_BOOL))
            return T_BOOL
        if isinstance(e, ql.Not):
            t = self._emit(e.expr, code)
            if t != T_BOOL:
                raise SiddhiAppCreationException("'not' needs a BOOL operand")
            code.append(Insn(OP_NOT, restype=T_BOOL))
            return T_BOOL
        if isinstance(e, ql.BinOp):
            if e.op in ("and", "or"):
                lt = self._emit(e.left, code)
                rt = self._emit(e.right, code)
                if lt != T_BOOL or rt != T_BOOL:
                    raise SiddhiAppCreationException(f"'{e.op}' needs BOOL operands")
                code.append(Insn(OP_AND if e.op == "and" else OP_OR, restype=T_BOOL))
                return T_BOOL
            if e.op in CMP_CODE:
                lt = self._emit(e.left, code)
                rt = self._emit(e.right, code)
                self._check_compare(e.op, lt, rt)
                code.append(Insn(OP_CMP, ltype=lt, rtype=rt, restype=T_BOOL, imm=CMP_CODE[e.op]))
                return T_BOOL
            if e.op in AR_CODE:
                lt = self._emit(e.left, code)
                rt = self._emit(e.right, code)
                if lt not in _NUMERIC or rt not in _NUMERIC:
                    # ExpressionParser.parseArithmeticOperationResultType:1389-1407
                    raise SiddhiAppCreationException("Arithmetic operation between non-numeric types")
                if T_DOUBLE in (lt, rt):
                    rtype = T_DOUBLE
                elif T_FLOAT in (lt, rt):
                    rtype = T_FLOAT
                elif T_LONG in (lt, rt):
                    rtype = T_LONG
                else:
                    rtype = T_INT
                code.append(Insn(OP_ARITH, ltype=lt, rtype=rt, restype=rtype, imm=AR_CODE[e.op]))
                return rtype
        raise SiddhiAppCreationException(f"unsupported expression {e!r}")

    @staticmethod
    def _check_compare(op, lt, rt):
        # ExpressionParser.parse*Compare (:539-1220): OperationNotSupportedException cases
        if (lt == T_STRING) != (rt == T_STRING):
            raise SiddhiAppCreationException("string cannot be compared with non-string")
        if (lt == T_BOOL) != (rt == T_BOOL):
            raise SiddhiAppCreationException("bool cannot be compared with non-bool")
        if op not in ("==", "!=") and (lt in (T_STRING, T_BOOL)):
            raise SiddhiAppCreationException("string/bool cannot be used in ordering comparisons")

    def _index(self, var_index, ref, slot) -> int:
        if var_index is None:
            return self.default_index
        if var_index <= LAST:
            # ExpressionParser.java:1341-1346 -- own alias inside own filter keeps [last] unshifted
            cs = self.current_state
            if (cs > -1 and self.meta[cs][0] is not None and ref is not None
                    and ref == self.meta[cs][0]):
                return var_index
            return var_index + 1
        return var_index

    def _resolve_stream(self, ref: str, index):
        for i, (alias, sd) in enumerate(self.meta):
            if (alias is None and sd.name == ref) or (alias is not None and alias == ref):
                return i, self._index(index, ref, i)
        raise SiddhiAppCreationException(f"Stream with reference : {ref} not found")

    def _resolve(self, v: ql.Var):
        if v.stream_ref is None:
            if self.current_state == UNKNOWN_STATE:
                found = None
                for i, (alias, sd) in enumerate(self.meta):
                    ai = sd.index_of(v.attr)
                    if ai >= 0:
                        if found is not None:
                            raise SiddhiAppCreationException(
                                f"attribute '{v.attr}' is ambiguous between input streams")
                        found = (i, ai, sd)
                if found is None:
                    raise SiddhiAppCreationException(f"attribute '{v.attr}' not found")
                i, ai, sd = found
            else:
                i = self.current_state
                sd = self.meta[i][1]
                ai = sd.index_of(v.attr)
                if ai < 0:
                    raise SiddhiAppCreationException(f"No attribute with name '{v.attr}' in {sd.name}")
            idx = self._index(v.index, None, i)
            return i, idx, ai, TYPE_CODE[sd.attrs[ai][1]]
        i, idx = self._resolve_stream(v.stream_ref, v.index)
        sd = self.meta[i][1]
        ai = sd.index_of(v.attr)
        if ai < 0:
            raise SiddhiAppCreationException(f"No attribute with name '{v.attr}' in {sd.name}")
        return i, idx, ai, TYPE_CODE[sd.attrs[ai][1]]


class _ProgramBuilder:
    def __init__(self, app: ql.App):
        self.app = app
        self.streams = []
        self.stream_idx = {}
        for name, sd in app.streams.items():
            self.stream_idx[name] = len(self.streams)
            self.streams.append(StreamIR(name, [a for a, _ in sd.attrs],
                                         [TYPE_CODE[t] if t in TYPE_CODE else -1 for _, t in sd.attrs]))
        self.strings: List[str] = []

    def intern(self, s: str) -> int:
        if s not in self.strings:
            self.strings.append(s)
        return self.strings.index(s)


class _QueryPlanner:
    def __init__(self, pb: _ProgramBuilder, q: ql.Query, partition_idx: int):
        self.pb = pb
        self.q = q
        self.qtype = Q_SEQUENCE if q.input.type == "SEQUENCE" else Q_PATTERN
        self.partitioned = partition_idx >= 0
        self.partition_idx = partition_idx
        self.states: List[StateIR] = []
        self.meta = []
        self.nodes: List[NodeIR] = []

    # -- state helpers (post-processor link setters) -------------------------------------------
    def _set_next_pre(self, post: int, target: int):
        s = self.states[post]
        s.next_pre = target
        if s.kind == K_LOGICAL:                      # LogicalPostStateProcessor.setNextStatePreProcessor
            self.states[s.partner].next_pre = target
        if s.kind == K_COUNT:                        # CountPostStateProcessor.setNextStatePreProcessor
            if s.is_start and self.qtype == Q_SEQUENCE and s.min == 0:
                self.states[target].callback_pre = post   # target pre's own post gets the callback

    def _set_next_every(self, post: int, target: int):
        s = self.states[post]
        s.next_every_pre = target
        if s.kind == K_LOGICAL:                      # LogicalPostStateProcessor.setNextEveryStatePreProcessor
            self.states[s.partner].next_every_pre = target

    def _new_node(self, n: NodeIR) -> int:
        self.nodes.append(n)
        return len(self.nodes) - 1

    # -- recursive parse (StateInputStreamParser.parse) -----------------------------------------
    def _parse_stream(self, se: ql.StreamSE, is_start: bool, kind: int, extra: dict) -> int:
        sd = self.pb.app.streams.get(se.stream)
        if sd is None:
            raise SiddhiAppCreationException(f"Stream '{se.stream}' is not defined")
        sid = len(self.states)
        self.meta.append((se.alias, sd))
        st = StateIR(kind=kind, stream_idx=self.pb.stream_idx[se.stream], is_start=is_start,
                     this_last_post=sid, alias=se.alias or "", **extra)
        self.states.append(st)
        comp = _ExprCompiler(self.pb, self.meta, sid, CURRENT)
        for f in se.filters:
            code, t = comp.compile(f)
            if t != T_BOOL:
                raise SiddhiAppCreationException("filter expression must return BOOL")
            st.filters.append(code)
        return sid

    def parse(self, e, is_start: bool, pres: list):
        """Returns (node, first_pre, last_post)."""
        if isinstance(e, ql.StreamSE):
            sid = self._parse_stream(e, is_start, K_STREAM, {})
            pres.append(sid)
            return self._new_node(NodeIR(N_STREAM, pre=sid)), sid, sid
        if isinstance(e, ql.AbsentSE):
            # AbsentStreamStateElement: a stream state with the absent pre/post pair and its own
            # scheduler (StateInputStreamParser.java:174-200)
            sid = self._parse_stream(e.stream, is_start, K_ABSENT, {"waiting_ms": e.waiting_ms})
            pres.append(sid)
            return self._new_node(NodeIR(N_STREAM, pre=sid)), sid, sid
        if isinstance(e, ql.NextSE):
            n1, f1, l1 = self.parse(e.first, is_start, pres)
            n2, f2, l2 = self.parse(e.next, False, pres)
            self._set_next_pre(l1, f2)
            return self._new_node(NodeIR(N_NEXT, a=n1, b=n2)), f1, l2
        if isinstance(e, ql.EverySE):
            inner_pres = []
            n, f, l = self.parse(e.inner, is_start, inner_pres)
            self._set_next_every(l, f)
            if not self.partitioned:
                for p in inner_pres:
                    self.states[p].within_every_pre = f
            pres.extend(inner_pres)
            return self._new_node(NodeIR(N_EVERY, a=n, pre=f)), f, l
        if isinstance(e, ql.LogicalSE):
            lt = L_AND if e.type == "and" else L_OR

            def side(x):
                # AbsentLogicalPre/PostStateProcessor sides (StateInputStreamParser.java:284-327):
                # waiting_ms -2 encodes a side without 'for' (the reference's waitingTime -1)
                if isinstance(x, ql.AbsentSE):
                    return x.stream, {"logical_type": lt, "waiting_ms": -2 if x.waiting_ms is None else x.waiting_ms}
                return x, {"logical_type": lt}
            st2, ex2 = side(e.s2)
            st1, ex1 = side(e.s1)
            s2 = self._parse_stream(st2, is_start, K_LOGICAL, ex2)
            pres.append(s2)
            s1 = self._parse_stream(st1, is_start, K_LOGICAL, ex1)
            pres.append(s1)
            self.states[s1].partner = s2
            self.states[s2].partner = s1
            n2 = self._new_node(NodeIR(N_STREAM, pre=s2))
            n1 = self._new_node(NodeIR(N_STREAM, pre=s1))
            return self._new_node(NodeIR(N_LOGICAL, a=n1, b=n2)), s1, s2
        if isinstance(e, ql.CountSE):
            mn = 0 if e.min == -1 else e.min
            mx = INT_MAX if e.max == -1 else e.max
            sid = self._parse_stream(e.stream, is_start, K_COUNT, {"min": mn, "max": mx})
            pres.append(sid)
            return self._new_node(NodeIR(N_COUNT, pre=sid)), sid, sid
        raise SiddhiAppCreationException(f"unsupported state element {e!r}")

    def _attach_selector(self, node: int):
        n = self.nodes[node]
        if n.type in (N_STREAM, N_COUNT):
            self.states[n.pre].has_selector = True
        elif n.type == N_NEXT:
            self._attach_selector(n.b)
        elif n.type == N_EVERY:
            self._attach_selector(n.a)
        elif n.type == N_LOGICAL:
            self._attach_selector(n.b)
            self._attach_selector(n.a)

    def build(self) -> QueryIR:
        pres: List[int] = []
        root, first, last = self.parse(self.q.input.element, True, pres)
        # root must be node 0 in the IR: re-index
        order = [root] + [i for i in range(len(self.nodes)) if i != root]
        remap = {old: new for new, old in enumerate(order)}
        nodes = []
        for old in order:
            n = self.nodes[old]
            nodes.append(NodeIR(n.type, remap.get(n.a, -1) if n.a >= 0 else -1,
                                remap.get(n.b, -1) if n.b >= 0 else -1, n.pre))
        self.nodes = nodes
        self._attach_selector(0)
        self.states[first].this_last_post = last
        within = -1 if self.q.input.within_ms is None else self.q.input.within_ms
        start_ids = [p for p in pres if self.states[p].is_start] if within >= 0 else []
        # receivers: one per stream id; processors in init (== state id) order
        by_stream = {}
        for sid, st in enumerate(self.states):
            by_stream.setdefault(st.stream_idx, []).append(sid)
        receivers = [ReceiverIR(si, R_SINGLE if len(ids) == 1 else R_MULTI, ids)
                     for si, ids in by_stream.items()]
        outputs = []
        if self.q.select is not None:
            comp = _ExprCompiler(self.pb, self.meta, UNKNOWN_STATE, 0)   # SelectorParser.java:193-195
            for oa in self.q.select:
                code, t = comp.compile(oa.expr)
                nm = oa.rename
                if nm is None:
                    if isinstance(oa.expr, ql.Var):
                        nm = oa.expr.attr
                    else:
                        raise SiddhiAppCreationException("output attribute needs a name ('as')")
                outputs.append(OutputIR(nm, t, code))
        return QueryIR(name=self.q.name, type=self.qtype, within_ms=within, states=self.states,
                       start_ids=start_ids, receivers=receivers, nodes=self.nodes, outputs=outputs,
                       partition_idx=self.partition_idx, output_stream=self.q.output_stream or "")


# ---- inner streams (`#X`, partition-local) on the pattern path ----------------------------------
# (1) A projection feeding a pattern: `from S[f] select a, b as c insert into #X` with S a partitioned
#     stream, read by pattern states `e=#X[g]`. The inner stream carries exactly the S events that
#     pass f, delivered while the projection query processes them (PartitionRuntime.clonePartition
#     subscribes the local junction #X+key; QueryRuntime -> InsertIntoStreamCallback), so the state is
#     the same state over S with filter f AND g and #X's attribute names mapped back to S's: the fold
#     rewrites the pattern's AST and the device never sees #X. R18 order is unchanged when no other
#     query of the partition reads S (the pattern then receives S events at the projection's place).
# (2) A selector chain over a pattern's output: the pattern inserts its rows into #X and plain
#     queries `from #X[f] select ... insert into Y` re-project them (ChainIR, applied by the host
#     selector in match order: each row passes through the chain when its match is delivered).
def _walk_expr(e, fn):
    e = fn(e)
    if isinstance(e, ql.IsNull):
        return ql.IsNull(_walk_expr(e.expr, fn))
    if isinstance(e, ql.Not):
        return ql.Not(_walk_expr(e.expr, fn))
    if isinstance(e, ql.BinOp):
        return ql.BinOp(e.op, _walk_expr(e.left, fn), _walk_expr(e.right, fn))
    return e


def _fold_projection(q: ql.Query, folds: dict) -> ql.Query:
    """Pattern query q with its states over folded inner streams rewritten onto their source streams."""
    import copy
    q = copy.deepcopy(q)
    alias_map = {}  # alias of a folded state -> {#X attribute: S attribute}

    def amap_of(p):
        if p.select is None:
            return None
        return {(oa.rename or oa.expr.attr): oa.expr.attr for oa in p.select}

    def rename_own(amap):
        def fn(e):
            if isinstance(e, ql.Var) and e.stream_ref is None and amap is not None:
                return ql.Var(None, e.index, amap.get(e.attr, e.attr))
            return e
        return fn

    def fix_stream(se: ql.StreamSE):
        p = folds.get(se.stream)
        if p is None:
            if se.stream.startswith("#"):
                raise SiddhiAppCreationException(f"inner stream '{se.stream}' has no projection to fold")
            return se
        amap = amap_of(p)
        if se.alias is not None:
            alias_map[se.alias] = amap
        own = [_walk_expr(f, rename_own(amap)) for f in se.filters]
        return ql.StreamSE(se.alias, p.stream, list(p.filters) + own)

    def fix_elem(e):
        if isinstance(e, ql.StreamSE):
            return fix_stream(e)
        if isinstance(e, ql.AbsentSE):
            return ql.AbsentSE(fix_stream(e.stream), e.waiting_ms)
        if isinstance(e, ql.NextSE):
            return ql.NextSE(fix_elem(e.first), fix_elem(e.next))
        if isinstance(e, ql.EverySE):
            return ql.EverySE(fix_elem(e.inner))
        if isinstance(e, ql.LogicalSE):
            return ql.LogicalSE(e.type, fix_elem(e.s1), fix_elem(e.s2))
        if isinstance(e, ql.CountSE):
            return ql.CountSE(fix_stream(e.stream), e.min, e.max)
        raise SiddhiAppCreationException(f"unsupported state element {e!r}")

    q.input.element = fix_elem(q.input.element)

    def rename_ref(e):
        if isinstance(e, ql.Var) and e.stream_ref in alias_map and alias_map[e.stream_ref] is not None:
            return ql.Var(e.stream_ref, e.index, alias_map[e.stream_ref].get(e.attr, e.attr))
        return e

    def fix_refs(e):
        if isinstance(e, (ql.StreamSE,)):
            e.filters = [_walk_expr(f, rename_ref) for f in e.filters]
        elif isinstance(e, ql.AbsentSE):
            fix_refs(e.stream)
        elif isinstance(e, ql.NextSE):
            fix_refs(e.first)
            fix_refs(e.next)
        elif isinstance(e, ql.EverySE):
            fix_refs(e.inner)
        elif isinstance(e, ql.LogicalSE):
            fix_refs(e.s1)
            fix_refs(e.s2)
        elif isinstance(e, ql.CountSE):
            fix_refs(e.stream)

    fix_refs(q.input.element)
    if q.select is not None:
        renamed = any(m is not None and any(k != v for k, v in m.items()) for m in alias_map.values())
        for oa in q.select:
            if renamed and any(isinstance(x, ql.Var) and x.stream_ref is None for x in _vars(oa.expr)):
                raise SiddhiAppCreationException("unqualified attribute over a renamed inner stream")
            oa.expr = _walk_expr(oa.expr, rename_ref)
    return q


def _vars(e):
    out = []
    _walk_expr(e, lambda x: (out.append(x), x)[1])
    return out


def _state_streams(e, acc):
    if isinstance(e, ql.StreamSE):
        acc.append(e.stream)
    elif isinstance(e, ql.AbsentSE):
        acc.append(e.stream.stream)
    elif isinstance(e, ql.NextSE):
        _state_streams(e.first, acc)
        _state_streams(e.next, acc)
    elif isinstance(e, ql.EverySE):
        _state_streams(e.inner, acc)
    elif isinstance(e, ql.LogicalSE):
        _state_streams(e.s1, acc)
        _state_streams(e.s2, acc)
    elif isinstance(e, ql.CountSE):
        acc.append(e.stream.stream)
    return acc


def _plan_inner_streams(app: ql.App, part: ql.Partition, part_streams: set):
    """(pattern queries with folded projections, plain chain queries) of one partition."""
    pattern = [q for q in part.queries if isinstance(q, ql.Query)]
    plain = [q for q in part.queries if isinstance(q, ql.PlainQuery)]
    producers = {}
    for q in part.queries:
        if q.output_stream and q.output_stream.startswith("#"):
            producers.setdefault(q.output_stream, []).append(q)
    folds, chains = {}, []
    for p in plain:
        if p.stream.startswith("#"):
            if not all(isinstance(x, ql.Query) for x in producers.get(p.stream, [])) or p.stream not in producers:
                raise SiddhiAppCreationException(f"inner stream '{p.stream}' must be a pattern query's output")
            chains.append(p)
        elif p.output_stream and p.output_stream.startswith("#") and p.stream in part_streams:
            if len(producers[p.output_stream]) != 1:
                raise SiddhiAppCreationException(f"inner stream '{p.output_stream}' has several producers")
            if p.select is not None and not all(isinstance(oa.expr, ql.Var) and oa.expr.stream_ref is None and
                                                oa.expr.index is None for oa in p.select):
                raise SiddhiAppCreationException("only attribute projections feed a pattern through an inner stream")
            folds[p.output_stream] = p
        else:
            raise SiddhiAppCreationException("plain stream queries are outside the accelerated path")
    for x, p in folds.items():
        readers = [q for q in pattern if p.stream in _state_streams(q.input.element, [])]
        readers += [c for c in plain if c is not p and c.stream == p.stream]
        if readers:
            raise SiddhiAppCreationException(f"stream '{p.stream}' feeds a pattern both directly and through '{x}'")
        if any(c.stream == x for c in chains):
            raise SiddhiAppCreationException(f"inner stream '{x}' feeds both a pattern and a plain query")
    return [_fold_projection(q, folds) if folds else q for q in pattern], chains


def _plan_chain(pb: "_ProgramBuilder", c: ql.PlainQuery, src: QueryIR) -> ChainIR:
    """A plain query over the inner stream `src` writes: compiled against #X's schema (src's outputs)."""
    rev = {v: k for k, v in TYPE_CODE.items()}
    sd = ql.StreamDef(c.stream, [(o.name, rev[o.type]) for o in src.outputs])
    comp = _ExprCompiler(pb, [(None, sd)], 0, CURRENT)
    filters = []
    for f in c.filters:
        code, t = comp.compile(f)
        if t != T_BOOL:
            raise SiddhiAppCreationException("filter expression must return BOOL")
        filters.append(code)
    outputs = []
    for oa in c.select or []:
        code, t = comp.compile(oa.expr)
        nm = oa.rename or (oa.expr.attr if isinstance(oa.expr, ql.Var) else None)
        if nm is None:
            raise SiddhiAppCreationException("output attribute needs a name ('as')")
        outputs.append(OutputIR(nm, t, code))
    return ChainIR(c.name, c.stream, [o.type for o in src.outputs], filters, outputs, c.output_stream or "")


def java_string_hash(s: str) -> int:
    """java.lang.String.hashCode over the UTF-16 code units (int32 wrap)."""
    h = 0
    data = s.encode("utf-16-le")
    for k in range(0, len(data), 2):
        h = (31 * h + (data[k] | data[k + 1] << 8)) & 0xFFFFFFFF
    return h - (1 << 32) if h >= 1 << 31 else h


def plan(app: ql.App) -> ProgramIR:
    """Lower a parsed app to the pattern IR."""
    with ql.no_gc():
        return _plan(app)


def _plan(app: ql.App) -> ProgramIR:
    pb = _ProgramBuilder(app)
    queries: List[QueryIR] = []
    partitions: List[PartitionIR] = []
    chains: List[ChainIR] = []
    for kind, obj in app.order:
        if kind == "query":
            if isinstance(obj, ql.PlainQuery):
                raise SiddhiAppCreationException("plain stream queries are outside the accelerated path")
            queries.append(_QueryPlanner(pb, obj, -1).build())
        else:
            pidx = len(partitions)
            keys = []
            part_streams = set()
            for k in obj.keys:
                sd = app.streams.get(k.stream)
                if sd is None:
                    raise SiddhiAppCreationException(f"Stream '{k.stream}' is not defined")
                if not isinstance(k.expr, ql.Var) or k.expr.stream_ref is not None:
                    raise SiddhiAppCreationException(
                        "only value partitions on a plain attribute are on the accelerated path")
                comp = _ExprCompiler(pb, [(None, sd)], 0, CURRENT)
                code, t = comp.compile(k.expr)
                if k.stream in part_streams:
                    raise SiddhiAppCreationException(f"stream '{k.stream}' is keyed twice in one partition")
                keys.append(PartitionKeyIR(pb.stream_idx[k.stream], code, t))
                part_streams.add(k.stream)
            kclass = {("num" if kk.type in (T_INT, T_LONG) else kk.type) for kk in keys}
            if len(kclass) > 1:
                raise SiddhiAppCreationException("mixed-type partition keys are not supported")
            qidx = []
            fanout = []
            pattern_qs, chain_qs = _plan_inner_streams(app, obj, part_streams)
            for q in pattern_qs:
                qp = _QueryPlanner(pb, q, pidx)
                qir = qp.build()
                for st in qir.states:
                    name = pb.streams[st.stream_idx].name
                    if name in part_streams or st.stream_idx in [f[0] for f in fanout]:
                        continue
                    # a stream the partition does not key reaches every key's instance, in the order
                    # of its receiver's ConcurrentHashMap of "streamId + key" junctions
                    # (PartitionStreamReceiver.java:277-281); the engine restates that order over
                    # String.valueOf of the key: int / long / bool text, a string's registered text
                    # hash (sdh_engine_set_strings), Java 8 Float / Double.toString (java_fmt.h)
                    fanout.append((st.stream_idx, java_string_hash(name), len(name)))
                qidx.append(len(queries))
                queries.append(qir)
            for c in chain_qs:
                src = [queries[i] for i in qidx if queries[i].output_stream == c.stream]
                chains.append(_plan_chain(pb, c, src[0]))
                if any([o.type for o in s.outputs] != chains[-1].input_types for s in src[1:]):
                    raise SiddhiAppCreationException(f"producers of '{c.stream}' disagree on its schema")
            # a key's junction holds the clones in PartitionRuntime.metaQueryRuntimeMap order
            # (clonePartition iterates its values(), PartitionRuntime.java:270; addStreamJunction
            # subscribes them in that order, PartitionStreamReceiver.java:300-307): a
            # ConcurrentHashMap keyed by query name (:177), holding every query of the partition
            names = [q.name for q in obj.queries]
            pos = chm.positions([java_string_hash(nm) for nm in names])
            first = {}
            for j, nm in enumerate(names):
                first.setdefault(nm, j)
            qidx.sort(key=lambda i: pos[first[queries[i].name]])
            partitions.append(PartitionIR(keys, qidx, fanout))
    names = [q.name for q in queries]
    if len(set(names)) != len(names):
        raise SiddhiAppCreationException("duplicate query names")
    return ProgramIR(name=app.name, streams=pb.streams, strings=pb.strings, queries=queries,
                     partitions=partitions, chains=chains)


def compile_app(src: str) -> ProgramIR:
    return plan(ql.parse(src))
