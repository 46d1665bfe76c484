"""SiddhiQL subset front end: tokenizer, recursive-descent parser and AST.

Covers the part of the SiddhiQL grammar that feeds the pattern/sequence (NFA) path:

* ``define stream S (a type, ...)``                       -- ``SiddhiQL.g4`` definition_stream
* ``@info(name='q') from <pattern|sequence> [within T] select ... insert into X``
  - pattern chains  ``every? a -> b -> ...``            -- ``SiddhiQL.g4:200-210``
    (``a -> b -> c`` folds LEFT into Next(Next(a,b),c), ``SiddhiQLBaseVisitorImpl.java:789-829``)
  - sequence chains ``every? a, b, c``                    -- ``SiddhiQL.g4:277-330``
    (first element is Next(first, rest), ``SiddhiQLBaseVisitorImpl.java:1126-1143``)
  - count ``<n>``, ``<n:m>``, ``<n:>``, ``<:m>``, ``*``, ``+``, ``?``
    (``SiddhiQLBaseVisitorImpl.java:1068-1089,1368-1400,2424-2439``)
  - logical ``a and b`` / ``a or b``                     -- ``SiddhiQL.g4:232-235``
* expressions with the grammar's precedence (``SiddhiQL.g4`` math_operation: NOT binds tightest,
  then * / %, + -, relational, equality, AND, OR), ``x is null``, ``eK[i].attr``, ``eK[last-k].attr``
* literals: ``20`` INT, ``20L`` LONG, ``20.5``/``20.5d`` DOUBLE, ``20.5f`` FLOAT (``SiddhiQL.g4:715-732``)
* ``partition with (attr of S, ...) begin <queries> end``

* absent states ``not S[..] for T`` (``SiddhiQL.g4:263-268``, ``basic_absent_pattern_source``) in
  pattern and sequence chains, with or without ``every``, and as sides of a logical state
  (``e1=A and not B``, ``not A for T or e2=B``, ...; ``logical_absent_stateful_source``,
  ``SiddhiQL.g4:251-260``)

Windows, joins, functions, group-by and output rate limiting are outside the accelerated path and
raise :class:`SiddhiParserException`.
"""
from __future__ import annotations

import gc
import re
from contextlib import contextmanager
from dataclasses import dataclass, field
from typing import List, Optional, Tuple, Union


class SiddhiParserException(Exception):
    """Raised for syntax the subset parser does not accept (mirrors SiddhiParserException)."""


class SiddhiAppCreationException(Exception):
    """Raised by the planner for semantically invalid apps (mirrors SiddhiAppCreationException)."""


# ----------------------------------------------------------------------------------------------
# AST
# ----------------------------------------------------------------------------------------------
ATTR_TYPES = ("int", "long", "float", "double", "bool", "string", "object")


@dataclass
class StreamDef:
    name: str
    attrs: List[Tuple[str, str]]  # (name, type) with type in ATTR_TYPES

    def index_of(self, attr: str) -> int:
        for i, (n, _) in enumerate(self.attrs):
            if n == attr:
                return i
        return -1


# expressions ---------------------------------------------------------------------------------
@dataclass
class Const:
    type: str          # int/long/float/double/bool/string
    value: object


@dataclass
class Var:
    stream_ref: Optional[str]     # alias (e1) or stream id; None for unqualified
    index: Optional[int]          # None, >=0, or <= -2 (LAST - k), grammar-level (SiddhiConstants.LAST = -2)
    attr: str


@dataclass
class StreamIsNull:
    stream_ref: str
    index: Optional[int]


@dataclass
class IsNull:
    expr: object


@dataclass
class Not:
    expr: object


@dataclass
class BinOp:
    op: str            # 'and','or','==','!=','>','>=','<','<=','+','-','*','/','%'
    left: object
    right: object


# state elements -------------------------------------------------------------------------------
@dataclass
class StreamSE:
    alias: Optional[str]
    stream: str
    filters: List[object] = field(default_factory=list)


@dataclass
class AbsentSE:
    """``not S[..] for T`` (AbsentStreamStateElement; the stream carries no alias). waiting_ms is
    None for a logical side written without 'for' (``e1=A and not B``)."""
    stream: StreamSE
    waiting_ms: Optional[int]


@dataclass
class NextSE:
    first: object
    next: object


@dataclass
class EverySE:
    inner: object


@dataclass
class LogicalSE:
    type: str          # 'and' | 'or'
    s1: StreamSE
    s2: StreamSE


@dataclass
class CountSE:
    stream: StreamSE
    min: int           # -1 = ANY
    max: int           # -1 = ANY


@dataclass
class StateInput:
    type: str          # 'PATTERN' | 'SEQUENCE'
    element: object
    within_ms: Optional[int]


@dataclass
class OutputAttr:
    expr: object
    rename: Optional[str]


@dataclass
class Query:
    name: str
    input: StateInput
    select: Optional[List[OutputAttr]]   # None == select *
    output_stream: Optional[str]
    annotations: dict = field(default_factory=dict)


@dataclass
class PlainQuery:
    """``from S[f] select ... insert into T`` (no state element). Only the inner-stream forms that
    chain to the pattern path are planned (planner.py): a projection feeding a pattern's state
    (folded into the state on the device) and a selector chain over a pattern's inner-stream
    output (host selector, selector.py)."""
    name: str
    stream: str                          # '#X' for an inner stream
    filters: List[object]
    select: Optional[List[OutputAttr]]   # None == select *
    output_stream: Optional[str]
    annotations: dict = field(default_factory=dict)


@dataclass
class PartitionKey:
    expr: object
    stream: str


@dataclass
class Partition:
    keys: List[PartitionKey]
    queries: List[Query]


@dataclass
class App:
    name: str
    streams: dict
    queries: List[Query]              # top-level queries in definition order
    partitions: List[Partition]
    order: List[Tuple[str, object]]   # ('query', Query) / ('partition', Partition) in definition order
    annotations: dict = field(default_factory=dict)


# ----------------------------------------------------------------------------------------------
# Tokenizer
# ----------------------------------------------------------------------------------------------
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[lLfFdD]?)
  | (?P<id>`[A-Za-z_][A-Za-z_0-9]*`|[A-Za-z_][A-Za-z_0-9]*)
  | (?P<op>->|==|!=|>=|<=|[-+*/%<>=(),;:\[\].@#!?])
""", re.VERBOSE | re.DOTALL)

_KEYWORDS = {
    "define", "stream", "from", "select", "insert", "into", "every", "within", "and", "or", "not",
    "is", "null", "true", "false", "as", "partition", "with", "of", "begin", "end", "last",
    "return", "group", "by", "having", "order", "limit", "offset", "output", "for", "current",
    "expired", "all", "events", "in", "join", "on", "unidirectional", "window", "table",
    "delete", "update", "set",
}

_TIME_UNITS = [
    # (regex, millis) matching SiddhiQL.g4:829-836 and Expression.Time
    (re.compile(r"^years?$", re.I), 365 * 24 * 3600 * 1000),
    (re.compile(r"^months?$", re.I), 30 * 24 * 3600 * 1000),
    (re.compile(r"^weeks?$", re.I), 7 * 24 * 3600 * 1000),
    (re.compile(r"^days?$", re.I), 24 * 3600 * 1000),
    (re.compile(r"^hours?$", re.I), 3600 * 1000),
    (re.compile(r"^min(utes?)?$", re.I), 60 * 1000),
    (re.compile(r"^sec(onds?)?$", re.I), 1000),
    (re.compile(r"^millisec(onds?)?$", re.I), 1),
]


@dataclass(slots=True)
class Tok:
    kind: str   # 'id','kw','num','str','op','eof'
    text: str
    pos: int


def tokenize(src: str) -> List[Tok]:
    toks: List[Tok] = []
    add = toks.append
    kws = _KEYWORDS
    i = 0
    for m in _TOKEN_RE.finditer(src):
        if m.start() != i:  # finditer skipped a character no token matches
            break
        i = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        text = m.group(kind)
        if kind == "id":
            if text[0] == "`":
                add(Tok("id", text[1:-1], m.start()))
            else:
                low = text.lower()
                add(Tok("kw", low, m.start()) if low in kws else Tok("id", text, m.start()))
        elif kind == "str":
            add(Tok("str", text[1:-1], m.start()))
        else:
            add(Tok(kind, text, m.start()))
    if i < len(src):
        raise SiddhiParserException(f"unexpected character {src[i]!r} at {i}")
    toks.append(Tok("eof", "", len(src)))
    return toks


def _time_unit_ms(word: str) -> Optional[int]:
    for rx, ms in _TIME_UNITS:
        if rx.match(word):
            return ms
    return None


# ----------------------------------------------------------------------------------------------
# Parser
# ----------------------------------------------------------------------------------------------
class Parser:
    def __init__(self, src: str):
        self.toks = tokenize(src)
        self._n = len(self.toks)
        self.i = 0
        self.query_counter = 0

    # token helpers -------------------------------------------------------------------------
    def peek(self, k: int = 0) -> Tok:
        j = self.i + k
        return self.toks[j] if j < self._n else self.toks[-1]

    def at(self, text: str, k: int = 0) -> bool:
        j = self.i + k
        t = self.toks[j] if j < self._n else self.toks[-1]
        return t.text == text and (t.kind == "op" or t.kind == "kw")

    def accept(self, text: str) -> bool:
        if self.at(text):
            self.i += 1
            return True
        return False

    def expect(self, text: str) -> Tok:
        if not self.at(text):
            t = self.peek()
            raise SiddhiParserException(f"expected {text!r} at {t.pos}, found {t.text!r}")
        t = self.peek()
        self.i += 1
        return t

    def name(self) -> str:
        t = self.peek()
        if t.kind == "id" or (t.kind == "kw" and t.text not in ("from", "select", "insert", "every",
                                                                  "within", "and", "or", "not")):
            self.i += 1
            return t.text
        raise SiddhiParserException(f"expected a name at {t.pos}, found {t.text!r}")

    def error(self, msg: str):
        raise SiddhiParserException(f"{msg} at {self.peek().pos}")

    # app -------------------------------------------------------------------------------------
    def parse_app(self) -> App:
        streams = {}
        queries: List[Query] = []
        partitions: List[Partition] = []
        order = []
        app_ann = {}
        while self.peek().kind != "eof":
            if self.accept(";"):
                continue
            anns = self.annotations()
            if self.at("define"):
                self.i += 1
                if not self.accept("stream"):
                    self.error("only 'define stream' is supported on this path")
                sd = self.stream_def()
                streams[sd.name] = sd
                app_ann.update({k: v for k, v in anns.items() if k.startswith("app:")})
            elif self.at("from"):
                q = self.query(anns)
                queries.append(q)
                order.append(("query", q))
            elif self.at("partition"):
                p = self.partition()
                partitions.append(p)
                order.append(("partition", p))
            elif anns:
                app_ann.update(anns)
            else:
                self.error(f"unexpected token {self.peek().text!r}")
        name = app_ann.get("app:name", "SiddhiApp")
        return App(name=name, streams=streams, queries=queries, partitions=partitions, order=order,
                   annotations=app_ann)

    def annotations(self) -> dict:
        out = {}
        while self.at("@"):
            self.i += 1
            nm = self.name()
            if self.accept(":"):
                nm = nm + ":" + self.name()
            nm = nm.lower()
            vals = []
            if self.accept("("):
                while not self.at(")"):
                    if self.peek().kind in ("id", "kw") and (self.at("=", 1) or self.at(".", 1)):
                        key = self.name()
                        while self.accept("."):  # dotted element keys (idle.time = '...')
                            key += "." + self.name()
                        self.expect("=")
                        vals.append((key.lower(), self.literal_text()))
                    else:
                        vals.append((None, self.literal_text()))
                    if not self.accept(","):
                        break
                self.expect(")")
            if nm == "info":
                for k, v in vals:
                    if k == "name":
                        out["info.name"] = v
            elif vals:
                out[nm] = vals[0][1]
            else:
                out[nm] = True
        return out

    def literal_text(self) -> str:
        t = self.peek()
        if t.kind in ("str", "num", "id", "kw"):
            self.i += 1
            return t.text
        self.error("expected an annotation value")

    def stream_def(self) -> StreamDef:
        nm = self.name()
        self.expect("(")
        attrs = []
        while True:
            an = self.name()
            ty = self.name().lower()
            if ty not in ATTR_TYPES:
                self.error(f"unknown attribute type {ty}")
            attrs.append((an, ty))
            if not self.accept(","):
                break
        self.expect(")")
        return StreamDef(nm, attrs)

    def partition(self) -> Partition:
        self.expect("partition")
        self.expect("with")
        self.expect("(")
        keys = []
        while True:
            e = self.expression()
            self.expect("of")
            s = self.name()
            keys.append(PartitionKey(e, s))
            if not self.accept(","):
                break
        self.expect(")")
        self.expect("begin")
        qs = []
        while not self.at("end"):
            if self.accept(";"):
                continue
            anns = self.annotations()
            qs.append(self.query(anns))
        self.expect("end")
        return Partition(keys, qs)

    # query -----------------------------------------------------------------------------------
    def query(self, anns: dict):
        self.expect("from")
        start = self.i
        plain = self._plain_source()
        if plain is not None:
            return self._plain_query(anns, plain)
        self.i = start
        inp = self.state_input()
        select = None
        if self.accept("select"):
            if self.accept("*"):
                select = None
            else:
                select = []
                while True:
                    e = self.expression()
                    rn = None
                    if self.accept("as"):
                        rn = self.name()
                    select.append(OutputAttr(e, rn))
                    if not self.accept(","):
                        break
            for kw in ("group", "having", "order", "limit", "offset"):
                if self.at(kw):
                    self.error(f"'{kw}' in pattern queries is outside the accelerated path")
        if self.at("output"):
            self.error("output rate limiting is outside the accelerated path")
        out = None
        if self.accept("insert"):
            if self.accept("all") or self.accept("expired") or self.accept("current"):
                self.expect("events")
            elif self.accept("events"):
                pass
            self.expect("into")
            if self.accept("#"):
                out = "#" + self.name()
            else:
                out = self.name()
        elif self.accept("return"):
            pass
        else:
            self.error("expected 'insert into' or 'return'")
        self.query_counter += 1
        name = anns.get("info.name") or f"query_{self.query_counter}"
        return Query(name=name, input=inp, select=select, output_stream=out, annotations=anns)

    def _plain_source(self):
        """A plain stream source (no alias, no state operator), or None."""
        if self.peek().kind in ("id", "kw") and self.at("=", 1):
            return None
        if self.at("every") or self.at("not") or self.at("("):
            return None
        try:
            se = self.std_source()
        except SiddhiParserException:
            return None
        if not (self.at("select") or self.at("insert") or self.at("return")):
            return None
        return se

    def _plain_query(self, anns: dict, se) -> "PlainQuery":
        select = None
        if self.accept("select"):
            if not self.accept("*"):
                select = []
                while True:
                    e = self.expression()
                    rn = self.name() if self.accept("as") else None
                    select.append(OutputAttr(e, rn))
                    if not self.accept(","):
                        break
            for kw in ("group", "having", "order", "limit", "offset"):
                if self.at(kw):
                    self.error(f"'{kw}' is outside the accelerated path")
        if self.at("output"):
            self.error("output rate limiting is outside the accelerated path")
        out = None
        if self.accept("insert"):
            if self.accept("all") or self.accept("expired") or self.accept("current"):
                self.expect("events")
            self.expect("into")
            out = ("#" + self.name()) if self.accept("#") else self.name()
        elif not self.accept("return"):
            self.error("expected 'insert into' or 'return'")
        self.query_counter += 1
        name = anns.get("info.name") or f"query_{self.query_counter}"
        return PlainQuery(name=name, stream=se.stream, filters=se.filters, select=select, output_stream=out,
                          annotations=anns)

    def state_input(self) -> StateInput:
        start = self.i
        # try pattern first; sequences use ',' as the separator
        elem, seps = self.chain(top=True)
        if "," in seps and "->" in seps:
            self.error("mixing '->' and ',' in one state chain")
        within = None
        if self.accept("within"):
            within = self.time_value()
        if "," in seps:
            return StateInput("SEQUENCE", elem, within)
        if "->" not in seps and not self._has_state_marker(elem):
            self.i = start
            self.error("plain (non-pattern) stream queries are outside the accelerated path")
        return StateInput("PATTERN", elem, within)

    @staticmethod
    def _has_state_marker(elem) -> bool:
        if isinstance(elem, StreamSE):
            return elem.alias is not None
        return True

    def time_value(self) -> int:
        total = 0
        got = False
        while self.peek().kind == "num" and re.fullmatch(r"\d+", self.peek().text):
            t = self.peek(1)
            ms = _time_unit_ms(t.text) if t.kind in ("id", "kw") else None
            if ms is None:
                break
            total += int(self.peek().text) * ms
            self.i += 2
            got = True
        if not got:
            self.error("expected a time value")
        return total

    # state chains ----------------------------------------------------------------------------
    def chain(self, top: bool = False):
        """Parse ``term (sep term)*``. Pattern '->' folds left; sequences follow
        every_sequence_source_chain: Next(first, left-fold(rest))."""
        seps = []
        terms = [self.chain_term()]
        while self.at("->") or self.at(","):
            seps.append(self.peek().text)
            self.i += 1
            terms.append(self.chain_term())
        if not terms:
            self.error("empty state chain")
        if "," in seps and top:
            # SiddhiQLBaseVisitorImpl.visitEvery_sequence_source_chain: Next(first, chain(rest))
            if len(terms) == 1:
                return terms[0], seps
            rest = terms[1]
            for t in terms[2:]:
                rest = NextSE(rest, t)
            return NextSE(terms[0], rest), seps
        elem = terms[0]
        for t in terms[1:]:
            elem = NextSE(elem, t)
        return elem, seps

    def chain_term(self):
        if self.accept("every"):
            if self.at("("):
                self.i += 1
                inner, seps = self.chain()
                self.expect(")")
                if "," in seps:
                    self.error("'every' over a parenthesised sequence chain is not valid SiddhiQL")
                return EverySE(inner)
            if self.at("not"):
                return EverySE(self.absent())
            return EverySE(self.source())
        if self.at("("):
            self.i += 1
            inner, seps = self.chain()
            self.expect(")")
            return inner
        if self.at("not"):
            return self.absent()
        return self.source()

    def absent_side(self, need_for: bool):
        """NOT basic_source [for_time] (SiddhiQL.g4:253-268)."""
        self.expect("not")
        s = self.std_source()
        if s.alias is not None:
            self.error("an absent stream ('not S') cannot carry an alias")
        w = None
        if self.accept("for"):
            w = self.time_value()
        elif need_for:
            self.error("an absent stream needs a 'for' waiting time")
        return AbsentSE(s, w)

    def absent(self):
        """basic_absent_pattern_source, or a logical_absent_stateful_source starting with one."""
        a = self.absent_side(need_for=False)
        if self.at("and") or self.at("or"):
            ty = self.peek().text
            self.i += 1
            if ty == "or" and a.waiting_ms is None:
                self.error("'not A or B' needs a 'for' time on the absent side")
            # NOT basic_source AND standard | basic_absent AND|OR standard | basic_absent AND|OR basic_absent
            if self.at("not"):
                if a.waiting_ms is None:
                    self.error("'not A and not B' needs 'for' times")
                s2 = self.absent_side(need_for=True)
            else:
                s2 = self.std_source()
            return LogicalSE(ty, a, s2)
        if a.waiting_ms is None:
            self.error("an absent stream needs a 'for' waiting time")
        return a

    def source(self):
        s1 = self.std_source()
        if self.at("and") or self.at("or"):
            ty = self.peek().text
            self.i += 1
            if self.at("not"):  # standard AND NOT basic_source [for T] | standard OR basic_absent
                s2 = self.absent_side(need_for=(ty == "or"))
                # the visitor puts the absent side first (State.logicalNotAnd / logicalOr(absent,
                # present): SiddhiQLBaseVisitorImpl.visitLogical_absent_stateful_source:975-1017)
                return LogicalSE(ty, s2, s1)
            s2 = self.std_source()
            return LogicalSE(ty, s1, s2)
        # count / kleene
        if self.at("<"):
            self.i += 1
            mn, mx = -1, -1
            if self.accept(":"):
                mx = self.int_lit()
            else:
                a = self.int_lit()
                if self.accept(":"):
                    mn = a
                    if self.peek().kind == "num":
                        mx = self.int_lit()
                else:
                    mn = mx = a
            self.expect(">")
            return CountSE(s1, mn, mx)
        if self.at("*"):
            self.i += 1
            return CountSE(s1, 0, -1)
        if self.at("+"):
            self.i += 1
            return CountSE(s1, 1, -1)
        if self.at("?"):
            self.i += 1
            return CountSE(s1, 0, 1)
        return s1

    def int_lit(self) -> int:
        t = self.peek()
        if t.kind != "num" or not re.fullmatch(r"\d+", t.text):
            self.error("expected an integer")
        self.i += 1
        return int(t.text)

    def std_source(self) -> StreamSE:
        alias = None
        if self.peek().kind in ("id", "kw") and self.at("=", 1):
            alias = self.name()
            self.expect("=")
        stream = ("#" + self.name()) if self.accept("#") else self.name()
        filters = []
        while self.at("[") or self.at("#"):
            if self.at("#"):
                self.error("stream functions / windows are outside the accelerated path")
            self.expect("[")
            filters.append(self.expression())
            self.expect("]")
        return StreamSE(alias, stream, filters)

    # expressions -----------------------------------------------------------------------------
    def expression(self):
        return self.or_expr()

    def or_expr(self):
        e = self.and_expr()
        while self.accept("or"):
            e = BinOp("or", e, self.and_expr())
        return e

    def and_expr(self):
        e = self.eq_expr()
        while self.accept("and"):
            e = BinOp("and", e, self.eq_expr())
        return e

    def eq_expr(self):
        e = self.rel_expr()
        while self.at("==") or self.at("!="):
            op = self.peek().text
            self.i += 1
            e = BinOp(op, e, self.rel_expr())
        if self.at("in"):
            self.error("'in <table>' is outside the accelerated path")
        return e

    def rel_expr(self):
        e = self.add_expr()
        while self.at(">=") or self.at("<=") or self.at(">") or self.at("<"):
            op = self.peek().text
            self.i += 1
            e = BinOp(op, e, self.add_expr())
        return e

    def add_expr(self):
        e = self.mul_expr()
        while self.at("+") or self.at("-"):
            op = self.peek().text
            self.i += 1
            e = BinOp(op, e, self.mul_expr())
        return e

    def mul_expr(self):
        e = self.unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = self.peek().text
            self.i += 1
            e = BinOp(op, e, self.unary())
        return e

    def unary(self):
        if self.accept("not"):
            return Not(self.unary())
        return self.primary()

    def primary(self):
        t = self.peek()
        if self.accept("("):
            e = self.expression()
            self.expect(")")
            return self._maybe_is_null(e)
        if t.kind == "kw" and t.text in ("true", "false"):
            self.i += 1
            return Const("bool", t.text == "true")
        if t.kind == "str":
            self.i += 1
            return Const("string", t.text)
        if t.kind == "num" or ((self.at("-") or self.at("+")) and self.peek(1).kind == "num"):
            return self.number()
        if t.kind in ("id", "kw"):
            if self.at("(", 1):
                self.error("functions are outside the accelerated path")
            return self._maybe_is_null(self.attribute_or_stream_ref())
        self.error(f"unexpected token {t.text!r} in expression")

    def _maybe_is_null(self, e):
        if self.at("is"):
            self.i += 1
            self.expect("null")
            if isinstance(e, StreamIsNull):
                return e
            return IsNull(e)
        if isinstance(e, StreamIsNull):
            # a bare stream reference that is not followed by 'is null' is an attribute name
            return Var(None, None, e.stream_ref) if e.index is None else self.error("bad reference")
        return e

    def attribute_or_stream_ref(self):
        n1 = self.name()
        idx = None
        if self.at("["):
            self.i += 1
            idx = self.attribute_index()
            self.expect("]")
        if self.accept("."):
            attr = self.name()
            return Var(n1, idx, attr)
        # stream_reference (only meaningful before 'is null') or attribute_name
        if self.at("is"):
            return StreamIsNull(n1, idx)
        if idx is not None:
            self.error("indexed reference without attribute")
        return Var(None, None, n1)

    def attribute_index(self) -> int:
        if self.accept("last"):
            idx = -2                      # SiddhiConstants.LAST
            if self.accept("-"):
                idx -= self.int_lit()     # SiddhiQLBaseVisitorImpl.visitAttribute_index:2338-2349
            return idx
        return self.int_lit()

    def number(self):
        neg = False
        if self.accept("-"):
            neg = True
        else:
            self.accept("+")
        t = self.peek()
        self.i += 1
        txt = t.text
        suf = txt[-1].lower()
        sign = -1 if neg else 1
        if suf == "l":
            return Const("long", sign * int(txt[:-1]))
        if suf == "f":
            return Const("float", sign * float(txt[:-1]))
        if suf == "d":
            return Const("double", sign * float(txt[:-1]))
        if re.fullmatch(r"\d+", txt):
            v = sign * int(txt)
            if not (-2 ** 31 <= v < 2 ** 31):
                raise SiddhiParserException(f"int literal {txt} out of range")
            return Const("int", v)
        return Const("double", sign * float(txt))


@contextmanager
def no_gc():
    """Parsing and planning build millions of small acyclic objects for a 100K-pattern app (C5): the
    cyclic collector's passes over them are pure overhead there."""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def parse(src: str) -> App:
    """Parse a SiddhiQL app string (``SiddhiCompiler.parse`` equivalent for the subset)."""
    with no_gc():
        return Parser(src).parse_app()
