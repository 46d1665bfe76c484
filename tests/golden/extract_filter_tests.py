#!/usr/bin/env python3
"""Transcribe the reference's predicate known-answer tests (FilterTestCase1/2,
IsNullTestCase) into JSON fixtures for the typed-compare rows A8/A9.

Reads the TestNG sources under ``/root/reference`` (at generation time only) and writes DATA: per
``@Test`` method, the stream definition, the filter condition of the query the callback observes
(SiddhiQL text, or the Java query-builder expression rendered as SiddhiQL), the events sent in
order, and the expected outcome -- the number of output events the test asserts
(``assertEquals(N, count.get())``) or waits for (``waitForEvents(.., N, count, ..)``), or that app
creation must fail (``expectedExceptions = SiddhiAppCreationException``).

A filter query ``from S[cond] select .. insert into O`` emits one event per input event that passes
``cond`` -- the same events as the one-state pattern ``from every e1=S[cond]``, which is how the
tests run them through the NFA engines (tests/test_filter_kat.py).

Skipped (listed in the output with the reason): chained queries (the callback's query reads another
query's output), windows / functions / joins, tests whose callback counts are not a plain
``count.addAndGet(inEvents.length)``, and send loops. BooleanCompareTestCase and
StringCompareTestCase are not transcribed: each of their 60 apps selects attributes the stream
does not define, so they fail creation on the select alone and pin no compare semantics.

Usage:  python tests/golden/extract_filter_tests.py   (writes tests/golden/reference_filter_kat.json)
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from extract_reference_tests import (_concat_value, _literal, _methods, _split_top,  # noqa: E402
                                     _statement, _strip_comments)

REF = "/root/reference/modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query"
FILES = ["FilterTestCase1.java", "FilterTestCase2.java", "IsNullTestCase.java"]

_TYPES = {"STRING": "string", "INT": "int", "LONG": "long", "FLOAT": "float", "DOUBLE": "double",
          "BOOL": "bool"}
_CMP = {"LESS_THAN": "<", "GREATER_THAN": ">", "LESS_THAN_EQUAL": "<=", "GREATER_THAN_EQUAL": ">=",
        "EQUAL": "==", "NOT_EQUAL": "!="}
_ARITH = {"add": "+", "subtract": "-", "multiply": "*", "divide": "/", "mod": "%"}


def _call(text: str):
    """'Expression.compare(a, b, c)' -> ('compare', ['a', 'b', 'c'])."""
    text = text.strip()
    m = re.match(r"Expression\s*\.\s*(\w+)\s*\(", text)
    if not m or not text.endswith(")"):
        raise ValueError(f"not an Expression call: {text[:60]!r}")
    return m.group(1), _split_top(text[m.end():-1])


def java_expr(text: str) -> str:
    """Render a siddhi-query-api Expression builder call as SiddhiQL."""
    name, args = _call(text)
    if name == "variable":
        (v,) = args
        return v.strip().strip('"')
    if name == "value":
        (v,) = args
        tok = _literal(v)
        kind, _, body = tok.partition(":")
        if tok == "null":
            raise ValueError("null literal")
        return {"s": lambda b: "'" + b + "'", "i": str, "l": lambda b: b + "L", "f": lambda b: b + "f",
                "d": lambda b: b + "d", "b": str}[kind](body)
    if name == "compare":
        a, op, b = args
        op = re.sub(r"\s+", "", op)
        opn = op.split(".")[-1]
        return f"({java_expr(a)} {_CMP[opn]} {java_expr(b)})"
    if name in ("and", "or"):
        a, b = args
        return f"({java_expr(a)} {name} {java_expr(b)})"
    if name == "not":
        (a,) = args
        return f"(not {java_expr(a)})"
    if name == "isNull":
        (a,) = args
        return f"({java_expr(a)} is null)"
    if name in _ARITH:
        a, b = args
        return f"({java_expr(a)} {_ARITH[name]} {java_expr(b)})"
    raise ValueError(f"unsupported Expression.{name}")


def _from_query_api(body: str):
    """(define-stream text, stream id, condition) of a query built with the Java query API."""
    defs = {}
    attr = r'attribute\s*\(\s*"(\w+)"\s*,\s*Attribute\s*\.\s*Type\s*\.\s*(\w+)\s*\)'
    for m in re.finditer(r'StreamDefinition\s*\.\s*id\("(\w+)"\)((?:\s*\.\s*' + attr.replace("(\\w+)", "\\w+") + r')+)', body):
        attrs = re.findall(attr, m.group(2))
        defs[m.group(1)] = ", ".join(f"{a} {_TYPES[t]}" for a, t in attrs)
    fm = re.search(r'query\s*\.\s*from\(\s*InputStream\s*\.\s*stream\("(\w+)"\)\s*\.\s*filter\(', body)
    if not fm:
        return None, "no filtered InputStream"
    depth, i = 1, fm.end()
    while depth:
        depth += {"(": 1, ")": -1}.get(body[i], 0)
        i += 1
    cond = java_expr(body[fm.end():i - 1])
    if ".window(" in body or "Expression.function" in body:
        return None, "window / function"
    stream = fm.group(1)
    if stream not in defs:
        return None, "stream not defined by the test"
    return (f"define stream {stream} ({defs[stream]});", stream, cond), None


def _from_siddhiql(app: str, cb_query: str):
    """(define-stream text, stream id, condition) of the callback query of a SiddhiQL app."""
    defs = dict(re.findall(r"define stream (\w+)\s*(\([^)]*\))", app))
    qm = None
    for m in re.finditer(r"@info\(\s*name\s*=\s*'(\w+)'\s*\)\s*from\s+(\w+)\s*\[(.*?)\]\s*(#?)", app, re.S):
        if m.group(1) == cb_query:
            qm = m
    if qm is None:
        return None, "callback query not found / not a plain filter query"
    if qm.group(4):
        return None, "window / stream function"
    stream, cond = qm.group(2), qm.group(3)
    if stream not in defs:
        return None, "chained query (reads another query's output)"
    return (f"define stream {stream} {defs[stream]};", stream, cond.strip()), None


def extract_method(body: str, expects_exception: bool):
    env = {}
    for m in re.finditer(r"String\s+(\w+)\s*=\s*", body):
        try:
            env[m.group(1)] = _concat_value(_statement(body, m.end()), env)
        except ValueError:
            pass
    cbs = re.findall(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)', body)
    if "new Query()" in body:
        parsed, why = _from_query_api(body)
    else:
        m = re.search(r"createSiddhiAppRuntime\(", body)
        if not m:
            return None, "no createSiddhiAppRuntime"
        app = _concat_value(_statement(body, m.end())[:-1], env)
        if expects_exception:
            qm = re.search(r"from\s+(\w+)\s*\[(.*?)\]", app, re.S)
            defs = dict(re.findall(r"define stream (\w+)\s*(\([^)]*\))", app))
            if not qm or qm.group(1) not in defs:
                return None, "no filter query"
            parsed, why = (f"define stream {qm.group(1)} {defs[qm.group(1)]};", qm.group(1),
                           qm.group(2).strip()), None
        else:
            if len(cbs) != 1 or cbs[0][1] != "QueryCallback":
                return None, f"{len(cbs)} callbacks / not a query callback"
            parsed, why = _from_siddhiql(app, cbs[0][0])
    if parsed is None:
        return None, why
    define, stream, cond = parsed
    if expects_exception:
        return {"define": define, "stream": stream, "condition": cond, "expect_creation_error": True}, None
    if len(cbs) != 1 or cbs[0][1] != "QueryCallback":
        return None, "not a single query callback"
    cb_start = body.index("addCallback(")
    cb_end = body.index("});", cb_start)
    cb = body[cb_start:cb_end]
    plain = ("count.addAndGet(inEvents.length)" in cb and len(re.findall(r"count\.\w+\(", cb)) == 1) or \
        (re.search(r"count = count \+ inEvents\.length;", cb) and "count." not in cb)
    if not plain:
        return None, "callback does not count plainly"
    rest = body[cb_end:]
    handlers = dict(re.findall(r'InputHandler\s+(\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body))
    events = []
    for sm in re.finditer(r'(\w+)\.send\(new Object\[\]\s*\{(.*?)\}\s*\);|for\s*\(', rest, re.S):
        if not sm.group(1):
            return None, "loop in send sequence"
        if handlers.get(sm.group(1)) != stream:
            return None, "sends to another stream"
        events.append([_literal(t) for t in _split_top(sm.group(2))])
    exact = re.findall(r"assertEquals\((\d+),\s*count(?:\.get\(\))?\)", rest)
    wait = re.findall(r"waitForEvents\(\s*\d+\s*,\s*(\d+)\s*,\s*count", rest)
    if exact:
        expected, kind = int(exact[-1]), "assertEquals"
    elif wait:
        expected, kind = int(wait[-1]), "waitForEvents"
    else:
        return None, "no count expectation"
    return {"define": define, "stream": stream, "condition": cond, "events": events,
            "expected_count": expected, "expectation": kind}, None


def main():
    out, skipped = [], []
    for rel in FILES:
        path = os.path.join(REF, rel)
        raw = open(path).read()
        src = _strip_comments(raw)
        for name, _, body in _methods(src):
            m = re.search(r"(@Test[^\n]*)\n\s*public void " + name + r"\s*\(", src)
            exc = bool(m and "SiddhiAppCreationException" in m.group(1))
            rm = re.search(r"public void " + name + r"\s*\(", raw)
            line = raw.count("\n", 0, rm.start()) + 1 if rm else 0
            tid = f"{rel[:-5]}.{name}"
            try:
                fx, why = extract_method(body, exc)
            except Exception as ex:  # noqa: BLE001
                fx, why = None, f"extract error: {ex}"
            if fx is None:
                skipped.append((tid, why))
                continue
            fx["id"] = tid
            fx["source"] = f"modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query/{rel}:{line}"
            out.append(fx)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_filter_kat.json")
    with open(dst, "w") as f:
        json.dump({"generator": "tests/golden/extract_filter_tests.py", "fixtures": out, "skipped": skipped},
                  f, indent=1)
    print(f"{len(out)} fixtures, {len(skipped)} skipped -> {dst}")


if __name__ == "__main__":
    main()
