#!/usr/bin/env python3
"""Transcribe the reference's pattern/sequence known-answer tests into JSON fixtures.

Reads the TestNG sources under ``/root/reference`` (at generation time only) and writes DATA:
for every ``@Test`` method, the SiddhiQL app, the ordered input events with synthetic timestamps
(the cumulative ``Thread.sleep`` gaps; SURVEY.md §8(c): every in-scope ``within`` test keeps >= 100 ms
of margin), the observed callback, and the hand-asserted expected rows and counts.

No reference source text is kept: only the queries (SiddhiQL strings the tests feed to the
engine), the event tuples and the expected outputs.

Usage:  python tests/golden/extract_reference_tests.py   (writes tests/golden/reference_kat.json)
"""
from __future__ import annotations

import json
import os
import re
import sys

REF = "/root/reference/modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query"
FILES = [
    "pattern/EveryPatternTestCase.java",
    "pattern/WithinPatternTestCase.java",
    "pattern/CountPatternTestCase.java",
    "pattern/LogicalPatternTestCase.java",
    "pattern/ComplexPatternTestCase.java",
    "sequence/SequenceTestCase.java",
    "partition/PatternPartitionTestCase.java",
    "partition/SequencePartitionTestCase.java",
    "IsNullTestCase.java",
]
TS0 = 1_500_000_000_000

_STR_LIT = re.compile(r'"((?:[^"\\]|\\.)*)"')


def _strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", "", src)


def _methods(src: str):
    """Yield (name, start_line, body) for every @Test method."""
    for m in re.finditer(r"@Test[^\n]*\n\s*public void (\w+)\s*\([^)]*\)[^{]*\{", src):
        start = m.end()
        depth, i = 1, start
        while depth and i < len(src):
            c = src[i]
            if c == '"':
                j = i + 1
                while src[j] != '"':
                    j += 2 if src[j] == "\\" else 1
                i = j
            elif c == "{":
                depth += 1
            elif c == "}":
                depth -= 1
            i += 1
        line = src.count("\n", 0, m.start()) + 1
        yield m.group(1), line, src[start:i - 1]


def _concat_value(expr: str, env: dict) -> str:
    out = []
    for part in re.split(r"\+(?=(?:[^\"]*\"[^\"]*\")*[^\"]*$)", expr):
        part = part.strip()
        if not part:
            continue
        if part.startswith('"'):
            out.append("".join(bytes(s, "utf-8").decode("unicode_escape") for s in _STR_LIT.findall(part)))
        elif part in env:
            out.append(env[part])
        else:
            raise ValueError(f"cannot evaluate string part {part!r}")
    return "".join(out)


def _statement(s: str, i: int) -> str:
    """Text from i up to the next ';' outside string literals."""
    j, q = i, False
    while j < len(s):
        c = s[j]
        if c == "\\" and q:
            j += 2
            continue
        if c == '"':
            q = not q
        elif c == ";" and not q:
            return s[i:j].strip()
        j += 1
    raise ValueError("unterminated statement")


def _split_top(s: str):
    parts, depth, cur, q = [], 0, "", False
    i = 0
    while i < len(s):
        c = s[i]
        if c == '"':
            q = not q
        if not q:
            if c in "({[":
                depth += 1
            elif c in ")}]":
                depth -= 1
            elif c == "," and depth == 0:
                parts.append(cur)
                cur = ""
                i += 1
                continue
        cur += c
        i += 1
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts]


def _literal(tok: str) -> str:
    """Java literal -> typed token: s:<str> i:<int> l:<long> f:<float> d:<double> b:<bool> null."""
    tok = tok.strip()
    tok = re.sub(r"^\((int|long|float|double)\)\s*", "", tok)
    if tok == "null":
        return "null"
    if tok.startswith('"'):
        return "s:" + bytes(tok[1:-1], "utf-8").decode("unicode_escape")
    if tok in ("true", "false"):
        return "b:" + tok
    m = re.fullmatch(r"(-?[\d.]+(?:[eE][-+]?\d+)?)([fFdDlL]?)", tok)
    if not m:
        raise ValueError(f"unsupported literal {tok!r}")
    num, suf = m.groups()
    if suf in "fF" and suf:
        return "f:" + num
    if suf in "dD" and suf:
        return "d:" + num
    if suf in "lL" and suf:
        return "l:" + num
    if "." in num or "e" in num.lower():
        return "d:" + num
    return "i:" + num


def _object_array(text: str):
    return [_literal(t) for t in _split_top(text)]


def extract_method(name: str, body: str):
    env = {}
    for m in re.finditer(r"String\s+(\w+)\s*=\s*", body):
        try:
            env[m.group(1)] = _concat_value(_statement(body, m.end()), env)
        except ValueError:
            pass
    m = re.search(r"createSiddhiAppRuntime\(", body)
    if not m:
        return None, "no createSiddhiAppRuntime"
    app = _concat_value(_statement(body, m.end())[:-1], env)
    cbs = re.findall(r'addCallback\("(\w+)",\s*new (QueryCallback|StreamCallback)', body)
    if len(cbs) != 1:
        return None, f"{len(cbs)} callbacks"
    cb_name, cb_kind = cbs[0]
    handlers = dict(re.findall(r'InputHandler\s+(\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body))
    # callback body: the text between addCallback( and the matching '});'
    cb_start = body.index("addCallback(")
    cb_end = body.index("});", cb_start)
    cb_body = body[cb_start:cb_end]
    rest = body[cb_end:]
    # expected rows, in source order, with their case / if-guard
    rows = []
    for am in re.finditer(r"assertArrayEquals\(new Object\[\]\s*\{(.*?)\}\s*,", cb_body, re.S):
        before = cb_body[:am.start()]
        guard = None
        cm = list(re.finditer(r"case\s+(\d+)\s*:", before))
        im = list(re.finditer(r"if\s*\(\s*\w+(?:\.get\(\))?\s*==\s*(\d+)\s*\)", before))
        last_case = cm[-1] if cm else None
        last_if = im[-1] if im else None
        cand = max([x for x in (last_case, last_if) if x is not None], key=lambda x: x.start(),
                   default=None)
        if cand is not None:
            # only count the guard if no 'break;' / closing of the if sits between it and the assert
            seg = before[cand.end():]
            if cand is last_case and "break;" not in seg:
                guard = int(cand.group(1))
            elif cand is last_if and seg.count("}") <= seg.count("{"):
                guard = int(cand.group(1))
        rows.append({"case": guard, "row": _object_array(am.group(1))})
    # actions after the callback: sends and sleeps, in order
    actions = []
    t = 0
    pat = re.compile(r'(\w+)\.send\(new Object\[\]\s*\{(.*?)\}\s*\);|Thread\.sleep\((\d+)\);|'
                     r'\w+\.getInputHandler\("(\w+)"\)\.send\(new Object\[\]\s*\{(.*?)\}\s*\);|'
                     r'for\s*\(int (\w+) = 0; \w+ < (\d+); \w+\+\+\)\s*\{(.*?)\}', re.S)
    for sm in pat.finditer(rest):
        if sm.group(3):
            t += int(sm.group(3))
        elif sm.group(1):
            if sm.group(1) not in handlers:
                return None, f"unknown handler {sm.group(1)}"
            actions.append({"stream": handlers[sm.group(1)], "data": _object_array(sm.group(2)),
                            "ts": TS0 + t})
        elif sm.group(4):
            actions.append({"stream": sm.group(4), "data": _object_array(sm.group(5)), "ts": TS0 + t})
        else:
            return None, "loop in send sequence"
    count = None
    cm = re.search(r'assertEquals\("Number of success events",\s*(\d+)', rest)
    if cm:
        count = int(cm.group(1))
    arrived = None
    am = re.search(r'assertEquals\("Event arrived",\s*(true|false)', rest)
    if am:
        arrived = am.group(1) == "true"
    return {"app": app, "callback": cb_name, "callback_kind": cb_kind, "events": actions,
            "expected_count": count, "expected_rows": rows, "event_arrived": arrived}, None


def main():
    out = []
    skipped = []
    for rel in FILES:
        path = os.path.join(REF, rel)
        src = _strip_comments(open(path).read())
        raw = open(path).read()
        for name, _, body in _methods(src):
            m = re.search(r"public void " + name + r"\s*\(", raw)
            line = raw.count("\n", 0, m.start()) + 1 if m else 0
            try:
                fx, why = extract_method(name, body)
            except Exception as ex:  # noqa: BLE001
                fx, why = None, f"extract error: {ex}"
            tid = f"{os.path.basename(rel)[:-5]}.{name}"
            if fx is None:
                skipped.append((tid, why))
                continue
            fx["id"] = tid
            fx["source"] = f"modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query/{rel}:{line}"
            out.append(fx)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kat.json")
    with open(dst, "w") as f:
        json.dump({"generator": "tests/golden/extract_reference_tests.py", "ts0": TS0,
                   "fixtures": out, "skipped": skipped}, f, indent=1)
    print(f"wrote {len(out)} fixtures, skipped {len(skipped)}", file=sys.stderr)
    for s in skipped:
        print("  skip", s, file=sys.stderr)


if __name__ == "__main__":
    main()
