#!/usr/bin/env python3
"""Transcribe the reference's absent-pattern known-answer tests into JSON fixtures.

Reads the TestNG sources of the absent suites under ``/root/reference`` (at generation time only)
and writes DATA: for every ``@Test`` method, the SiddhiQL app, whether it runs in playback mode, the
callback's ordered expected rows (``TestUtil.addQueryCallback(runtime, name, expected...)``), and the
timeline after ``siddhiAppRuntime.start()``:

* ``send``: an event at the wall-clock time it is sent -- the cumulative ``Thread.sleep`` gaps
  since start (``ts0`` + gaps), or its explicit timestamp in playback apps;
* ``advance``: the end of a sleep (a live runtime's schedulers fire while the test sleeps; in
  playback apps time only moves with events, so no advances are written);
* ``check``: an asserted in-event count at that point of the timeline.

No reference source text is kept: only the queries, the event tuples and the expected outputs.

Usage:  python tests/golden/extract_absent_tests.py   (writes tests/golden/reference_absent_kat.json)
"""
from __future__ import annotations

import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from extract_reference_tests import _concat_value, _methods, _object_array, _split_top, _statement, \
    _strip_comments  # noqa: E402

REF = "/root/reference/modules/siddhi-core/src/test/java/org/wso2/siddhi/core/query"
FILES = [
    "pattern/absent/AbsentPatternTestCase.java",
    "pattern/absent/EveryAbsentPatternTestCase.java",
    "pattern/absent/AbsentWithEveryPatternTestCase.java",
    "pattern/absent/LogicalAbsentPatternTestCase.java",
    "sequence/absent/AbsentSequenceTestCase.java",
    "sequence/absent/EveryAbsentSequenceTestCase.java",
    "sequence/absent/AbsentWithEverySequenceTestCase.java",
    "sequence/absent/LogicalAbsentSequenceTestCase.java",
]
TS0 = 1_500_000_000_000


def _callback(body: str):
    m = re.search(r'TestUtil\.add(Query|Stream)Callback\(\s*\w+\s*,\s*"(\w+)"\s*(,|\))', body)
    if not m:
        return None
    start = m.end(0) - 1
    # the argument list up to the matching ')'
    depth, i = 0, start
    while i < len(body):
        c = body[i]
        if c == '"':
            j = i + 1
            while body[j] != '"':
                j += 2 if body[j] == "\\" else 1
            i = j
        elif c == "(":
            depth += 1
        elif c == ")":
            if depth == 0:
                break
            depth -= 1
        i += 1
    args = body[start + 1:i] if m.group(3) == "," else ""
    rows = []
    for a in _split_top(args):
        am = re.fullmatch(r"new\s+Object\[\]\s*\{(.*)\}", a.strip(), re.S)
        if not am:
            raise ValueError(f"unsupported expected row {a!r}")
        rows.append(_object_array(am.group(1)))
    return {"kind": m.group(1).lower(), "name": m.group(2), "end": m.end(0)}, rows


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
    cb = _callback(body)
    if cb is None:
        return None, "no TestUtil callback"
    cbinfo, rows = cb
    handlers = dict(re.findall(r'InputHandler\s+(\w+)\s*=\s*\w+\.getInputHandler\("(\w+)"\)', body))
    playback = "@app:playback" in app.replace(" ", "")
    st = re.search(r"\w+\.start\(\);", body)
    if not st:
        return None, "runtime never started"
    rest = body[st.end():]
    if re.search(r"\bfor\s*\(|\bwhile\s*\(", rest):
        return None, "loop in the timeline"
    pat = re.compile(
        r'(?P<h>\w+)\.send\((?:(?P<tsv>\w+)\s*,\s*)?new Object\[\]\s*\{(?P<d>.*?)\}\s*\);'
        r'|Thread\.sleep\((?P<sl>\d+)\);'
        r'|long\s+(?P<tv>\w+)\s*=\s*(?:System\.currentTimeMillis\(\)|(?P<tlit>\d+)L?);'
        r'|(?P<ta>\w+)\s*\+=\s*(?P<tn>\d+)\s*;'
        r'|assertEquals\("Number of success events[^"]*",\s*(?P<cnt>\d+)\s*,\s*\w+\.getInEventCount\(\)\)'
        r'|assert(?P<arr>True|False)\("Event (?:not )?arrived",\s*\w+\.isEventArrived\(\)\)'
        r'|\w+\.shutdown\(\);', re.S)
    t = 0            # wall-clock ms since start
    tvars = {}
    actions = []
    count = None
    arrived = None
    for sm in pat.finditer(rest):
        if sm.group(0).endswith(".shutdown();"):
            break
        if sm.group("sl"):
            t += int(sm.group("sl"))
            if not playback:
                actions.append({"advance": TS0 + t})
        elif sm.group("tv"):
            tvars[sm.group("tv")] = int(sm.group("tlit")) if sm.group("tlit") else TS0 + t
        elif sm.group("ta"):
            if sm.group("ta") not in tvars:
                return None, f"unknown time variable {sm.group('ta')}"
            tvars[sm.group("ta")] += int(sm.group("tn"))
        elif sm.group("h"):
            h = sm.group("h")
            if h not in handlers:
                return None, f"unknown handler {h}"
            if sm.group("tsv"):
                if not playback:
                    return None, "explicit timestamps outside playback"
                lit = re.fullmatch(r"(\d+)L?", sm.group("tsv"))
                if lit:
                    ts = int(lit.group(1))
                elif sm.group("tsv") in tvars:
                    ts = tvars[sm.group("tsv")]
                else:
                    return None, f"unknown time variable {sm.group('tsv')}"
            else:
                if playback:
                    return None, "playback send without a timestamp"
                ts = TS0 + t
            actions.append({"send": handlers[h], "data": _object_array(sm.group("d")), "ts": ts})
        elif sm.group("cnt"):
            count = int(sm.group("cnt"))
            actions.append({"check": count})
        elif sm.group("arr"):
            arrived = sm.group("arr") == "True"
    return {"app": app, "playback": playback, "callback": cbinfo["name"], "callback_kind": cbinfo["kind"],
            "expected_rows": rows, "actions": actions, "expected_count": count, "event_arrived": arrived}, None


def main():
    out, skipped = [], []
    for rel in FILES:
        path = os.path.join(REF, rel)
        raw = open(path).read()
        src = _strip_comments(raw)
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
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_absent_kat.json")
    with open(dst, "w") as f:
        json.dump({"generator": "tests/golden/extract_absent_tests.py", "ts0": TS0, "fixtures": out,
                   "skipped": skipped}, f, indent=1)
    print(f"wrote {len(out)} fixtures, skipped {len(skipped)}", file=sys.stderr)
    for s in skipped:
        print("  skip", s, file=sys.stderr)


if __name__ == "__main__":
    main()
