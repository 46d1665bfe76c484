"""Seeded random SiddhiQL pattern/sequence apps over two small streams, for differential tests of
the device engines against the CPU oracle (count, logical and/or, every scopes, within, sequences,
partitions, cross-references, arithmetic, nulls)."""
import random

import numpy as np

STREAMS = ("define stream A (k int, v int, p float, s string); "
           "define stream B (k int, v int, p float, s string);")
ATTRS = [("v", "int"), ("p", "float")]


def _pred(rng, prev_aliases, stream):
    a, _ = rng.choice(ATTRS)
    op = rng.choice([">", "<", ">=", "<=", "==", "!="])
    r = rng.random()
    if prev_aliases and r < 0.45:
        al = rng.choice(prev_aliases)
        b, _ = rng.choice(ATTRS)
        idx = rng.choice(["", "", "[0]", "[last]"]) if al.endswith("c") else ""
        rhs = f"{al}{idx}.{b}"
        if rng.random() < 0.2:
            rhs = f"{rhs} + {rng.randint(1, 3)}"
        return f"{a} {op} {rhs}"
    if r < 0.55:
        return f"s == '{rng.choice('xyz')}'"
    c = rng.randint(0, 9)
    if a == "p":
        c = f"{c}.5" if rng.random() < 0.5 else str(c)
    return f"{a} {op} {c}"


def random_query(rng, name, seq=False):
    n = rng.randint(2, 4)
    parts, aliases = [], []
    for i in range(n):
        st = rng.choice("AB")
        al = f"e{i}"
        kind = rng.random()
        if kind < 0.2 and not seq and i > 0:
            al2 = f"e{i}x"
            st2 = rng.choice("AB")
            p1 = _pred(rng, aliases, st)
            p2 = _pred(rng, aliases, st2)
            parts.append(f"{al}={st}[{p1}] {rng.choice(['and', 'or'])} {al2}={st2}[{p2}]")
            aliases += [al, al2]
            continue
        pred = _pred(rng, aliases, st)
        cnt = ""
        if kind > 0.75:
            mn = rng.randint(0 if seq else 1, 2)
            mx = mn + rng.randint(0, 2)
            cnt = rng.choice([f"<{mn}:{mx}>", f"<{mx}>", f"<{mn}:>"]) if not seq else rng.choice(["+", "*", "?"])
            al = al + "c"
        parts.append(f"{al}={st}[{pred}]{cnt}")
        aliases.append(al)
    if rng.random() < 0.6:
        parts[0] = "every " + parts[0] if rng.random() < 0.7 else "every (" + parts[0] + ")"
    sep = ", " if seq else " -> "
    # `every` without `within` piles up partials without bound: keep those runs short-lived
    has_every = parts[0].startswith("every")
    within = f" within {rng.choice([5, 20, 60])} milliseconds" if (has_every or rng.random() < 0.5) else ""
    sel_al = aliases[-1].rstrip("x")
    return (f"@info(name='{name}') from {sep.join(parts)}{within} "
            f"select {aliases[0]}.v as a, {sel_al}.v as b insert into Out;")


def random_app(seed, n_queries=4, partition=False):
    rng = random.Random(seed)
    qs = [STREAMS]
    body = [random_query(rng, f"q{i}", seq=rng.random() < 0.35) for i in range(n_queries)]
    if partition:
        np_ = rng.randint(1, n_queries)
        qs.append("partition with (k of A, k of B) begin " + " ".join(body[:np_]) + " end;")
        qs += body[np_:]
    else:
        qs += body
    return " ".join(qs)


def random_events(seed, n=300, keys=3):
    rng = np.random.default_rng(seed)
    ev = []
    t = 0
    for _ in range(n):
        t += int(rng.integers(0, 4))
        row = [int(rng.integers(0, keys)), int(rng.integers(0, 10)),
               float(np.float32(rng.integers(0, 20) / 2.0)), str(rng.choice(list("xyz")))]
        if rng.random() < 0.03:
            row[int(rng.integers(1, 4))] = None
        ev.append(("A" if rng.random() < 0.55 else "B", row, t))
    return ev


def random_seq_app(seed):
    """Unpartitioned every-start sequences of 2-4 stream states over A and B (cross-references,
    arithmetic, strings, nulls; some with `within`)."""
    rng = random.Random(seed)
    qs = [STREAMS]
    for qn in range(6):
        n = rng.randint(2, 4)
        parts, al = [], []
        for i in range(n):
            st = rng.choice("AB") if seed % 2 else "A"
            parts.append(f"e{i}={st}[{_pred(rng, al, st)}]")
            al.append(f"e{i}")
        parts[0] = "every " + parts[0]
        w = f" within {rng.choice([3, 10, 40])} milliseconds" if rng.random() < 0.5 else ""
        qs.append(f"@info(name='s{qn}') from {', '.join(parts)}{w} select e0.v as a, e{n - 1}.v as b insert into O;")
    return " ".join(qs)


def random_absent_app(seed, n_queries=4, partition=False):
    """Patterns / sequences of 2-4 states with absent states (`not S[..] for T`, maybe under
    `every`) at any position and absent logical sides, over A and B (cross-references into earlier
    states, within); `partition`: some of them inside `partition with (k of A, k of B)`."""
    rng = random.Random(seed)
    qs = [STREAMS]
    body = []
    for qn in range(n_queries):
        seq = rng.random() < 0.35
        n = rng.randint(2, 4)
        parts, aliases = [], []
        absent_at = rng.randrange(n)
        for i in range(n):
            st = rng.choice("AB")
            pred = _pred(rng, aliases, st)
            r = rng.random()
            if r < 0.25 and i != absent_at:  # a logical state with an absent side
                al = f"e{i}"
                st2 = rng.choice("AB")
                ab = f"not {st2}[{_pred(rng, aliases, st2)}]"
                ty = rng.choice(["and", "or"])
                if ty == "or" or rng.random() < 0.6:
                    ab += f" for {rng.randint(2, 12)} milliseconds"
                pres = f"{al}={st}[{pred}]"
                parts.append(f"{pres} {ty} {ab}" if rng.random() < 0.5 else f"{ab} {ty} {pres}")
                aliases.append(al)
                continue
            if i == absent_at or (i > 0 and rng.random() < 0.15):
                ab = f"not {st}[{pred}] for {rng.randint(2, 12)} milliseconds"
                if rng.random() < 0.3 and (not seq or i == 0):  # sequences: `every` only at the start
                    ab = "every " + ab
                parts.append(ab)
                continue
            al = f"e{i}"
            parts.append(f"{al}={st}[{pred}]")
            aliases.append(al)
        if not aliases:  # the selector needs a stream state
            parts.append(f"e{n}={rng.choice('AB')}[v >= 0]")
            aliases.append(f"e{n}")
        if not parts[0].startswith("every") and rng.random() < 0.5:
            parts[0] = "every " + parts[0]
        w = f" within {rng.choice([8, 20, 60])} milliseconds" if rng.random() < 0.5 else ""
        sep = ", " if seq else " -> "
        body.append(f"@info(name='a{qn}') from {sep.join(parts)}{w} "
                    f"select {aliases[0]}.v as a, {aliases[-1]}.v as b insert into Out;")
    if partition:
        np_ = rng.randint(1, n_queries)
        qs.append("partition with (k of A, k of B) begin " + " ".join(body[:np_]) + " end;")
        qs += body[np_:]
    else:
        qs += body
    return " ".join(qs)


def random_timeline(seed, n=200):
    """Events of random_events interleaved with time advances (the gaps a live runtime idles)."""
    rng = np.random.default_rng(seed + 1000)
    out = []
    for stream, row, t in random_events(seed, n=n):
        if rng.random() < 0.15:
            out.append(("advance", None, t - 1 if t > 0 else 0))
        out.append((stream, row, t))
    return out


# ---- distinct-stream patterns (the K_slab class, siddhi_amd/csrc/slab.h): every state reads its own
# stream, inside `partition with` one key over all streams ----
SLAB_STREAMS = tuple(f"S{i}" for i in range(6))


def slab_streams_def():
    return " ".join(f"define stream {s} (k int, a float, b int, s string);" for s in SLAB_STREAMS)


def _slab_pred(rng, refs, own=None):
    """A filter over the current event, constants and earlier slots (refs: (alias, is_count));
    own: this state's alias when it is a count state (its own [last] reads the previous event)."""
    def operand():
        r = rng.random()
        if refs and r < 0.5:
            al, cnt = rng.choice(refs)
            idx = rng.choice(["", "[0]", "[last]"]) if cnt else ""
            return f"{al}{idx}.{rng.choice('ab')}"
        if own and r < 0.6:
            return f"{own}[last].{rng.choice('ab')}"
        return None
    terms = []
    for _ in range(rng.choice([1, 1, 2])):
        attr = rng.choice("ab")
        op = rng.choice([">", "<", ">=", "<=", "==", "!="])
        rhs = operand()
        if rhs is None:
            if rng.random() < 0.1:
                terms.append(f"s == '{rng.choice('xyz')}'")
                continue
            c = rng.randint(0, 9)
            rhs = f"{c}.5" if attr == "a" and rng.random() < 0.5 else str(c)
        elif rng.random() < 0.25:
            rhs = f"{rhs} {rng.choice(['+', '*', '-'])} {rng.choice(['1', '2', '0.5'])}"
        terms.append(f"{attr} {op} {rhs}")
    if len(terms) == 2 and rng.random() < 0.3:
        return f"{terms[0]} or {terms[1]}"
    if rng.random() < 0.08 and refs:
        al, cnt = rng.choice([x for x in refs if not x[1]] or refs)
        if not cnt:
            return f"not ({terms[0]}) and {al}.b is null" if rng.random() < 0.5 else f"{terms[0]} or {al}.b is null"
    return " and ".join(terms)


def random_slab_query(rng, name):
    streams = list(SLAB_STREAMS)
    rng.shuffle(streams)
    n_el = rng.randint(2, 4)
    parts, refs, sel = [], [], []
    prev_count = False
    for i in range(n_el):
        r = rng.random()
        if i > 0 and r < 0.3 and len(streams) >= 2:
            s1, s2 = streams.pop(), streams.pop()
            a1, a2 = f"e{i}", f"e{i}x"
            p1, p2 = _slab_pred(rng, refs), _slab_pred(rng, refs)
            parts.append(f"{a1}={s1}[{p1}] {rng.choice(['and', 'or'])} {a2}={s2}[{p2}]")
            refs += [(a1, False), (a2, False)]
            sel.append(a1)
            prev_count = False
            continue
        st = streams.pop()
        al = f"e{i}"
        if i > 0 and r < 0.55 and not prev_count:
            mn = rng.randint(1, 3)
            mx = mn + rng.randint(0, 3)
            cnt = rng.choice([f"<{mn}:{mx}>", f"<{mx}>", f"<{mn}:{mx}>"])
            parts.append(f"{al}={st}[{_slab_pred(rng, refs, own=al if rng.random() < 0.3 else None)}]{cnt}")
            refs.append((al, True))
            sel.append(al)
            prev_count = True
            continue
        parts.append(f"{al}={st}[{_slab_pred(rng, refs)}]")
        refs.append((al, False))
        sel.append(al)
        prev_count = False
    if rng.random() < 0.8:
        parts[0] = "every " + parts[0]
    within = f" within {rng.choice([5, 12, 30, 80])} milliseconds" if rng.random() < 0.7 else ""
    return (f"@info(name='{name}') from {' -> '.join(parts)}{within} "
            f"select {sel[0]}.a as x, {sel[-1]}.b as y insert into Out;")


def random_slab_app(seed, n_queries=6):
    rng = random.Random(seed)
    body = " ".join(random_slab_query(rng, f"q{i}") for i in range(n_queries))
    keys = ", ".join(f"k of {s}" for s in SLAB_STREAMS)
    return f"{slab_streams_def()} partition with ({keys}) begin {body} end;"


def random_slab_events(seed, n=600, keys=4):
    """(stream, row, ts) with rows (k, a, b, s); timestamps non-decreasing, now and then a null."""
    rng = np.random.default_rng(seed)
    ev, t = [], 0
    for _ in range(n):
        t += int(rng.integers(0, 3))
        row = [int(rng.integers(0, keys)), float(np.float32(rng.integers(0, 20) / 2.0)), int(rng.integers(0, 10)),
               str(rng.choice(list("xyz")))]
        if rng.random() < 0.02:
            row[int(rng.integers(1, 4))] = None
        ev.append((SLAB_STREAMS[int(rng.integers(0, len(SLAB_STREAMS)))], row, t))
    return ev


# ---- a stream the partition does not key (fan-out to every key's instances in the reference's
# ConcurrentHashMap order, PartitionStreamReceiver.java:277-281) ----
FAN_STREAMS = ("define stream A (k {kt}, v int, p float, s string); "
               "define stream B (k int, v int, p float, s string);")


def fanout_app(seed, key_type="int"):
    """Partition keyed by A.k only; its patterns read B too (every key's instance sees every B
    event): starts on A or on B, 2-3 states, cross-references, within, a sequence."""
    rng = random.Random(seed)
    qs = [FAN_STREAMS.format(kt=key_type), "partition with (k of A) begin"]
    forms = [
        "from every e1=A[v > {a}] -> e2=B[p > e1.p] within {w} milliseconds",
        "from e1=A[v < {a}] -> e2=B[v == e1.v or v > 8]",
        "from every e1=B[v > {a}] -> e2=A[p < e1.p] within {w} milliseconds",
        "from every e1=A[v > {a}], e2=B[v >= {b}]",
        "from every e1=B[v > {a}] -> e2=B[v < e1.v] -> e3=A[v > {b}] within {w} milliseconds",
        "from every e1=A[v > {a}] -> e2=B[v > {b}] or e3=A[v < {b}] within {w} milliseconds",
    ]
    picks = rng.sample(range(len(forms)), 4)
    for qn, f in enumerate(picks):
        body = forms[f].format(a=rng.randint(1, 7), b=rng.randint(1, 7), w=rng.randint(5, 40))
        qs.append(f"@info(name='f{qn}') {body} select e1.v as x insert into O;")
    qs.append("end;")
    return " ".join(qs)


def fanout_events(seed, n=600, keys=40, key_type="int"):
    rng = np.random.default_rng(seed)
    out, t = [], 0
    for _ in range(n):
        t += int(rng.integers(0, 3))
        k = int(rng.integers(0, keys))
        if key_type == "long":
            k = k * 1_000_003 - 7_000_000_000 if k % 2 else k
        elif key_type == "bool":
            k = bool(k % 2)
        elif key_type == "string":  # texts of several lengths (the map hashes "A" + the text)
            k = ("IBM", "WSO2", "ORCL", "é", "")[k % 5] + "x" * (k // 5)
        elif key_type in ("float", "double"):  # Float / Double.toString forms: plain, E-notation, NaN, -0.0
            k = (0.1 * k, k * 1.0e9, -k / 3.0, 2.0 ** -(k + 130), float("nan"), -0.0, 1.0e-5 * k, 2.0e23)[k % 8]
        row = [k, int(rng.integers(0, 10)), float(np.float32(rng.integers(0, 20) / 2.0)),
               str(rng.choice(list("xyz")))]
        st = "A" if rng.random() < 0.6 else "B"
        if st == "B":
            row[0] = int(rng.integers(0, 5))  # (B.k is an int nobody partitions by)
        out.append((st, row, t))
    return out
