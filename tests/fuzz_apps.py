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
