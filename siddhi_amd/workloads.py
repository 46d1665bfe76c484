"""Seeded synthetic streams and pattern families of SURVEY.md §8(d) / BASELINE.json configs.

Counter-based: h_j(i) = splitmix64(seed ^ (4*i + j)), so any shard can regenerate any range.

* ts_i     = 1_700_000_000_000 + i                 (1 event / ms)
* price_i  = (float)(h_1 % 10000) / 100.0f         in [0, 100)
* volume_i = 1 + h_2 % 1000
* sym_i    = h_3 % K                               (dictionary id of "SYM<k>")

C1: every e1=StockStream[price>20] -> e2=StockStream[price>e1.price] within 10 sec
C2: P patterns  every e1=StockStream[price > T_p] -> e2=StockStream[price > e1.price] within W_p
    T_p = 20 + (p % 750) / 10.0 (a DOUBLE literal -> Float x Double compare),
    W_p in {1, 10, 60} sec picked by splitmix64(7 ^ p) % 3.
C4: fraud-rule sequences (strict contiguity, R14) over the Txn stream (same counter-based
    generator: amount_i = (float)(h_1 % 100000) / 100.0f in [0, 1000), risk_i = h_2 % 100,
    account_i = h_3 % K):
    every e1=Txn[amount > A_p], e2=Txn[amount > e1.amount * M_p], e3=Txn[amount > e2.amount and
    risk > R_p] within 1 min.
"""
from __future__ import annotations

import numpy as np

TS0 = 1_700_000_000_000
EVENT_SEED = 42
PATTERN_SEED = 7
STOCK_STREAM = "define stream StockStream (symbol string, price float, volume int);"

_M64 = (1 << 64) - 1


def splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def stock_events(start: int, n: int, n_symbols: int = 100, seed: int = EVENT_SEED):
    """Events [start, start+n) of the seeded StockStream: (ts int64, sym int32, price float32,
    volume int32)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    s = np.uint64(seed)
    h1 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(1)))
    h2 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(2)))
    h3 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(3)))
    ts = (np.int64(TS0) + i.astype(np.int64)).astype(np.int64)
    price = (h1 % np.uint64(10000)).astype(np.float32) / np.float32(100.0)
    volume = (np.uint64(1) + h2 % np.uint64(1000)).astype(np.int32)
    sym = (h3 % np.uint64(n_symbols)).astype(np.int32)
    return ts, sym, price.astype(np.float32), volume


def c1_app() -> str:
    return (STOCK_STREAM + " @info(name='q0') from every e1=StockStream[price>20] -> "
            "e2=StockStream[price>e1.price] within 10 sec select e1.price as p1, e2.price as p2 "
            "insert into OutStream;")


def c2_threshold_text(p: int) -> str:
    t10 = 200 + (p % 750)
    return f"{t10 // 10}.{t10 % 10}"


def c2_within_sec(p: int, seed: int = PATTERN_SEED) -> int:
    return (1, 10, 60)[splitmix64(seed ^ p) % 3]


def c2_app(n_patterns: int, within=None, first: int = 0, step: int = 1) -> str:
    """1K concurrent 2-state filter+reference patterns (BASELINE.json configs[1]); a shard holds
    patterns first, first+step, ... (n_patterns of them: a contiguous range, or with step = N the
    strided shard of N GPUs, which balances the thresholds)."""
    qs = [STOCK_STREAM]
    for p in range(first, first + n_patterns * step, step):
        w = c2_within_sec(p) if within is None else within
        qs.append(f"@info(name='p{p}') from every e1=StockStream[price > {c2_threshold_text(p)}] -> "
                  f"e2=StockStream[price > e1.price] within {w} sec "
                  f"select e1.price as p1, e2.price as p2 insert into OutStream;")
    return " ".join(qs)


def c2x_volume(p: int) -> int:
    return 200 + (p % 7) * 100


def c2x_app(n_patterns: int, first: int = 0, step: int = 1) -> str:
    """The C2 family with one more event-only conjunct on e2: `e2=StockStream[price
    > e1.price and volume > V_p]`, V_p in 200 .. 800. A partial survives an event whose volume fails
    V_p whatever its price, so the pending keys are no longer monotone (K_ratchet's deque argument,
    DESIGN.md §3.1) -- the gated form of the ratchet plan (§3.1, "gated e2") handles it."""
    qs = [STOCK_STREAM]
    for p in range(first, first + n_patterns * step, step):
        qs.append(f"@info(name='x{p}') from every e1=StockStream[price > {c2_threshold_text(p)}] -> "
                  f"e2=StockStream[price > e1.price and volume > {c2x_volume(p)}] within {c2_within_sec(p)} sec "
                  f"select e1.price as p1, e2.price as p2 insert into OutStream;")
    return " ".join(qs)


def c3_query(p: int, seed: int = PATTERN_SEED) -> str:
    """Pattern p of the C3 family: count <2:5>, logical and, logical or, within 10 sec,
    all inside `partition with (symbol of StockStream)`."""
    t = c2_threshold_text(p)
    v = 100 + (splitmix64(seed ^ (p + 1000)) % 800)
    kind = p % 3
    if kind == 0:
        # count <2:5> in the middle of the chain (chained events, shared with the next state while it
        # keeps counting). `every e1=S[..]<2:5>` at the START is avoided: there the reference's
        # shallow every-clones share one event chain, two appends per event can skip over `max`, and
        # such partials then stay pending for ever (unbounded state in the reference itself).
        body = (f"every e1=StockStream[price > {t}] -> e2=StockStream[volume > {v // 4}] <2:5> -> "
                f"e3=StockStream[price > e2[last].price] within 10 sec "
                f"select e1.price as a, e2[0].volume as b, e3.price as c")
    elif kind == 1:
        body = (f"every e1=StockStream[price > {t}] -> e2=StockStream[volume > {v}] and "
                f"e3=StockStream[price < {t}] within 10 sec select e1.price as a, e2.volume as b")
    else:
        body = (f"every e1=StockStream[volume < {v}] -> e2=StockStream[price > {t}] or "
                f"e3=StockStream[volume > {1000 - v // 4}] within 10 sec select e1.volume as a, e2.price as b")
    return f"@info(name='c3p{p}') from {body} insert into OutStream;"


def c3_app(n_patterns: int, first: int = 0, step: int = 1) -> str:
    """C3 (BASELINE.json configs[2]): count/kleene <2:5> plus logical and/or patterns,
    `partition with (symbol)` (keys = the stream's symbols)."""
    qs = " ".join(c3_query(p) for p in range(first, first + n_patterns * step, step))
    return f"{STOCK_STREAM} partition with (symbol of StockStream) begin {qs} end;"


TXN_STREAM = "define stream Txn (account string, amount float, risk int);"


def txn_events(start: int, n: int, n_accounts: int = 100_000, seed: int = EVENT_SEED):
    """Events [start, start+n) of the seeded Txn stream: (ts int64, account int32 dictionary id,
    amount float32, risk int32)."""
    i = np.arange(start, start + n, dtype=np.uint64)
    s = np.uint64(seed)
    h1 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(1)))
    h2 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(2)))
    h3 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(3)))
    ts = (np.int64(TS0) + i.astype(np.int64)).astype(np.int64)
    amount = (h1 % np.uint64(100000)).astype(np.float32) / np.float32(100.0)
    risk = (h2 % np.uint64(100)).astype(np.int32)
    account = (h3 % np.uint64(n_accounts)).astype(np.int32)
    return ts, account, amount.astype(np.float32), risk


def c4_query(p: int, seed: int = PATTERN_SEED) -> str:
    """Fraud rule p of the C4 family: a 3-event strict-contiguity sequence."""
    h = splitmix64(seed ^ (p + 2000))
    a = 100 + p % 800
    m = ("1.05", "1.1", "1.2", "1.5")[h % 4]
    r = (h >> 8) % 90
    return (f"@info(name='f{p}') from every e1=Txn[amount > {a}], e2=Txn[amount > e1.amount * {m}], "
            f"e3=Txn[amount > e2.amount and risk > {r}] within 1 min "
            f"select e1.account as acct, e1.amount as a1, e3.amount as a3 insert into Alerts;")


def c4_app(n_patterns: int, first: int = 0, step: int = 1) -> str:
    """C4 (BASELINE.json configs[3]): fraud-rule sequences; a shard holds patterns first,
    first+step, ... (pattern-set sharding across GPUs)."""
    return " ".join([TXN_STREAM] + [c4_query(p) for p in range(first, first + n_patterns * step, step)])


# ---- the same streams generated on a device with torch (int64 ops wrap like uint64; logical shifts
# and unsigned remainders are spelled out), bit-identical to the numpy generators above ----
def _c64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _srl(z, k: int):
    return (z >> k) & ((1 << (64 - k)) - 1)


def _splitmix64_t(x):
    z = x + _c64(0x9E3779B97F4A7C15)
    z = (z ^ _srl(z, 30)) * _c64(0xBF58476D1CE4E5B9)
    z = (z ^ _srl(z, 27)) * _c64(0x94D049BB133111EB)
    return z ^ _srl(z, 31)


def _umod_t(u, m: int):
    return ((_srl(u, 1) % m) * 2 + (u & 1)) % m


def _hashes_t(start: int, n: int, seed: int, device):
    import torch
    i = torch.arange(start, start + n, dtype=torch.int64, device=device)
    return i, [_splitmix64_t(seed ^ (i * 4 + j)) for j in (1, 2, 3)]


def stock_events_torch(start: int, n: int, n_symbols: int, device, seed: int = EVENT_SEED):
    """stock_events as torch tensors on `device`: (ts int64, sym int32, price float32, volume int32)."""
    import torch
    i, (h1, h2, h3) = _hashes_t(start, n, seed, device)
    price = _umod_t(h1, 10000).to(torch.float32) / 100.0
    return TS0 + i, _umod_t(h3, n_symbols).to(torch.int32), price, (1 + _umod_t(h2, 1000)).to(torch.int32)


def txn_events_torch(start: int, n: int, n_accounts: int, device, seed: int = EVENT_SEED):
    """txn_events as torch tensors on `device`: (ts int64, account int32, amount float32, risk int32)."""
    import torch
    i, (h1, h2, h3) = _hashes_t(start, n, seed, device)
    amount = _umod_t(h1, 100000).to(torch.float32) / 100.0
    return TS0 + i, _umod_t(h3, n_accounts).to(torch.int32), amount, _umod_t(h2, 100).to(torch.int32)


# ---- C5 family (BASELINE.json configs[4]): mixed 2-4-state patterns over four
# joined streams, `partition with` one account key across all four, `within 1 hour` ----
C5_STREAMS = ("Card", "Login", "Transfer", "Device")


def c5_streams_def() -> str:
    return " ".join(f"define stream {s} (acct int, amount float, code int);" for s in C5_STREAMS)


def c5_query(p: int, seed: int = PATTERN_SEED) -> str:
    """Pattern p of the C5 family: kind p % 4 (2-state cross-stream reference, logical and, logical
    or, 4-state with a count state) over a fixed stream route per kind (so a kind is one shape and
    64 patterns fill one wave), thresholds from splitmix64(seed ^ (p + 5000)). Start filters pass
    0.1-5 % of events: fraud rules, with state sparse per account."""
    h = splitmix64(seed ^ (p + 5000))
    a = 950 + (h >> 8) % 49
    m = ("1.01", "1.05", "1.1", "1.25")[(h >> 20) % 4]
    c = (h >> 24) % 100
    kind = p % 4
    if kind == 0:
        body = (f"every e1=Card[amount > {a}] -> e2=Transfer[amount > e1.amount * {m}] within 1 hour "
                f"select e1.acct as k, e1.amount as a1, e2.amount as a2")
    elif kind == 1:
        body = (f"every e1=Login[amount > {a}] -> e2=Transfer[code == e1.code] and e3=Device[amount < {1000 - a}] "
                f"within 1 hour select e1.acct as k, e2.code as c2, e3.amount as a3")
    elif kind == 2:
        body = (f"every e1=Card[amount > {a}] -> e2=Login[amount > e1.amount] or e3=Device[code > {c}] "
                f"within 1 hour select e1.acct as k, e2.amount as a2, e3.code as c3")
    else:
        body = (f"every e1=Card[amount > {a}] -> e2=Transfer[amount < e1.amount]<1:3> -> "
                f"e3=Device[amount > e2[last].amount] -> e4=Login[code == e1.code] within 1 hour "
                f"select e1.acct as k, e2[0].amount as a2, e4.code as c4")
    return f"@info(name='c5p{p}') from {body} insert into Alerts;"


def c5_app(n_patterns: int, first: int = 0, step: int = 1) -> str:
    """C5 (BASELINE.json configs[4]): n_patterns mixed patterns in one `partition with (acct of
    Card, acct of Login, acct of Transfer, acct of Device)`; a shard holds patterns first ..
    first+n_patterns-1 (key sharding spreads the accounts over GPUs)."""
    qs = " ".join(c5_query(p) for p in range(first, first + n_patterns * step, step))
    keys = ", ".join(f"acct of {s}" for s in C5_STREAMS)
    return f"{c5_streams_def()} partition with ({keys}) begin {qs} end;"


def c5_events(stream: int, start: int, n: int, n_accounts: int, seed: int = EVENT_SEED):
    """Events [start, start+n) of C5 stream `stream` (1 event / ms each): (ts int64, acct int32,
    amount float32 in [0, 1000), code int32 in [0, 100))."""
    i = np.arange(start, start + n, dtype=np.uint64)
    s = np.uint64(seed ^ (0x5C5 + stream))
    h1 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(1)))
    h2 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(2)))
    h3 = splitmix64_np(s ^ (i * np.uint64(4) + np.uint64(3)))
    ts = (np.int64(TS0) + i.astype(np.int64)).astype(np.int64)
    amount = (h1 % np.uint64(100000)).astype(np.float32) / np.float32(100.0)
    code = (h2 % np.uint64(100)).astype(np.int32)
    acct = (h3 % np.uint64(n_accounts)).astype(np.int32)
    return ts, acct, amount.astype(np.float32), code


def c5_events_torch(stream: int, start: int, n: int, n_accounts: int, device, seed: int = EVENT_SEED):
    """c5_events as torch tensors on `device`."""
    import torch
    i, (h1, h2, h3) = _hashes_t(start, n, seed ^ (0x5C5 + stream), device)
    amount = _umod_t(h1, 100000).to(torch.float32) / 100.0
    return TS0 + i, _umod_t(h3, n_accounts).to(torch.int32), amount, _umod_t(h2, 100).to(torch.int32)
