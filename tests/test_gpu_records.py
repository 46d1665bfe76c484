"""Device records (SDH_FLAG_DEVICE_MATCHES + sdh_engine_poll_records, include/siddhi_hip.h).

A push in device-record mode leaves every match in HBM as the kernels wrote it. These tests read the
records through the C-ABI descriptor only -- the formats documented in include/siddhi_hip.h, decoded
here independently of the library -- and compare them with what a normal-mode engine delivers for
the same pushes (sdh_engine_poll / poll_compact: the R18-ordered matches the oracle pins elsewhere).
Records carry no delivery order, so the comparison is as multisets.
"""
import ctypes

import numpy as np
import pytest

from harness import App

pytestmark = pytest.mark.gpu

D2H, D2D = 2, 3


def _hip():
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return lib


def _host(ptr, n, dtype):
    """n elements of dtype at device pointer ptr -> numpy."""
    out = np.zeros(n, dtype)
    if n:
        assert _hip().hipMemcpy(out.ctypes.data, ptr, out.nbytes, D2H) == 0
    return out


def _torch(ptr, nbytes, dev):
    """nbytes at device pointer ptr -> a uint8 torch tensor (device-to-device copy)."""
    import torch
    t = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    if nbytes:
        assert _hip().hipMemcpy(t.data_ptr(), ptr, nbytes, D2D) == 0
    return t


def decode_ratchet_torch(rec, dev):
    """Part 1 (K_ratchet blocks) decoded with torch from the header's layout alone -> int64 [n, 3]
    (query, e2 - seq_base, e2 - e1)."""
    import torch
    from siddhi_amd.engine import SDH_REC_4, SDH_REC_8
    nb, bb = rec.r_blocks, rec.r_blk_bytes
    blk = _torch(rec.r_base, nb * bb, dev).view(torch.int32).view(nb, bb // 4)
    cnt = _torch(rec.r_count, nb * 4, dev).view(torch.int32).long()
    grp = _torch(rec.r_group, nb * 4, dev).view(torch.int32).long()
    ngr = int(grp.max().item()) + 1
    lq = _torch(rec.r_lane_query, ngr * 64 * 4, dev).view(torch.int32).long()
    W = bb // 4
    col = torch.arange(W, device=dev)
    if rec.r_format == SDH_REC_4:
        side = _torch(rec.r_side, nb * 4, dev).view(torch.int32).long()
        assert bool((side >= 0).all())  # (every block of these launches is a rec4 block)
        ent = blk[col[None, :].expand(nb, W) < cnt[:, None]].long() & 0xFFFFFFFF
        eb = torch.repeat_interleave(torch.arange(nb, device=dev), cnt)
        first = torch.cumsum(cnt, 0) - cnt  # entry index within its block: position - the block's first
        ei = torch.arange(len(eb), device=dev) - first[eb]
        pairs = blk.view(nb, W // 2, 2).flip(1)  # side entry j = pairs[b, j] = (first, e2)
        S = W // 2
        smask = torch.arange(S, device=dev)[None, :].expand(nb, S) < side[:, None]
        sp = pairs[smask].long()  # rows in (block, j) order: keys ascend
        sb = torch.repeat_interleave(torch.arange(nb, device=dev), side)
        skey = sb * (1 << 24) + sp[:, 0]
        ekey = eb * (1 << 24) + ei
        j = torch.searchsorted(skey, ekey, right=True) - 1
        assert bool((sb[j] == eb).all())
        e2 = sp[j, 1]
        lane = ent >> 26
        d = ent & ((1 << 26) - 1)
    else:
        assert rec.r_format == SDH_REC_8
        pr = blk.view(nb, W // 2, 2)
        m = torch.arange(W // 2, device=dev)[None, :].expand(nb, W // 2) < cnt[:, None]
        v = pr[m].long() & 0xFFFFFFFF
        eb = torch.repeat_interleave(torch.arange(nb, device=dev), cnt)
        e2 = v[:, 0] & ((1 << 26) - 1)
        lane = v[:, 0] >> 26
        s2 = (rec.seq_base + e2) & 0xFFFFFFFF
        d = (s2 - v[:, 1]) & 0xFFFFFFFF
    q = lq[grp[eb] * 64 + lane]
    return torch.stack([q, e2, d], 1)


def _key(t):
    """(query, e2, e2 - e1) rows -> one sortable int64 key each (e2 < 2^24, query < 2^14, d < 2^26)."""
    return (t[:, 1] << 40) | (t[:, 0] << 26) | t[:, 2]


def test_device_records_decode_to_compact_rows():
    """A 1M-event push of the 1K-pattern C2 family in device-record mode (rec4 blocks): the records
    handed out by sdh_engine_poll_records, decoded (a) by sdh_engine_records_compact and (b) here from
    the documented layout, are exactly the compact rows a normal-mode engine's poll_compact returns
    for the same push (as sorted sets of (query, e2, e2 - e1))."""
    import torch
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, SDH_REC_4, HipEngine
    from siddhi_amd.workloads import c2_app, stock_events_torch
    app = App(c2_app(1000), engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    dev = torch.device("cuda:0")
    n = 1 << 20
    ts, sym, price, vol = stock_events_torch(0, n, 100, dev)
    ptrs = [sym.data_ptr(), price.view(torch.int32).data_ptr(), vol.data_ptr()]
    torch.cuda.synchronize()
    normal = HipEngine(app.blob, stream_types=types)
    normal.push_device(0, n, ts.data_ptr(), ptrs)
    c = normal.poll_compact(device=True)
    assert c.width == 4 and c.n > 3e8
    want = _torch(ctypes.cast(c.rows, ctypes.c_void_p).value, c.n * 16, dev).view(torch.int32).view(-1, 4).long()
    normal.close()
    assert bool((want[:, 3] == 0).all())
    want_k = torch.sort(_key(want[:, :3]))[0]
    del want

    devr = HipEngine(app.blob, stream_types=types, flags=SDH_FLAG_DEVICE_MATCHES)
    devr.push_device(0, n, ts.data_ptr(), ptrs)
    assert devr.pending_matches() == c.n
    rec = devr.poll_records()
    assert rec.r_format == SDH_REC_4 and rec.n == rec.r_n == c.n and rec.f_n == 0 and rec.c_n == 0
    assert rec.seq_base == 0 and rec.n_events == n and rec.r_bytes < 5 * rec.r_n
    assert devr.pending_matches() == 0  # handed out
    # (a) the library's decode
    rows = torch.empty((rec.r_n, 4), dtype=torch.int32, device=dev)
    assert devr.records_compact(rows.data_ptr(), rec.r_n, 4) == rec.r_n
    got = rows.long()
    del rows
    assert bool((got[:, 3] == 0).all())
    assert torch.equal(torch.sort(_key(got[:, :3]))[0], want_k)
    del got
    # (b) the header's layout, decoded here
    mine = decode_ratchet_torch(rec, dev)
    assert torch.equal(torch.sort(_key(mine))[0], want_k)
    devr.close()


def test_device_records_8b_and_chain_segments():
    """The other K_ratchet record form (8-B records: a chunked push of a key without a float column
    takes them) and the K_chain segments (the same queries with the ratchet plan off) decode to the
    normal-mode matches."""
    import torch
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, SDH_FLAG_NO_RATCHET, SDH_REC_8, HipEngine
    src = "define stream S (v int, w long);"
    for p in range(80):
        src += (f" @info(name='i{p}') from every e1=S[v > {900 + p}] -> e2=S[v > e1.v] within {1 + p % 5} sec "
                "select e1.v as a insert into O;")
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    rng = np.random.default_rng(5)
    n = 200_000
    ts = np.arange(n, dtype=np.int64) * 3
    v = rng.integers(0, 1000, n).astype(np.int32)
    w = rng.integers(0, 1 << 40, n).astype(np.int64)
    normal = HipEngine(app.blob, stream_types=types)
    normal.push_columns(0, ts, [v, w])
    q, k, t, off, words, seq, tb = normal.poll(with_seq=True)
    want = sorted(zip(q.tolist(), seq.tolist(), words[off[:-1] + 1].tolist()))
    assert len(want) > 10000
    normal.close()
    for flags in (SDH_FLAG_DEVICE_MATCHES, SDH_FLAG_DEVICE_MATCHES | SDH_FLAG_NO_RATCHET):
        e = HipEngine(app.blob, stream_types=types, flags=flags)
        e.push_columns(0, ts, [v, w])
        rec = e.poll_records()
        assert rec.n == len(want)
        if flags & SDH_FLAG_NO_RATCHET:  # part 3: {query, ts, seq_0 .. seq_{S-1}} per record
            assert rec.c_n == rec.n and rec.r_n == 0
            offs = _host(rec.c_off, rec.c_items, np.int64)
            cnts = _host(rec.c_count, rec.c_items, np.int64)
            tot = int((offs + cnts).max()) * rec.c_words
            allw = _host(rec.c_base, tot, np.int64).reshape(-1, rec.c_words)
            got = []
            for o, c in zip(offs.tolist(), cnts.tolist()):
                for r in allw[o:o + c]:
                    got.append((int(r[0]), int(r[3]), int(r[2])))
                    assert r[1] == ts[r[3]]
        else:
            assert rec.r_format == SDH_REC_8 and rec.r_n == rec.n
            d = decode_ratchet_torch(rec, torch.device("cuda:0")).cpu().numpy()
            got = [(int(a), int(b), int(b - c)) for a, b, c in d]
        assert sorted(got) == want
        e.close()


def _slots(r, sq, kind):
    """A narrow K_part / K_seq record's slot words, expanded as matches.hip append_gen_kernel does."""
    lo = lambda x: int(np.int32(np.uint32(int(x) & 0xFFFFFFFF)))  # noqa: E731
    hi = lambda x: int(np.int32(np.uint32((int(x) >> 32) & 0xFFFFFFFF)))  # noqa: E731
    out = []
    if kind == 2:
        S = hi(r[1])
        for j in range(S - 1):
            out += [1, sq - (hi(r[2 + j // 2]) if j & 1 else lo(r[2 + j // 2]))]
        return out + [1, sq]
    e1 = sq - lo(r[2])
    out = [1, e1]
    if kind == 1:
        c = hi(r[2])
        out.append(c)
        for j in range(c):
            out.append(sq - (hi(r[3 + j // 2]) if j & 1 else lo(r[3 + j // 2])))
        return out + [1, sq]
    for dd in (hi(r[2]), lo(r[3])):
        out += [0] if dd == -(1 << 31) else [1, sq - dd]
    return out


def walk_flat(rec):
    """Part 2 (flat records) walked by the first word's length -> [(query, key, trigger seq, slot words)]."""
    words = _host(rec.f_base, rec.f_words, np.int64)
    qk_ptrs = {}
    keys = {}
    out, i, pads = [], 0, 0
    while i < len(words):
        w0 = int(words[i])
        lo = int(np.int32(np.uint32(w0 & 0xFFFFFFFF)))
        if lo >= 0:
            r = words[i:i + lo]
            S = int(r[6]) & 0xFFFF
            out.append((int(r[1]), int(r[2]), int(r[4]), tuple(int(x) for x in r[7:lo])))
            assert S >= 1
            i += lo
            continue
        kind, nw = (-lo) >> 16, (-lo) & 0xFFFF
        assert nw > 0 and kind in (0, 1, 2, 4), (i, hex(w0))
        if kind == 4:
            pads += 1
            i += nw
            continue
        r = words[i:i + nw]
        q = w0 >> 32
        off = int(r[1]) & 0xFFFFFFFF
        sq = rec.seq_base + off
        key = -1
        if kind != 2:
            kid = (int(r[1]) >> 32) & 0xFFFFFFFF
            if q not in qk_ptrs:  # f_query_keys[q]: the query's key table (device pointer)
                qk_ptrs[q] = int(_host(rec.f_query_keys + 8 * q, 1, np.uint64)[0])
            if (q, kid) not in keys:
                keys[(q, kid)] = int(_host(qk_ptrs[q] + kid * 8, 1, np.int64)[0])
            key = keys[(q, kid)]
        out.append((q, key, sq, tuple(_slots(r, sq, kind))))
        i += nw
    assert i == len(words)
    return out, pads


@pytest.mark.parametrize("family", ["c3", "c4", "gen"])
def test_device_records_flat_part(family):
    """Flat device records (K_part narrow records with key ids, K_seq windows, K_gen full records)
    walked by their documented first-word lengths over padding: the same (query, key, trigger seq,
    slots) multiset as the normal-mode engine's poll, over several pushes."""
    from siddhi_amd.engine import SDH_FLAG_DEVICE_MATCHES, SDH_FLAG_FORCE_GEN, HipEngine
    from siddhi_amd.workloads import c3_app, c4_app, stock_events, txn_events
    if family == "c4":
        src, gen, K, extra = c4_app(256), txn_events, 2000, 0
    else:
        src, gen, K, extra = c3_app(128), stock_events, 50, (SDH_FLAG_FORCE_GEN if family == "gen" else 0)
    app = App(src, engine_factory=lambda blob: None)
    types = [s.attr_types for s in app.ir.streams]
    kw = dict(stream_types=types, gen_max_keys=4096)
    normal = HipEngine(app.blob, flags=extra, **kw)
    devr = HipEngine(app.blob, flags=extra | SDH_FLAG_DEVICE_MATCHES, **kw)
    lo, total = 0, 0
    for n in (3000, 17, 9000):
        ts, x, y, z = gen(lo, n, K)
        lo += n
        cols = [x, y.view(np.uint32) if y.dtype == np.float32 else y, z]
        normal.push_columns(0, ts, cols)
        devr.push_columns(0, ts, cols)
        q, k, t, off, words, seq, tb = normal.poll(with_seq=True)
        want = sorted((int(q[i]), int(k[i]), int(seq[i]), tuple(int(v) for v in words[off[i]:off[i + 1]]))
                      for i in range(len(q)))
        rec = devr.poll_records()
        assert rec.n == rec.f_n == len(want) and rec.r_n == 0
        got, pads = walk_flat(rec) if rec.f_n else ([], 0)
        assert sorted(got) == want
        total += len(want)
    assert total > 1000
    normal.close()
    devr.close()
