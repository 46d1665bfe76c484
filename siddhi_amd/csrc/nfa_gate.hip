// nfa_gate.hip -- K_gate: the gated ratchet family
//
//     every e1=S[f0] -> e2=S[cur.a OP e1.a and g] [within T]      OP in {<, <=, >, >=}
//
// where g is a conjunction of event-only compares with per-pattern constants (e.g. the C2x family,
// `e2=StockStream[price > e1.price and volume > V_p]`, workloads.c2x_app).
//
// Reference semantics are K_ratchet's (nfa_ratchet.hip: StreamPreStateProcessor.processAndReturn
// :292-337 visits every pending partial of state 1 in insertion order on every event; expired ->
// removed, filter passes -> emitted and removed, else kept; the partial an event opens is pending
// from the next event). What changes is the shape of the pending list: an event whose g fails
// matches nothing, so it neither removes the partials below its key nor dominates them, and the
// keys along the list are no longer monotone -- K_ratchet's deque argument fails. The list is kept
// as it is, in insertion order:
//   * an event whose g passes matches exactly the partials with `x OP key` -- anywhere in the list;
//     each lane caches the extreme key of its list (the min for >, >=; the max for <, <=), so the
//     list is scanned only when the event can match one of them (one compare per event otherwise);
//   * expiry is lazy: an expired partial can never match again (timestamps non-decreasing), so it
//     is dropped when a scan reaches it, and the persisted list is compacted at the item's last
//     event -- the pending set the reference holds there. Out-of-order timestamps take the FULL
//     form, which expires eagerly at every event (|ts - ts0| > within, isExpired:102-113).
// Storage: the insertion order of a lane's pending partials does not matter here -- a partial's fate
// depends on its own key and deadline, and a query's matches of one event are ordered by e1's seq
// where the R18 order is needed (the match table's tiebreak) -- so a lane keeps them sorted by key
// instead: the GML best (the smallest for >, >=) in an LDS ring ordered best first, so an event's
// matches there are a prefix (popped like K_ratchet's deque top, O(matches)); a new partial is
// inserted at its rank (binary search, then the shorter side of the ring shifts by one). The rest --
// keys worse than every LDS key -- sit unordered in a per-item spill in HBM, scanned only when an
// event matches the spill's own best key. Expiry is checked where a partial is reached (lazily);
// an expired partial that is never reached leaves at an eviction's or the write-back's compaction.
// Chunked items rebuild their sets at the chunk
// start by a reverse scan over the `within` window: partial i (f0 passed) is pending before event
// c0 iff it has not expired at c0-1 and no event j in (i, c0) passes g with `x_j OP key_i` -- i.e.
// iff the lane's reduction (max for >, >=) of x over the g-passing events after it does not match
// it. Tiles whose best key every lane's reduction already matches are skipped on their summary (their
// g-passing events cannot move the reductions either), as in K_ratchet's warm-up.
// Output: K_ratchet's per-wave blocks of 8-B records {e2 offset | lane << 26, e1 seq low 32} (16-B
// past 2^26-event batches), decoded by the same readers (matches.hip; sdh_records part 1).
#include "ratchet_common.h"

namespace sdh {

// LDS entries per lane: occupancy outweighs the spill (C2x at 10K patterns, 4M-event steps: GML 4
// 515 ms/step, 8 341, 16 404, 32 670; waves per SIMD aimed at 4 / 6: same, 8: 525 -- register spills)
#ifndef SDH_GATE_GML
#define SDH_GATE_GML 8
#endif
constexpr int GML = SDH_GATE_GML;  // LDS entries per lane (a power of two)
#ifndef SDH_GATE_WPE
#define SDH_GATE_WPE 4  // resident waves per SIMD the register allocation aims at
#endif

extern __shared__ uint2 gate_lds[];  // [GML][64] {key, seq}, then [GML][64] expiry words (int32 / FULL: int64)

// FULL: out-of-order timestamps (eager expiry at every event); otherwise the lazy form
template <int KK, int XM, int NF, int NG, int PM, bool FULL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SDH_GATE_WPE))) void nfa_gate_kernel(RatchetLaunch L,
                                                                                            int SC) {
  static_assert(!KT<KK>::W64, "K_gate holds 32-bit keys");
  using U = uint32_t;
  const int lane = threadIdx.x;
  const int wid = blockIdx.x;
  if (wid >= L.n_items) return;
  const RatchetItem W = L.items[wid];
  const RatchetGroup* __restrict__ G = L.groups + W.g;
  const bool active = lane < G->n_lanes;
  const int64_t within = G->within[lane & 63];
  const int64_t wmax = G->wmax;
  const bool has_within = wmax >= 0;
  const int xmask = G->xmask, kconv = G->key_conv, kattr = G->key_attr;
  const bool is_max = (xmask & CM_GT) != 0;  // the reduction over events (warm-up): max for >, >=
  const int64_t seq_base = L.b.seq_base;
  // extreme key of a list = the one a later event matches first: min for >, >=; max for <, <=
  auto ext_better = [&](U a, U b) { return xcmp<KK>(is_max ? CM_LT : CM_GT, a, b); };
  auto red_better = [&](U a, U b) { return xcmp<KK>(is_max ? CM_GT : CM_LT, a, b); };

  // ---- constant atoms of f0 (start filter) and g (e2's event-only conjuncts), as per-lane
  // intervals of sortable keys (nfa_ratchet.hip f0_interval); K_gate's atoms are constant atoms ----
  struct AtomCols {
    int64_t lo, hi;
    bool neg;
    int f64, conv, w;
    const void* ptr;
    const uint8_t* nul;
  };
  AtomCols fa[NF], ga[NG];
  const int n_f0 = G->n_f0, n_g = G->n_g;
  auto setup = [&](const RatchetAtom& A0, int64_t c, AtomCols& o) {
    int m = A0.mask;
    if (!A0.cur_left) {
      const int lt = m & CM_LT, gt = m & CM_GT;
      m = (m & (CM_EQ | CM_NOT)) | (lt ? CM_GT : 0) | (gt ? CM_LT : 0);
    }
    f0_interval(m, A0.f64 != 0, c, o.lo, o.hi, o.neg);
    o.f64 = A0.f64;
    o.conv = A0.conv;
    o.ptr = pick(L.b.col, A0.attr);
    o.w = pick(L.b.width, A0.attr);
    o.nul = pick(L.b.nul, A0.attr);
  };
#pragma unroll
  for (int a = 0; a < NF; ++a)
    if (a < n_f0) setup(G->f0[a], G->f0c[a][lane & 63], fa[a]);
#pragma unroll
  for (int a = 0; a < NG; ++a)
    if (a < n_g) setup(G->g[a], G->gc[a][lane & 63], ga[a]);
  const void* k_ptr = pick(L.b.col, kattr);
  const uint8_t* k_nul = pick(L.b.nul, kattr);
  const int k_w = pick(L.b.width, kattr);

  // one event per lane of a 64-event tile: ts, key, the atoms' sortable operand keys, validity bits
  // (bit 0 key valid, 1 + a: f0 atom a's operand null, 1 + NF + a: g atom a's operand null)
  int64_t fk[NF], gk[NG];
  auto stage = [&](int64_t e, bool live, int64_t& ets, U& xk, uint32_t& vb) {
    ets = live ? L.b.ts[e] : INT64_MAX;
    bool xok = false;
    xk = live ? (U)stage_key<KK>(load_raw(k_ptr, k_w, e), kconv, k_nul && k_nul[e], xok) : 0u;
    uint32_t v = xok ? 1u : 0u;
    auto opnd = [&](const AtomCols& o, int bit, int64_t& key) {
      key = 0;
      if (!live) return;
      const int64_t k1 = to_key(load_raw(o.ptr, o.w, e), o.conv);
      key = o.f64 ? sortable_f64(k1) : k1;
      if (o.nul && o.nul[e]) v |= 1u << bit;
    };
#pragma unroll
    for (int a = 0; a < NF; ++a)
      if (a < n_f0) opnd(fa[a], 1 + a, fk[a]);
#pragma unroll
    for (int a = 0; a < NG; ++a)
      if (a < n_g) opnd(ga[a], 1 + NF + a, gk[a]);
    vb = v;
  };
  auto pass = [&](const AtomCols* at, const int64_t* keys, int n, int bit0, int k, uint32_t vb) {
    bool ok = true;
#pragma unroll
    for (int a = 0; a < (NF > NG ? NF : NG); ++a)
      if (a < n) {
        const int64_t v = readlane64(keys[a], k);
        ok = ok && !((vb >> (bit0 + a)) & 1u) && (((v >= at[a].lo) && (v <= at[a].hi)) != at[a].neg);
      }
    return ok;
  };
  auto f0_pass = [&](int k, uint32_t vb) { return active && (vb & 1u) && pass(fa, fk, n_f0, 1, k, vb); };
  auto g_pass = [&](int k, uint32_t vb) { return active && (vb & 1u) && pass(ga, gk, n_g, 1 + NF, k, vb); };

  // ---- the lane's pending set: LDS slots [0, ln) (the best keys), spill slots [0, sn) (the rest) ----
  uint2* __restrict__ KQ = gate_lds;
  // an LDS entry's expiry word: the lazy form's 32-bit deadline relative to the item's first
  // timestamp (nfa_ratchet.hip rel_deadline; its ts0 is the batch's ts at its seq, since only this
  // batch's partials enter LDS -- carried ones stay in the spill), FULL's 64-bit ts0
  int32_t* __restrict__ DL = reinterpret_cast<int32_t*>(gate_lds + GML * WAVE);
  int64_t* __restrict__ TS = reinterpret_cast<int64_t*>(gate_lds + GML * WAVE);
  uint4* __restrict__ SP = L.spillA + (size_t)wid * SC * WAVE;
  const int64_t T0 = L.b.ts[W.c0];
  int lbot = 0, ln = 0, sn = 0;     // LDS ring slots lbot .. lbot + ln - 1, best key first
  U tk = 0;                         // the LDS ring's best key (valid while ln > 0)
  bool shas = false;                // best key of the spill part
  U sext = 0;
  uint32_t oq = 0;                  // low seq bits of the oldest held partial (a bound: removals keep it)
  const uint32_t llo = (uint32_t)(seq_base + W.c1 - 1);
  const int64_t slast = seq_base + W.c1 - 1;
  auto full_seq = [&](uint32_t q) { return slast - (int64_t)(uint32_t)(llo - q); };
  int overflow = 0, unordered = 0, mover = 0, aged = 0;
  auto li = [&](int slot) { return (slot & (GML - 1)) * WAVE + lane; };
  auto si = [&](int slot) { return (size_t)slot * WAVE + lane; };
  auto sput = [&](int slot, int64_t ts, U key, uint32_t seq) {
    SP[si(slot)] = make_uint4((uint32_t)ts, (uint32_t)((uint64_t)ts >> 32), key, seq);
  };
  auto sget = [&](int slot, int64_t& ts, U& key, uint32_t& seq) {
    const uint4 a = SP[si(slot)];
    ts = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
    key = a.z;
    seq = a.w;
  };
  // LDS entries as {key, seq, x}: x the expiry word (lazy: deadline; FULL: ts0)
  auto lput = [&](int slot, int64_t ts, U key, uint32_t seq) {
    KQ[li(slot)] = make_uint2(key, seq);
    if constexpr (FULL) TS[li(slot)] = ts;
    else DL[li(slot)] = rel_deadline(sat_add(ts, within), T0);
  };
  auto lgetx = [&](int slot, int64_t& xw, U& key, uint32_t& seq) {
    const uint2 a = KQ[li(slot)];
    key = a.x;
    seq = a.y;
    if constexpr (FULL) xw = TS[li(slot)];
    else xw = DL[li(slot)];
  };
  auto lputx = [&](int slot, int64_t xw, U key, uint32_t seq) {
    KQ[li(slot)] = make_uint2(key, seq);
    if constexpr (FULL) TS[li(slot)] = xw;
    else DL[li(slot)] = (int32_t)xw;
  };
  auto ts_of = [&](int64_t xw, uint32_t seq) -> int64_t {  // an LDS entry's ts0
    if constexpr (FULL) return xw;
    else return L.b.ts[full_seq(seq) - seq_base];
  };
  // (ts0, key, seq) of an LDS entry
  auto lget = [&](int slot, int64_t& ts, U& key, uint32_t& seq) {
    int64_t xw;
    lgetx(slot, xw, key, seq);
    ts = ts_of(xw, seq);
  };
  auto lmove = [&](int to, int from) {
    KQ[li(to)] = KQ[li(from)];
    if constexpr (FULL) TS[li(to)] = TS[li(from)];
    else DL[li(to)] = DL[li(from)];
  };
  auto dead = [&](int64_t t0, int64_t tt) {  // (ordered: tt >= t0; FULL: |tt - t0|, isExpired)
    if constexpr (FULL) return expired(t0, tt, within);
    else return tt > sat_add(t0, within);
  };
  // an LDS entry (expiry word xw) expired at tt (tt32: tt in the deadline domain)
  auto ldead = [&](int64_t xw, int64_t tt, int32_t tt32) {
    if constexpr (FULL) return expired(xw, tt, within);
    else return tt32 > (int32_t)xw;
  };
  auto rel32 = [&](int64_t tt) {
    return tt >= T0 + (INT32_MAX - 1) ? INT32_MAX - 1 : tt <= T0 + INT32_MIN ? INT32_MIN : (int32_t)(tt - T0);
  };
  auto add_ext = [&](bool& has, U& ext, U key) {
    ext = (!has || ext_better(key, ext)) ? key : ext;
    has = true;
  };
  auto note_seq = [&](uint32_t seq) {  // keep oq the oldest
    oq = (ln + sn == 0 || (uint32_t)(llo - seq) > (uint32_t)(llo - oq)) ? seq : oq;
  };
  // the spill with its expired entries dropped (in place); its best key recomputed
  auto spill_compact = [&](int64_t tt) {
    int w = 0;
    shas = false;
    for (int i = 0; i < sn; ++i) {
      int64_t t0; U k; uint32_t q;
      sget(i, t0, k, q);
      if (dead(t0, tt)) continue;
      if (w != i) sput(w, t0, k, q);
      add_ext(shas, sext, k);
      ++w;
    }
    sn = w;
  };
  auto spill_push = [&](int64_t ts, U key, uint32_t seq, int64_t tt) {
    if (sn == SC) spill_compact(tt);
    if (sn == SC) {
      overflow = 1;  // (the host re-runs the push with a larger spill)
      return;
    }
    sput(sn++, ts, key, seq);
    add_ext(shas, sext, key);
  };
  // a new pending partial at its rank in the LDS ring (tt: the current event time, for a compaction
  // of a full spill). A full ring gives its worst key to the spill -- or the new one goes there if it
  // is no better than every LDS key.
  auto push = [&](int64_t ts, U key, uint32_t seq, int64_t tt) {
    note_seq(seq);
    if (!FULL && full_seq(seq) < seq_base) {  // a carried partial: its ts0 is not in this batch
      spill_push(ts, key, seq, tt);
      return;
    }
    if (ln == GML) {
      int64_t t0; U k0; uint32_t q0;
      lget(lbot + GML - 1, t0, k0, q0);
      if (!ext_better(key, k0)) {
        spill_push(ts, key, seq, tt);
        return;
      }
      spill_push(t0, k0, q0, tt);
      --ln;
    }
    // rank p: the entries strictly better than the key -- 0 when it is at least as good as the best
    // (every push at an event that matched), else by binary search over the ring
    int p = 0;
    if (ln > 0 && ext_better(tk, key)) {
      int lo = 1, hi = ln;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (ext_better(KQ[li(lbot + m)].x, key)) lo = m + 1;
        else hi = m;
      }
      p = lo;
    }
    if (p <= ln - p) {  // the better side moves one slot toward the front
      lbot = (lbot - 1) & (GML - 1);
      for (int i = 0; i < p; ++i) lmove(lbot + i, lbot + i + 1);
    } else {            // the worse side moves one slot back
      for (int i = ln - 1; i >= p; --i) lmove(lbot + i + 1, lbot + i);
    }
    lput(lbot + p, ts, key, seq);
    ++ln;
    tk = p == 0 ? key : tk;
  };

  // ---- output blocks (K_ratchet's: one atomic per block, mbcnt ranks inside) ----
  constexpr bool WIDE = PM == 3;
  constexpr int FULL_FILL = 1 << 30;
  int blk = -1, fill = FULL_FILL;
  unsigned long long n_emit = 0, n_bytes = 0;
  __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(L.match, 0, 0, 0x00020000);
  auto roll = [&]() {
    if (blk >= 0) {
      if (lane == 0) {
        L.blk_count[blk] = fill;
        L.blk_side[blk] = -1;
      }
      n_emit += (unsigned long long)fill;
      n_bytes += (unsigned long long)fill * (WIDE ? 16 : 8);
    }
    int nb = 0;
    if (lane == 0) nb = atomicAdd(L.blk_next, 1);
    nb = __builtin_amdgcn_readfirstlane(nb);
    if (nb >= L.n_blocks) {
      mover = 1;
      blk = -1;
      nb = L.n_blocks;  // (the spare block; the host re-runs with enough blocks)
    } else {
      if (lane == 0) L.blk_group[nb] = W.g;
      blk = nb;
    }
    fill = 0;
    constexpr int rb = WIDE ? 16 : 8;
    const uint64_t base = (uint64_t)(reinterpret_cast<char*>(L.match) + (size_t)nb * L.blk_recs * rb);
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base),
                   bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    wrs = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)bhi << 32) | blo), 0,
                                            __builtin_amdgcn_readfirstlane(L.blk_recs * rb), 0x00020000);
  };
  // one record per lane with `mt` (ballot m): e2 = batch event `off`, e1 = the partial with seq q1
  auto emit = [&](bool mt, uint64_t m, uint32_t off, uint32_t q1) {
    if (m == 0) return;
    if (fill > L.blk_recs - WAVE) roll();
    if (mt) {
      const int r = fill + wave_mbcnt(m);
      if constexpr (!WIDE) {
        const u32x2 v = {off | ((uint32_t)lane << 26), q1};
        __builtin_amdgcn_raw_buffer_store_b64(v, wrs, r * 8, 0, 0);
      } else {
        const u32x4 v = {off, (uint32_t)lane, q1, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, wrs, r * 16, 0, 0);
      }
    }
    fill += __popcll(m);
  };

  // ---- the lists at the item's first event ----
  const size_t gb = (size_t)W.g * L.rsmax * WAVE;
  const int n_in = pick(L.st, W.inb)[W.g].n[lane];
  const int64_t* __restrict__ i_ts = pick(L.ent_ts, W.inb);
  const int64_t* __restrict__ i_sq = pick(L.ent_seq, W.inb);
  const int64_t* __restrict__ i_ky = pick(L.ent_key, W.inb);
  if (W.c0 == 0) {
    const int64_t t_first = L.b.ts[0];
    for (int i = 0; i < n_in; ++i) {
      const size_t o = gb + (size_t)i * WAVE + lane;
      push(i_ts[o], (U)i_ky[o], (uint32_t)i_sq[o], t_first);
    }
  } else {
    // reverse scan (ordered timestamps; FULL items are never chunked): candidates newest first
    const int64_t t_last = L.b.ts[W.c0 - 1];
    const int64_t w0 = has_within ? lower_bound_ts(L.b.ts, W.c0, t_last - wmax, lane) : 0;
    bool mh = false;  // this lane's reduction of x over the g-passing events after the scan point
    U mv = 0;
    auto detail_tile = [&](int64_t lo, int64_t hi) {
      const int64_t e = lo + lane;
      const bool live = e >= w0 && e < hi;
      int64_t ets;
      U xk;
      uint32_t vb;
      stage(e, live, ets, xk, vb);
      for (int k = (int)(hi - lo) - 1; k >= 0; --k) {
        const uint32_t vbk = __builtin_amdgcn_readlane(vb, k);
        if (!(vbk & 1u)) continue;  // (no valid key: neither a candidate nor a reduction term)
        const U x = (U)__builtin_amdgcn_readlane(xk, k);
        const int64_t tk = readlane64(ets, k);
        if (lo + k >= w0 && f0_pass(k, vbk) && !dead(tk, t_last) && !(mh && xop<KK, XM>(xmask, mv, x)))
          push(tk, x, (uint32_t)(seq_base + lo + k), t_last);
        if (g_pass(k, vbk) && (!mh || red_better(x, mv))) {
          mv = x;
          mh = true;
        }
      }
    };
    int64_t hi = W.c0;
    const int64_t al = W.c0 & ~(int64_t)63;
    if (al < hi) {
      detail_tile(al, hi);
      hi = al;
    }
    const int slot = G->sum_slot;
    while (hi > w0) {
      const int64_t jt = (hi >> 6) - 1;  // the tile [jt * 64, jt * 64 + 64)
      const size_t o = (size_t)slot * L.n_tiles + jt;
      const bool th = L.tsum_has[o] != 0;
      const U tb = (U)(is_max ? L.tsum_max[o] : L.tsum_min[o]);
      // skip: no valid key, or every active lane's reduction already matches the tile's best key
      // (then it matches every key of the tile, and the tile's g-passing x cannot move it)
      const bool need = th && active && !(mh && xop<KK, XM>(xmask, mv, tb));
      if (wballot(need) != 0) detail_tile(jt * 64, jt * 64 + 64);
      hi = jt * 64;
    }
    if (w0 == 0) {
      if (L.b.prev_ts > L.b.ts[0]) unordered = 1;
      for (int i = n_in - 1; i >= 0; --i) {
        const size_t o = gb + (size_t)i * WAVE + lane;
        const int64_t t0 = i_ts[o];
        const U ky = (U)i_ky[o];
        if (!dead(t0, t_last) && !(mh && xop<KK, XM>(xmask, mv, ky))) push(t0, ky, (uint32_t)i_sq[o], t_last);
      }
    }
  }

  // ---- forward step over the item's events ----
  int64_t prev_tile_ts = (W.c0 == 0) ? L.b.prev_ts : L.b.ts[W.c0 - 1];
  for (int64_t t = W.c0; t < W.c1; t += WAVE) {
    int64_t ets;
    U xk;
    uint32_t vb;
    stage(t + lane, t + lane < W.c1, ets, xk, vb);
    int64_t pred = __shfl_up(ets, 1, WAVE);
    if (lane == 0) pred = prev_tile_ts;
    if (t + lane < W.c1 && ets < pred) unordered = 1;
    prev_tile_ts = __shfl(ets, WAVE - 1, WAVE);
    const int cnt = (int)((W.c1 - t) < WAVE ? (W.c1 - t) : WAVE);
    // a live partial must stay < 2^31 events old (seq low bits). oq bounds the oldest held partial's
    // age from above; past 2^30 events the lane finds its true oldest live one
    const uint32_t tlo = (uint32_t)(seq_base + t + cnt - 1);
    if (sn + ln > 0 && tlo - oq >= 0x40000000u) {
      const int64_t tlast = __shfl(ets, cnt - 1, WAVE);
      bool any = false;
      auto older = [&](int64_t t0, uint32_t q) {
        if (dead(t0, tlast)) return;
        oq = (!any || tlo - q > tlo - oq) ? q : oq;
        any = true;
      };
      for (int i = 0; i < ln; ++i) {
        int64_t t0; U ky; uint32_t q;
        lget(lbot + i, t0, ky, q);
        older(t0, q);
      }
      for (int i = 0; i < sn; ++i) {
        int64_t t0; U ky; uint32_t q;
        sget(i, t0, ky, q);
        older(t0, q);
      }
      if (any && tlo - oq >= 0x80000000u) aged = 1;
      if (!any) oq = tlo;
    }
    for (int k = 0; k < cnt; ++k) {
      const uint32_t vbk = __builtin_amdgcn_readlane(vb, k);
      const U x = (U)__builtin_amdgcn_readlane(xk, k);
      const int64_t tt = readlane64(ets, k);
      const uint32_t off = (uint32_t)(t + k);
      const int32_t tt32 = FULL ? 0 : rel32(tt);
      if constexpr (FULL) {  // out-of-order timestamps: every expired partial leaves before the event (eager)
        int w = 0;
        for (int i = 0; i < ln; ++i) {
          int64_t xw; U ky; uint32_t q;
          lgetx(lbot + i, xw, ky, q);
          if (ldead(xw, tt, tt32)) continue;
          if (w != i) lputx(lbot + w, xw, ky, q);  // (order kept)
          ++w;
        }
        ln = w;
        if (ln > 0) tk = KQ[li(lbot)].x;
        spill_compact(tt);
      }
      // ---- matches: an event passing g matches every pending partial with `x OP key` ----
      const bool gate = g_pass(k, vbk);
      // the LDS part: its matches are a prefix (best keys first); an expired entry there leaves
      // unmatched
      // (one entry per round: a round of four, reading the next three unconditionally as K_ratchet
      // does, measured 363 ms per C2x step against 341 -- a lane pops one or two entries per match)
      bool pop = gate && ln > 0 && xop<KK, XM>(xmask, x, tk);
      while (wballot(pop) != 0) {
        int64_t xw = 0;
        U ky = 0;
        uint32_t q = 0;
        if (pop) lgetx(lbot, xw, ky, q);
        const bool mt = pop && !ldead(xw, tt, tt32);
        emit(mt, wballot(mt), off, q);
        if (pop) {
          lbot = (lbot + 1) & (GML - 1);
          --ln;
          tk = KQ[li(lbot)].x;  // (a stale slot when ln reaches 0: tk is then unused)
          pop = ln > 0 && xop<KK, XM>(xmask, x, tk);
        }
      }
      const bool scan_s = gate && shas && xop<KK, XM>(xmask, x, sext);
      if (wballot(scan_s) != 0) {  // (rare: the spill holds old survivors, whose keys few events reach)
        int w = 0;
        bool nh = false;
        U nx = 0;
        for (int i = 0;; ++i) {
          const bool here = scan_s && i < sn;
          if (wballot(here) == 0) break;
          int64_t t0 = 0;
          U ky = 0;
          uint32_t q = 0;
          if (here) sget(i, t0, ky, q);
          const bool live = here && !dead(t0, tt);
          const bool mt = live && xop<KK, XM>(xmask, x, ky);
          emit(mt, wballot(mt), off, q);
          if (live && !mt) {
            if (w != i) sput(w, t0, ky, q);
            ++w;
            add_ext(nh, nx, ky);
          }
        }
        if (scan_s) {
          sn = w;
          shas = nh;
          sext = nx;
        }
      }
      // ---- start state: an event passing f0 opens a partial (pending from the next event) ----
      if (f0_pass(k, vbk)) push(tt, x, (uint32_t)(seq_base + t + k), tt);
    }
  }

  // ---- outputs ----
  if (blk >= 0) {
    if (lane == 0) {
      L.blk_count[blk] = fill;
      L.blk_side[blk] = -1;
    }
    n_emit += (unsigned long long)fill;
    n_bytes += (unsigned long long)fill * (WIDE ? 16 : 8);
  }
  const uint64_t any_over = wballot(overflow != 0), any_unord = wballot(unordered != 0), any_aged = wballot(aged != 0);
  if (lane == 0) {
    if (L.dev_records && n_emit) atomicAdd(L.rec_total, n_emit);
    if (L.dev_records && n_bytes) atomicAdd(L.rec_total + 2, n_bytes);
    if (any_over) atomicOr(&L.err[0], 1);
    if (any_unord) atomicOr(&L.err[1], 1);
    if (mover) atomicOr(&L.err[2], 1);
    if (any_aged) atomicOr(&L.err[3], 1);
  }
  if (W.chunk == W.n_chunks - 1) {  // the last chunk owns the group's lists: the pending set after its last event
    const int64_t t_end = L.b.ts[W.c1 - 1];
    const int ob = 1 - W.inb;
    int64_t* __restrict__ o_ts = pick(L.ent_ts, ob);
    int64_t* __restrict__ o_sq = pick(L.ent_seq, ob);
    int64_t* __restrict__ o_ky = pick(L.ent_key, ob);
    int n = 0;
    auto out = [&](int64_t t0, U ky, uint32_t sq) {
      if (dead(t0, t_end)) return;
      if (n >= L.rsmax) {
        overflow = 1;
        return;
      }
      const size_t o = gb + (size_t)n * WAVE + lane;
      o_ts[o] = t0;
      o_ky[o] = (int64_t)(uint64_t)ky;
      o_sq[o] = slast - (int64_t)(uint32_t)(llo - sq);
      ++n;
    };
    for (int i = 0; i < sn; ++i) {
      int64_t t0; U ky; uint32_t sq;
      sget(i, t0, ky, sq);
      out(t0, ky, sq);
    }
    for (int i = 0; i < ln; ++i) {
      int64_t t0; U ky; uint32_t sq;
      lget(lbot + i, t0, ky, sq);
      out(t0, ky, sq);
    }
    pick(L.st, ob)[W.g].n[lane] = n;
    if (wballot(overflow != 0) && lane == 0) atomicOr(&L.err[0], 1);
  }
}

}  // namespace sdh

template <int KK, int XM, int NF, int PM, bool FULL>
static void gate_launch_one(const sdh::RatchetLaunch* L, int SC, hipStream_t s) {
  const size_t lds = (size_t)sdh::GML * 64 * (FULL ? 16 : 12);
  hipLaunchKernelGGL((sdh::nfa_gate_kernel<KK, XM, NF, NF, PM, FULL>), dim3(L->n_items), dim3(64), lds, s, *L, SC);
}

// instantiations: the one-atom lazy form (the C2x family's), and the general form for wide batches
// (16-B records), several atoms, and out-of-order timestamps (FULL)
template <int KK, int XM>
static void gate_launch_atoms(const sdh::RatchetLaunch* L, int nf, int ng, int SC, int full, hipStream_t s) {
  constexpr int R = sdh::RMAXF0;
  if (full) {
    if (L->wide) gate_launch_one<KK, XM, R, 3, true>(L, SC, s);
    else gate_launch_one<KK, XM, R, 0, true>(L, SC, s);
  } else if (L->wide) {
    gate_launch_one<KK, XM, R, 3, false>(L, SC, s);
  } else if (nf <= 1 && ng <= 1) {
    gate_launch_one<KK, XM, 1, 0, false>(L, SC, s);
  } else {
    gate_launch_one<KK, XM, R, 0, false>(L, SC, s);
  }
}

template <int KK>
static void gate_launch_kk(int xm, const sdh::RatchetLaunch* L, int nf, int ng, int SC, int full, hipStream_t s) {
  switch (xm) {
    case 0: gate_launch_atoms<KK, 0>(L, nf, ng, SC, full, s); break;
    case 1: gate_launch_atoms<KK, 1>(L, nf, ng, SC, full, s); break;
    case 2: gate_launch_atoms<KK, 2>(L, nf, ng, SC, full, s); break;
    default: gate_launch_atoms<KK, 3>(L, nf, ng, SC, full, s); break;
  }
}

// K_gate launch over L->n_items items of gated groups (key kinds KK_F32 / KK_I32; xmask as
// sdh_launch_ratchet's; nf / ng: max f0 / g atoms; SC: spill entries per lane, a power of two)
extern "C" hipError_t sdh_launch_gate(int key_kind, int xmask, int full, int nf, int ng, int SC,
                                      const sdh::RatchetLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  if (SC < 1 || (SC & (SC - 1)) || nf > sdh::RMAXF0 || ng > sdh::RMAXF0) return hipErrorInvalidValue;
  const int xm = xmask == sdh::CM_GT ? 0 : xmask == (sdh::CM_GT | sdh::CM_EQ) ? 1 : xmask == sdh::CM_LT ? 2 : 3;
  switch (key_kind) {
    case sdh::KK_F32: gate_launch_kk<sdh::KK_F32>(xm, L, nf, ng, SC, full, s); break;
    case sdh::KK_I32: gate_launch_kk<sdh::KK_I32>(xm, L, nf, ng, SC, full, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// resident waves per CU of the K_gate instantiation
extern "C" int sdh_gate_occupancy(int nf, int ng) {
  int nb = 0;
  const size_t lds = (size_t)sdh::GML * 64 * 12;
  const hipError_t r = (nf <= 1 && ng <= 1)
                           ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                 &nb, sdh::nfa_gate_kernel<sdh::KK_F32, 0, 1, 1, 0, false>, 64, lds)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                 &nb, sdh::nfa_gate_kernel<sdh::KK_F32, 0, sdh::RMAXF0, sdh::RMAXF0, 0, false>, 64, lds);
  return r == hipSuccess ? nb : 0;
}
