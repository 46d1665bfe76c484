// slab.h -- K_slab: sparse per-(query, partition key) partial tables for distinct-stream patterns
// (the C5 family, BASELINE configs[4]: 100K patterns x 1M keys). Shared by the device kernel
// (nfa_slab.hip) and the host cross-check (tests/native/slab_host.cpp, test infrastructure).
//
// Shapes (slab_lower.h decides): a PATTERN `[every] e1=S0[f0] -> X1 -> X2 ... [within T]` inside a
// partition, where every element X is a stream state `e=S[f]`, a count state `e=S[f]<min:max>`
// (1 <= min <= max <= SL_CMAX, never two counts in a row) or a logical pair `e=S[f] and|or e'=S'[f']`,
// and EVERY state reads its own stream. Filters may read the current event, e1 and any earlier slot
// (count slots at [0] / [last]).
//
// Why per-partial entries are exact (paths relative to core/query/input/stream/state/). With one
// processor per stream, an event reaches exactly one processor of the query (its receiver has one
// pre, PatternSingleProcessStreamReceiver), so the reference's per-key object graph reduces to a set
// of StateEvents each of which is in a few pending lists:
//   * e1 (StreamPreStateProcessor.processAndReturn:292-337, the start state never expires) holds one
//     armed partial; `every` re-arms it with a clone on every pass (StreamPostStateProcessor:53-72,
//     StateEventCloner:46-58), so each f0-passing event opens ONE new partial, which enters the next
//     element's newAndEvery list and is promoted before that element's stream is processed again
//     (two-phase add/update, R4; a different stream cannot run before the promotion);
//   * a stream / logical pre-processor walks its pending list and treats each partial on its own:
//     isExpired (:102-113), the filter over (partial, event), the post (StreamPost:53-72,
//     LogicalPost:59-87: AND forwards only with the partner slot filled, OR drops partials whose
//     partner is filled); a count pre (CountPreStateProcessor:53-93, no `within` check) appends,
//     filters, removes the last event on failure, forwards at len == min (CountPost:45-95) and drops
//     the partial once slot id+1 or id+2 is filled;
//   * so per (partial, event) the outcome depends on that partial and the event alone; the list
//     ORDER only fixes the emission order and the order in which partials arrive in the next list.
// An entry therefore stores one partial: per state its slot (sequence numbers; a count chain up to
// max), the captured attribute words later filters read, the `within` start time, per state an
// in-list bit, and per chain element its position in that element's list (the partial's rank in
// the reference's pending list: R18 emission index, and the order of arrivals in the next list).
//
// Entry words (uint32):
//   w0 flags   lane (0-5) | marker (6) | moved-this-event (7) | in-list bit per state id (8-15) |
//              count len per count ordinal (16-31, 4 bits each)
//   w1, w2     position in the list of the even / odd chain elements the partial is in (a partial is
//              in at most two elements' lists: a count and the element after it)
//   w3, w4     ts of e1 (the `within` start slot, start_ids == {0})
//   w5         null bits of the captured words
//   then per state its sequence numbers (2 words each; -1 = empty slot; a count: max of them) and
//   the captured words (a count slot: a first- and a last-event copy).
// A marker entry (flag 6, no partial) records that a non-`every` start state has fired for the
// instance (StreamPreStateProcessor.init:157-166 seeds it once per key, R3).
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif
#include "kgen.h"

namespace sdh {
namespace slab {

constexpr int SL_MAXS = kg::GMAXS;  // states per query
constexpr int SL_CMAX = 8;          // count <min:max> with max <= SL_CMAX
constexpr int SL_MAXCOUNT = 4;      // count states per query (4-bit lengths in the flags word)
constexpr int SL_MAXEW = 64;        // entry words
constexpr int SL_HDR = 6;           // flags, pos even, pos odd, ts0 lo, ts0 hi, null bits

enum : uint32_t { EF_LANE = 0x3fu, EF_MARKER = 0x40u, EF_MOVED = 0x80u };
KG_FN uint32_t in_bit(int state) { return 1u << (8 + state); }
constexpr uint32_t EF_INLIST = 0xff00u;

// one query shape's entry layout and chain structure (host-built, wave-uniform on the device)
struct Shape {
  int32_t S, EW, every, n_elem;
  int32_t kind[SL_MAXS];        // kg::K_STREAM / K_COUNT / K_LOGICAL
  int32_t elem[SL_MAXS];        // chain element of each state (e1 = element 0)
  int32_t partner[SL_MAXS], ltype[SL_MAXS], min[SL_MAXS], max[SL_MAXS], has_sel[SL_MAXS];
  int32_t cnt_ord[SL_MAXS];     // count states: nibble of their length in the flags word, else -1
  int32_t nxt[SL_MAXS][2];      // states of the element after this state's element (-1: none)
  int32_t drop[SL_MAXS][2];     // count states: ids whose filled slot drops the partial (id+1, id+2)
  int32_t proc[kg::GMAXSTREAM]; // the state stream s feeds, -1
  int32_t o_seq[SL_MAXS];       // first word of the state's sequence numbers (-1: not stored)
  int32_t o_cf[SL_MAXS], o_cl[SL_MAXS];  // first / last (count) copy of the captured words (-1: none)
  int32_t nb_f[SL_MAXS], nb_l[SL_MAXS];  // first null bit of those copies
  int32_t ncap[SL_MAXS];        // captured words per copy (the state stream's kg::GQuery::n_cap)
  int32_t pad[2];
  int8_t crank[kg::GMAXCODE];   // per instruction its rank among the shape's CONST ones (kg::LaneConsts)
};

// ---- entry accessors (E: uint32 pointer of one entry, contiguous words) ----
KG_FN int64_t get64(const uint32_t* e, int o) { return (int64_t)((uint64_t)e[o] | ((uint64_t)e[o + 1] << 32)); }
KG_FN void set64(uint32_t* e, int o, int64_t v) {
  e[o] = (uint32_t)(uint64_t)v;
  e[o + 1] = (uint32_t)((uint64_t)v >> 32);
}
KG_FN int lane_of(const uint32_t* e) { return (int)(e[0] & EF_LANE); }
KG_FN int count_len(const Shape& sh, const uint32_t* e, int st) {
  return (int)((e[0] >> (16 + 4 * sh.cnt_ord[st])) & 0xfu);
}
KG_FN void set_count_len(const Shape& sh, uint32_t* e, int st, int len) {
  const int b = 16 + 4 * sh.cnt_ord[st];
  e[0] = (e[0] & ~(0xfu << b)) | ((uint32_t)len << b);
}
KG_FN uint32_t pos_of(const uint32_t* e, int elem) { return e[1 + (elem & 1)]; }
KG_FN void set_pos(uint32_t* e, int elem, uint32_t p) { e[1 + (elem & 1)] = p; }
KG_FN int64_t ts0_of(const uint32_t* e) { return get64(e, 3); }
// slot `st` holds an event (the reference's StateEvent.streamEvents[st] != null)
KG_FN bool filled(const Shape& sh, const uint32_t* e, int st) {
  if (st == 0) return true;
  if (sh.kind[st] == kg::K_COUNT) return count_len(sh, e, st) > 0;
  return sh.o_seq[st] >= 0 && get64(e, sh.o_seq[st]) != -1;
}
KG_FN bool cap_null(const uint32_t* e, int bit) { return (e[5] >> bit) & 1u; }
// StreamPreStateProcessor.isExpired:102-113 for start_ids == {0}: Math.abs(e1.ts - ts) > within
KG_FN bool dev_expired(int64_t ts1, int64_t ts, int64_t within) {
  if (within < 0) return false;
  const int64_t d = (int64_t)((uint64_t)ts1 - (uint64_t)ts);
  const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

// the current event of a step: ts, global sequence number, the stream's captured words and null bits
struct Ev {
  int64_t ts, seq;
  const int64_t* w;  // word j at w[j * wstride]
  int wstride;
  uint32_t nul;
  KG_FN int64_t word(int j) const { return w[j * wstride]; }
  KG_FN bool null(int j) const { return (nul >> j) & 1u; }
};

KG_FN kg::Val typed_word(int res, int64_t raw, bool isnull) {
  kg::Val v{res, 1, 0};
  if (!isnull) {
    v.null = 0;
    v.bits = res == kg::T_INT ? (int64_t)(int32_t)raw : res == kg::T_FLOAT ? (int64_t)(uint32_t)raw : raw;
  }
  return v;
}

// copy `n` captured words of the event into words o.. and their null bits at nb..
KG_FN void capture(uint32_t* e, int o, int nb, int n, const Ev& ev) {
  for (int j = 0; j < n; ++j) {
    e[o + j] = (uint32_t)ev.word(j);  // captured types are <= 4 bytes (slab_lower.h checks)
    if (ev.null(j)) e[5] |= 1u << (nb + j);
    else e[5] &= ~(1u << (nb + j));
  }
}

// The reference's view of slot `a` at chain index `b` while state `st`'s filters run over partial e
// and the current event (StateEvent.getStreamEvent:138-182 through VariableExpressionExecutor):
// the state's own slot holds the current event (a count slot: appended to its chain of `len`).
// *where: 0 = null, 1 = the current event, 2 = a stored copy at word *o / null bit *nb.
KG_FN int slot_ref(const Shape& sh, const uint32_t* e, int st, int len, int a, int64_t b, int* o, int* nb) {
  if (a == st) {
    if (sh.kind[st] != kg::K_COUNT) return (b == 0 || b == -1) ? 1 : 0;
    if (b == -1 || (b == 0 && len == 0)) return 1;
    if (b == 0) { *o = sh.o_cf[st]; *nb = sh.nb_f[st]; return 2; }
    if (b == -2 && len > 0) { *o = sh.o_cl[st]; *nb = sh.nb_l[st]; return 2; }
    return 0;
  }
  if (!filled(sh, e, a)) return 0;
  if (sh.kind[a] == kg::K_COUNT) {
    if (b == 0) { *o = sh.o_cf[a]; *nb = sh.nb_f[a]; return 2; }
    if (b == -1) { *o = sh.o_cl[a]; *nb = sh.nb_l[a]; return 2; }
    return 0;
  }
  if (b == 0 || b == -1) { *o = sh.o_cf[a]; *nb = sh.nb_f[a]; return 2; }
  return 0;
}

// state st's filters (FilterProcessor.process:55-66 over the typed bytecode)
KG_FN bool filters_pass(const Shape& sh, const kg::GQuery* q, const kg::LaneConsts& lk, int st, const uint32_t* e,
                        int len, const Ev& ev) {
  const kg::GState& gs = q->st[st];
  for (int f = 0; f < gs.n_filt; ++f) {
    const kg::Val v = kg::eval_code_imm<kg::RegStack>(
        q, [&](int pc) { return lk.imm(pc, sh.crank[pc]); }, gs.fb[f], gs.fe[f],
        [&](const kg::GInsn& in) {
          int o = 0, nb = 0;
          const int w = slot_ref(sh, e, st, len, in.a, in.b, &o, &nb);
          if (w == 1) return typed_word(in.res, ev.word((int)in.imm), ev.null((int)in.imm));
          if (w == 2) return typed_word(in.res, (int64_t)e[o + (int)in.imm], cap_null(e, nb + (int)in.imm));
          return kg::Val{in.res, 1, 0};
        },
        [&](const kg::GInsn& in) {
          int o = 0, nb = 0;
          return slot_ref(sh, e, st, len, in.a, in.b, &o, &nb) == 0;
        });
    if (v.null || !v.bits) return false;
  }
  return true;
}

// the start state: does e1's filter pass the event? (its slot is the event; nothing else is read)
KG_FN bool start_pass(const Shape& sh, const kg::GQuery* q, const kg::LaneConsts& lk, const Ev& ev) {
  uint32_t dummy[SL_HDR] = {0, 0, 0, 0, 0, 0};
  return filters_pass(sh, q, lk, 0, dummy, 0, ev);
}

// A new partial opened by e1 at event ev: it joins the next element's lists at position `pos`
KG_FN void open_partial(const Shape& sh, uint32_t* e, int lane, uint32_t pos, const Ev& ev) {
  for (int w = 0; w < sh.EW; ++w) e[w] = 0;
  for (int i = 1; i < sh.S; ++i)
    if (sh.o_seq[i] >= 0) {
      const int n = sh.kind[i] == kg::K_COUNT ? sh.max[i] : 1;
      for (int k = 0; k < n; ++k) set64(e, sh.o_seq[i] + 2 * k, -1);
    }
  uint32_t fl = (uint32_t)lane;
  for (int k = 0; k < 2; ++k)
    if (sh.nxt[0][k] >= 0) fl |= in_bit(sh.nxt[0][k]);
  e[0] = fl;
  set_pos(e, 1, pos);
  set64(e, 3, ev.ts);
  set64(e, sh.o_seq[0], ev.seq);
  if (sh.o_cf[0] >= 0) capture(e, sh.o_cf[0], sh.nb_f[0], sh.ncap[0], ev);
}

enum : int { R_EMIT = 1, R_MOVE = 2, R_CHANGED = 4 };

// slot st of e <- the current event (a one-event slot)
KG_FN void fill_slot(const Shape& sh, uint32_t* e, int st, const Ev& ev) {
  if (sh.o_seq[st] >= 0) set64(e, sh.o_seq[st], ev.seq);
  if (sh.o_cf[st] >= 0) capture(e, sh.o_cf[st], sh.nb_f[st], sh.ncap[st], ev);
}

// the count states that drop a partial once slot st is filled (CountPreStateProcessor:60-66)
KG_FN void drop_counts(const Shape& sh, uint32_t* e, int st) {
  for (int c = 0; c < sh.S; ++c)
    if (sh.kind[c] == kg::K_COUNT && (sh.drop[c][0] == st || sh.drop[c][1] == st)) e[0] &= ~in_bit(c);
}

// One partial at one event of the stream that feeds state st (st > 0, the partial in st's list).
// Returns R_* bits: R_EMIT (the query's last post returned it: a match, trigger = this event),
// R_MOVE (it arrives in the next element's lists), R_CHANGED (the entry changed).
KG_FN int step(const Shape& sh, const kg::GQuery* q, const kg::LaneConsts& lk, int st, uint32_t* e, const Ev& ev,
               int64_t within) {
  if (!(e[0] & in_bit(st))) return 0;
  const int kind = sh.kind[st];
  if (kind == kg::K_COUNT) {  // CountPreStateProcessor.processAndReturn:53-93 + CountPost.process:45-71
    const int len = count_len(sh, e, st);
    if (!filters_pass(sh, q, lk, st, e, len, ev)) return 0;  // removeLastEvent: chain unchanged
    set64(e, sh.o_seq[st] + 2 * len, ev.seq);
    if (len == 0 && sh.o_cf[st] >= 0) capture(e, sh.o_cf[st], sh.nb_f[st], sh.ncap[st], ev);
    if (sh.o_cl[st] >= 0) capture(e, sh.o_cl[st], sh.nb_l[st], sh.ncap[st], ev);
    const int n = len + 1;
    set_count_len(sh, e, st, n);
    int r = R_CHANGED;
    if (n == sh.min[st]) {  // processMinCountReached:73-85
      if (sh.has_sel[st]) r |= R_EMIT;
      if (sh.nxt[st][0] >= 0) r |= R_MOVE;
    }
    if (n == sh.max[st] || (n == sh.min[st] && sh.has_sel[st])) e[0] &= ~in_bit(st);  // stateChanged
    return r;
  }
  // StreamPreStateProcessor.processAndReturn:292-337 / LogicalPreStateProcessor:133-178
  if (dev_expired(ts0_of(e), ev.ts, within)) {
    e[0] &= ~in_bit(st);
    return R_CHANGED;
  }
  const int pt = kind == kg::K_LOGICAL ? sh.partner[st] : -1;
  if (pt >= 0 && sh.ltype[st] == kg::L_OR && filled(sh, e, pt)) {
    e[0] &= ~in_bit(st);
    return R_CHANGED;
  }
  if (!filters_pass(sh, q, lk, st, e, 0, ev)) return 0;  // slot cleared, kept (PATTERN)
  e[0] &= ~in_bit(st);  // stateChanged: removed from this list
  fill_slot(sh, e, st, ev);
  drop_counts(sh, e, st);
  if (pt >= 0 && sh.ltype[st] == kg::L_AND && !filled(sh, e, pt)) return R_CHANGED;  // LogicalPost:63-66
  if (pt >= 0 && sh.ltype[st] == kg::L_OR) e[0] &= ~in_bit(pt);  // its next partner event drops it
  int r = R_CHANGED;
  if (sh.has_sel[st]) r |= R_EMIT;
  if (sh.nxt[st][0] >= 0) r |= R_MOVE;
  return r;
}

// match record words: [len, qid, key, ts, trigger seq, idx, S | stream << 16, (count, seqs...) x S]
KG_FN int record_words(const Shape& sh, const uint32_t* e, int st) {
  int w = 7;
  for (int j = 0; j < sh.S; ++j) {
    if (sh.kind[j] == kg::K_COUNT) w += 1 + count_len(sh, e, j);
    else w += 1 + ((j == st || filled(sh, e, j)) ? 1 : 0);
  }
  return w;
}
template <class R>  // R: a word pointer or a pointer-like record (dev::WaveOutT::Rec)
KG_FN void write_record(const Shape& sh, const uint32_t* e, int st, int words, int64_t qid, int64_t key, int64_t idx,
                        int stream, const Ev& ev, R r) {
  r[0] = words;
  r[1] = qid;
  r[2] = key;
  r[3] = ev.ts;
  r[4] = ev.seq;
  r[5] = idx;
  r[6] = sh.S | (stream << 16);
  int p = 7;
  for (int j = 0; j < sh.S; ++j) {
    if (sh.kind[j] == kg::K_COUNT) {
      const int n = count_len(sh, e, j);
      r[p++] = n;
      for (int k = 0; k < n; ++k) r[p++] = get64(e, sh.o_seq[j] + 2 * k);
    } else if (j == st) {
      r[p++] = 1;
      r[p++] = ev.seq;
    } else if (filled(sh, e, j)) {
      r[p++] = 1;
      r[p++] = get64(e, sh.o_seq[j]);
    } else {
      r[p++] = 0;
    }
  }
}

}  // namespace slab
}  // namespace sdh
