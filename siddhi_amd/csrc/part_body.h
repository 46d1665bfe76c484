// part_body.h -- K_part: partitioned count / logical patterns on compact partial tables (the C3
// family); the kernel body, instantiated by nfa_part.hip with the interpreted filters
// (PartInterp) and by spec.hip with a shape's filters compiled to straight-line code.
//
// Shapes (kpart_shape in engine.hip decides; every filter in the IR's typed bytecode):
//   PK_OR / PK_AND  every e1=S[f1] -> e2=S[f2] or|and e3=S[f3] [within T]     (f1, f2, f3 event-only)
//   PK_COUNT        every e1=S[f1] -> e2=S[f2] <min:max> -> e3=S[f3] [within T]
//                   (f1, f2 event-only; f3 may read e1, e2[0], e2[last] and the current event)
//
// Why compact tables are exact -- the reference's object graph for these shapes reduces to one list
// of partials in creation order (paths relative to core/query/input/stream/state/):
//   * every partial is created by e1 (StreamPostStateProcessor.java:53-72; the every-clone re-arms
//     e1, R13) and enters the next state's lists at the next event (two-phase add/update, R4);
//   * the processors of one stream run in reverse registration order (R5): for the logical pair the
//     side registered second (sB, the logical's first element) before sA, then e1; for the count
//     chain e3, then the count state, then e1;
//   * f1, f2 (and f3 of the logical shapes) read only the current event, so an event either passes
//     them for every partial of an instance or for none: LogicalPreStateProcessor.processAndReturn
//     (:133-178) then fills the same side of every pending partial at once. For AND the partials
//     whose side is filled are always a prefix of the list filled on ONE side (an event passing the
//     other side empties that class, LogicalPostStateProcessor.java:59-87), so a partial is
//     (e1, fill) plus the list's (F, side); for OR every pending partial completes together;
//   * for the count chain a partial appends every f2-passing event while it is in the count state's
//     list (CountPreStateProcessor.java:53-93, no `within` check there, R9) and joins e3's list when
//     its chain reaches min (CountPostStateProcessor.java:45-95), so the e3 list is the creation-
//     ordered subset of partials with len >= min; e3 (StreamPreStateProcessor.java:292-337) sees the
//     chain as it is at that event (the object is shared: aliasing, SURVEY §7 hard part 1);
//   * `within` (isExpired :102-113) is checked at every event for every partial a stream / logical
//     pre-processor holds, so expiry is exact for any timestamp order.
// The matches are K_gen-format records (nfa_gen.hip) with the emission index in the reference's
// pending-list order, so the device match table orders them exactly (R18).
//
// Mapping to CDNA4: one wave = 64 same-shape queries x one partition key (the key's events in order,
// wave-uniform: staged 64 at a time in LDS, read by broadcast); one lane = one (query, key)
// instance; its partials live in the output state block (lane-interleaved, so the k-th partial of
// every lane is one coalesced 512-B access per word). The state is double-buffered across pushes:
// an entry-capacity overflow re-runs the push exactly with a larger table.
#pragma once
#include "dev_common.h"

namespace sdh {

// the current event of a K_part step: captured words and null bits from the LDS staging tile
struct PartEv {
  const int64_t* w;  // t_w[0] + te: word j at w[j * 64]
  uint32_t nul;
  __device__ int64_t word(int j) const { return w[j * 64]; }
  __device__ bool null(int j) const { return (nul >> j) & 1u; }
};

// entry word offsets of a count partial: chain words 3 .. 3+cmax-1, then e1's, the chain's first
// and its last event's captured words (those f3 reads)
struct PartOffs {
  int cmax, n_e1, n_first, n_last;
  __device__ int o_e1() const { return 3 + cmax; }
  __device__ int o_first() const { return 3 + cmax + n_e1; }
  __device__ int o_last() const { return 3 + cmax + n_e1 + n_first; }
};

// A partial's words wherever they live: GRef in the lane's global state block (stride 64 words),
// RRef in registers (a row of the lane's register table; an index that is not a compile-time
// constant selects among the row's words, so the row never leaves VGPRs)
struct GRef {
  int64_t* p;
  __device__ int64_t get(int w) const { return p[(int64_t)w * 64]; }
  __device__ void set(int w, int64_t v) const { p[(int64_t)w * 64] = v; }
};
template <int EW>
struct RRef {
  int64_t* p;
  __device__ int64_t get(int w) const {
    int64_t v = p[0];
#pragma unroll
    for (int x = 1; x < EW; ++x) v = (w == x) ? p[x] : v;
    return v;
  }
  // (value selects and unconditional stores: conditional stores to different words get merged into
  // one store through a selected pointer, which keeps the row out of registers)
  __device__ void set(int w, int64_t v) const {
#pragma unroll
    for (int x = 0; x < EW; ++x) p[x] = (w == x) ? v : p[x];
  }
};

// a count partial as f3 sees it: e1's words, the chain's first and last event words and their null
// bits in the flags word (16 / 24 / 32 + j)
template <class Ref>
struct PartEnt {
  Ref e;
  int64_t fl;
  PartOffs of;
  __device__ int64_t e1(int j) const { return e.get(of.o_e1() + j); }
  __device__ int64_t first(int j) const { return e.get(of.o_first() + j); }
  __device__ int64_t last(int j) const { return e.get(of.o_last() + j); }
  __device__ bool e1_null(int j) const { return (fl >> (16 + j)) & 1; }
  __device__ bool first_null(int j) const { return (fl >> (24 + j)) & 1; }
  __device__ bool last_null(int j) const { return (fl >> (32 + j)) & 1; }
};

template <class Ref>
__device__ __forceinline__ PartEnt<Ref> part_ent(const Ref& e, int64_t fl, const PartOffs& of) {
  return PartEnt<Ref>{e, fl, of};
}

// The lane's partial table: entries 0 .. RC-1 in registers (RC = 0: none), the rest in its global
// state block; every walk visits the entries in list (creation) order
template <int RC, int EW>
struct PartTable {
  int64_t r[RC > 0 ? RC : 1][EW];
  int64_t* g;  // entry kk word w at g[(kk * ew + w) * 64]
  int ew;
  __device__ GRef gref(int kk) const { return GRef{g + (int64_t)kk * ew * 64}; }
  // body(kk, ref) for kk = 0 .. n-1
  template <class F>
  __device__ void each(int n, F&& body) {
    if constexpr (RC > 0) {
#pragma unroll
      for (int kk = 0; kk < RC; ++kk)
        if (kk < n) body(kk, RRef<EW>{r[kk]});
    }
    for (int kk = RC; kk < n; ++kk) body(kk, gref(kk));
  }
  // entry w <- the `words` words of src (w <= the index src was read from)
  template <class Ref>
  __device__ void put(int w, const Ref& src, int words) {
    if constexpr (RC > 0) {
      if (w < RC) {
        int64_t v[EW];
#pragma unroll
        for (int x = 0; x < EW; ++x) v[x] = src.get(x);
#pragma unroll
        for (int t = 0; t < RC; ++t)
#pragma unroll
          for (int x = 0; x < EW; ++x) r[t][x] = (w == t && x < words) ? v[x] : r[t][x];
        return;
      }
    }
    const GRef d = gref(w);
    for (int x = 0; x < words; ++x) d.set(x, src.get(x));
  }
  // word x of entry kk
  __device__ int64_t get(int kk, int x) const {
    if constexpr (RC > 0) {
      if (kk < RC) {
        int64_t v = r[0][0];
#pragma unroll
        for (int t = 0; t < RC; ++t)
#pragma unroll
          for (int y = 0; y < EW; ++y) v = (kk == t && x == y) ? r[t][y] : v;
        return v;
      }
    }
    return gref(kk).get(x);
  }
  // one word of entry w
  __device__ void set(int w, int x, int64_t v) {
    if constexpr (RC > 0) {
      if (w < RC) {
#pragma unroll
        for (int t = 0; t < RC; ++t)
#pragma unroll
          for (int y = 0; y < EW; ++y) r[t][y] = (w == t && x == y) ? v : r[t][y];
        return;
      }
    }
    gref(w).set(x, v);
  }
};

// A count partial's hot words in registers -- ts, seq, flags, then e1's, the chain's first and last
// event's captured words (what f3 and the chain updates read) -- with its chain of seqs (written
// once per appended event, read once by a match) in the lane's global block. get / set take the
// entry's word index (PartOffs layout), so f3 reads it as PartEnt reads any entry.
template <int HMAX>
struct HotRef {
  int64_t* h;   // [HMAX] registers: word w < 3 at h[w], word o_e1 + j at h[3 + j] (HMAX 0: none, all global)
  int64_t* g;   // the entry's global words (word w at g[w * 64])
  int o_e1;
  __device__ int slot(int w) const { return w < 3 ? w : 3 + (w - o_e1); }
  __device__ int64_t get(int w) const {
    if (HMAX == 0 || (w >= 3 && w < o_e1)) return g[(int64_t)w * 64];
    const int s = slot(w);
    int64_t v = h[0];
#pragma unroll
    for (int x = 1; x < HMAX; ++x) v = (s == x) ? h[x] : v;
    return v;
  }
  __device__ void set(int w, int64_t v) const {
    if (HMAX == 0 || (w >= 3 && w < o_e1)) {
      g[(int64_t)w * 64] = v;
      return;
    }
    const int s = slot(w);
#pragma unroll
    for (int x = 0; x < HMAX; ++x) h[x] = (s == x) ? v : h[x];
  }
};

#ifdef SDH_PART_PROF  // phase clocks (measurement builds only: SDH_PART_PROF=1 at engine creation)
#define PPROF_T(v) const unsigned long long v = clock64()
#define PPROF_ADD(i, d) (prof_acc[i] += (d))
#else
#define PPROF_T(v) ((void)0)
#define PPROF_ADD(i, d) ((void)0)
#endif

template <int KIND, class Spec>
__device__ __forceinline__ void part_body(const PartLaunch& L) {
#ifdef SDH_PART_PROF
  unsigned long long prof_acc[6] = {0, 0, 0, 0, 0, 0};
#endif
  PPROF_T(c_start);
  constexpr int RC = Spec::kRegEntries, EW = Spec::kEW;
  const int lane = threadIdx.x;
  const int item = (int)dev::grid_item(L.xcd);
  if (item >= L.n_items) return;
  const int seg = item / L.gn, g = L.g0 + item % L.gn;
  const uint32_t kid = L.seg_kid[seg];
  if (kid == 0xFFFFFFFFu) return;  // null / foreign partition keys
  const int64_t e0 = L.seg_begin[seg], e1 = e0 + L.seg_len[seg];
  const int qi = L.lane_q[(int64_t)(L.group_base + g) * 64 + lane];
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[L.group_base + g];  // wave-uniform shape
  const kg::GQuery* __restrict__ ql = L.queries + (qi >= 0 ? qi : L.group_tmpl[L.group_base + g]);
  // the lane's query id, `within` and constants from the group's lane-constant table (one coalesced
  // row per value; kg::LaneConsts), loaded once: a per-lane global load inside the event loop would
  // wait (vmcnt is in order) for every record store issued before it
  const int64_t* __restrict__ lcol = L.lconst + ((int64_t)(L.group_base + g) * L.lc_slots) * 64 + lane;
  typename Spec::K k;
  Spec::load(k, ql, L, lcol);
  const PartOffs of = Spec::offs(L);
  const int stream = L.b.stream;
  const int ncap = q->n_cap[stream];
  const int64_t within = lcol[kg::LC_WITHIN * 64];
  const int64_t qid = lcol[kg::LC_QID * 64];
  const int cmin = q->st[1].min, cmax = q->st[1].max;  // PK_COUNT: this shape's <min:max>
  const int64_t key = L.key_of_id[kid];
  const int ew = RC > 0 ? EW : L.ew;
  const int64_t bw = PK_HDR + (int64_t)L.cap * ew;
  const int64_t block = (int64_t)kid * L.groups + g;
  const int cb = L.cur[kid];
  const int64_t* __restrict__ in = L.st + ((int64_t)cb * L.blocks + block) * bw * 64 + lane;
  int64_t* __restrict__ st = L.st + ((int64_t)(1 - cb) * L.blocks + block) * bw * 64 + lane;
  if (g == 0 && lane == 0) L.nxt[kid] = 1 - cb;

  // the lane's table: input buffer -> registers (first RC entries) and the output block (the rest)
  PartTable<RC, EW> tab;
  tab.g = st + PK_HDR * 64;
  tab.ew = ew;
  int n = (int)in[0];
  const int64_t hdr1 = in[64];
  if constexpr (KIND != PK_COUNT) {  // (the count tables are read entry by entry, count_tile below)
    const GRef src{const_cast<int64_t*>(in) + PK_HDR * 64};
    for (int kk = 0; kk < n; ++kk) {
      const GRef e{src.p + (int64_t)kk * ew * 64};
      if (kk < RC) tab.put(kk, e, ew);
      else
        for (int w = 0; w < ew; ++w) tab.gref(kk).set(w, e.get(w));
    }
  }

  // the key's events, staged 64 at a time (one coalesced index load and one gather per lane), then
  // read by broadcast: ts, seq, null bits and the captured words
  // (LDS per wave bounds the resident waves: the staging holds the shape's captured words only, and
  // the Spec sizes the output buffer)
  using Out = dev::WaveOutT<Spec::kOutW, true>;  // (swizzled LDS records: 4- to 8-word records)
  __shared__ int64_t t_ts[64], t_seq[64], t_w[Spec::kNA][64];
  __shared__ uint32_t t_nul[64];
  __shared__ typename Out::Shared out_sh;
  Out o;
  o.g = dev::LaneOut{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  o.sh = &out_sh;
  o.init();
  unsigned long long nrec = 0;
  bool cap_over = false;
  const bool live = qi >= 0;
  const int sA = L.sA;
  int F = (int)(hdr1 & 0xffffffff), side = (int)(hdr1 >> 32);  // logical: filled prefix and its side

  // ---- PK_COUNT, entry-major: each partial is loaded once per event tile, run through the tile's
  // events in registers (its chain appended to its global slot), and stored once, compacted in
  // creation order; the partials the tile's events open follow, each from the event after its own.
  // A partial's fate depends on the events and its own words only (f1 / f2 read the event, f3 the
  // event and the partial), so this is the event-major walk of the reference (every event visits
  // the e3 list, then the count list, then e1) reordered, with the same result: a partial matches
  // at the first event it completes on, and the matches of one event keep the pending-list order
  // (emission index = e1's seq, increasing along the list). (The OR / AND tables above stay
  // event-major: their state is small and their output is per event.)
  const bool nb_ok = L.b.n < (int64_t)INT32_MAX;  // batch offsets fit a narrow record's int32
  auto count_tile = [&](int cnt, bool first_tile) {
    // the hot words in registers (shape-compiled kernels), or in the entry's global slot (the
    // interpreter, whose rows are GMAXNA wide)
    constexpr int HMAX = Spec::kHotRegs ? 3 + 3 * Spec::kNA : 0;
    const int nh = 3 + of.n_e1 + of.n_first + of.n_last;
    auto hot_word = [&](int x) { return x < 3 ? x : of.o_e1() + x - 3; };
    uint64_t m1 = 0, m2 = 0;  // the tile's events passing f1 / f2 (this lane's query)
    if (live)
      for (int te = 0; te < cnt; ++te) {
        const PartEv ev{&t_w[0][te], t_nul[te]};
        if (Spec::f1(k, q, ql, L, ev)) m1 |= 1ull << te;
        if (Spec::f2(k, q, ql, L, ev)) m2 |= 1ull << te;
      }
    int wmax = n;
    for (int o2 = 32; o2 > 0; o2 >>= 1) wmax = max(wmax, __shfl_xor(wmax, o2));
    const int64_t* __restrict__ src = (first_tile ? in : st) + PK_HDR * 64;
    int64_t* __restrict__ dst = st + PK_HDR * 64;
    int wpos = 0;             // entries kept so far: slots 0 .. wpos-1 of dst
    // one partial per lane and call (collective: the call's record emit): the lane's entry kk held
    // before the tile (kk >= 0), or the one event tc opens (kk < 0); has: the lane has it
    auto run = [&](bool has, int kk, int tc) {
      // no slot for it: the push re-runs exactly with a larger table. (The entry-major walk counts the
      // partials that survive the tile, not those alive at the event that opened this one -- the
      // event-major rule's count -- so the re-run can fire on a different push than it once did;
      // the matches are the same either way, test_kpart_table_growth_reruns_exactly)
      if (has && wpos >= L.cap) {
        cap_over = true;
        has = false;
      }
      int64_t h[HMAX > 0 ? HMAX : 1];
#pragma unroll
      for (int x = 0; x < (HMAX > 0 ? HMAX : 1); ++x) h[x] = 0;
      int64_t* gd = dst + (int64_t)wpos * ew * 64;  // the partial's slot if it survives the tile
      const HotRef<HMAX> e{h, gd, of.o_e1()};
      int te0 = cnt, len = 0;
      bool inL3 = false;
      int64_t fl = 0;
      if (has && kk < 0) {  // opened by event tc: in the lists from the next event on
        const PartEv ev{&t_w[0][tc], t_nul[tc]};
        e.set(0, t_ts[tc]);
        e.set(1, t_seq[tc]);
        for (int j = 0; j < of.n_e1; ++j) e.set(of.o_e1() + j, ev.word(j));
        fl = (int64_t)(ev.nul & 0xff) << 16;  // e1's null bits
        te0 = tc + 1;
      } else if (has) {
        const int64_t* gs = src + (int64_t)kk * ew * 64;
        if constexpr (HMAX > 0) {
#pragma unroll
          for (int x = 0; x < HMAX; ++x)
            if (x < nh) h[x] = gs[(int64_t)hot_word(x) * 64];
        } else if (gs != gd) {
          for (int x = 0; x < nh; ++x) gd[(int64_t)hot_word(x) * 64] = gs[(int64_t)hot_word(x) * 64];
        }
        fl = e.get(2);
        len = (int)(fl & 0xff);
        inL3 = (fl >> 8) & 1;
        if (gs != gd)
          for (int c = 0; c < len; ++c) gd[(int64_t)(3 + c) * 64] = gs[(int64_t)(3 + c) * 64];
        te0 = live ? 0 : cnt;
      }
      bool alive = has && te0 < cnt;
      int done = -1;  // the event the partial completes on
      // (wave-uniform bounds: from the earliest first event of the wave's partials, until none lives)
      int tstart = alive ? te0 : cnt;
      for (int o2 = 32; o2 > 0; o2 >>= 1) tstart = min(tstart, __shfl_xor(tstart, o2));
      for (int te = tstart; te < cnt; ++te) {
        if (!__ballot(alive)) break;
        if (!alive || te < te0) continue;
        const PartEv ev{&t_w[0][te], t_nul[te]};
        // e3 first: expiry, then f3 over the partial as it is now
        if (inL3) {
          if (dev::expired(e.get(0), t_ts[te], within)) {
            inL3 = false;
          } else if (Spec::f3(k, q, ql, L, ev, part_ent(e, fl, of))) {
            done = te;
            alive = false;
            continue;
          }
        }
        // count state: a partial with len < max appends every f2-passing event
        if (len < cmax && ((m2 >> te) & 1)) {
          gd[(int64_t)(3 + len) * 64] = t_seq[te];
          const int64_t nb = (int64_t)(ev.nul & 0xff);
          if (len == 0) {
            for (int j = 0; j < of.n_first; ++j) e.set(of.o_first() + j, ev.word(j));
            fl = (fl & ~(0xffll << 24)) | (nb << 24);
          }
          for (int j = 0; j < of.n_last; ++j) e.set(of.o_last() + j, ev.word(j));
          fl = (fl & ~(0xffll << 32)) | (nb << 32);
          ++len;
          if (len == cmin) inL3 = true;  // CountPost: next.addState at n == min (visible next event)
        }
        if (!inL3 && len >= cmax) alive = false;  // in neither list any more
      }
      if (done >= 0) ++nrec;
      if (L.write_records && __ballot(done >= 0)) {
        // the narrow record (nfa_types.h) when e1's distance fits int32, else the K_gen record
        // [words, qid, key, ts, seq, idx, 3 | stream, (1, e1), (len, chain...), (1, seq)]
        const int64_t sq = done >= 0 ? t_seq[done] : 0;
        const int64_t e1s = e.get(1);
        const bool nar = nb_ok && sq - e1s <= (int64_t)INT32_MAX;
        const int words = nar ? nrec_count_words(len) : 7 + 2 + 1 + len + 2;
        o.emit_n(done >= 0 ? 1 : 0, words, [&](auto r) {
          if (nar) {
            r[0] = nrec_pack(-(words + 0x10000), qid);
            r[1] = nrec_pack(sq - L.b.seq_base, (int64_t)kid);
            r[2] = nrec_pack(sq - e1s, len);
            for (int c = 0; c < len; c += 2)
              r[3 + c / 2] = nrec_pack(sq - gd[(int64_t)(3 + c) * 64], c + 1 < len ? sq - gd[(int64_t)(4 + c) * 64] : 0);
            return;
          }
          r[0] = words;
          r[1] = qid;
          r[2] = key;
          r[3] = t_ts[done];
          r[4] = sq;
          r[5] = e1s;  // emission index: e1's seq (the pending-list order)
          r[6] = 3 | (stream << 16);
          r[7] = 1;
          r[8] = e1s;
          r[9] = len;
          for (int c = 0; c < len; ++c) r[10 + c] = gd[(int64_t)(3 + c) * 64];
          r[10 + len] = 1;
          r[11 + len] = sq;
        });
      }
      // kept: alive at the tile's end, or not run at all (opened by the tile's last event, or a lane
      // without a query)
      if (has && (alive || (done < 0 && te0 >= cnt))) {
        e.set(2, (fl & ~0x1ffll) | (int64_t)len | ((int64_t)inL3 << 8));
        if constexpr (HMAX > 0) {
#pragma unroll
          for (int x = 0; x < HMAX; ++x)
            if (x < nh) gd[(int64_t)hot_word(x) * 64] = h[x];
        }
        ++wpos;
      }
    };
    // the entries held before the tile all start at its first event; the new ones, grouped by the
    // event that opens them, start together too (a wave's lanes run the same events)
    for (int kk = 0; kk < wmax; ++kk) run(kk < n, kk, 0);
    for (int tc = 0; tc < cnt; ++tc)
      if (__ballot((m1 >> tc) & 1)) run((m1 >> tc) & 1, -1, tc);
    n = wpos;
  };

  PPROF_T(c_setup);
  PPROF_ADD(0, c_setup - c_start);
  for (int64_t t0 = e0; t0 < e1; t0 += 64) {
    PPROF_T(c_t0);
    const int cnt = e1 - t0 < 64 ? (int)(e1 - t0) : 64;
    if (lane < cnt) {
      // (a key-ordered copy of the batch makes the tile's reads contiguous: L.sorted)
      const int64_t e = L.ev_idx[t0 + lane], p = L.sorted ? t0 + lane : e;
      t_ts[lane] = L.b.ts[p];
      t_seq[lane] = L.b.seq_base + e;
      uint32_t nb = 0;
      for (int j = 0; j < ncap; ++j) {
        bool nl = false;
        if (j < Spec::kNA) t_w[j][lane] = dev::raw_word(L.b, q->cap_attr[stream][j], p, nl);
        if (nl) nb |= 1u << j;
      }
      t_nul[lane] = nb;
    }
    __syncthreads();
    PPROF_T(c_t1);
    PPROF_ADD(1, c_t1 - c_t0);
    if constexpr (KIND == PK_COUNT) {
      count_tile(cnt, t0 == e0);
    } else {
    for (int te = 0; te < cnt && live; ++te) {
      const int64_t seq = t_seq[te];
      const int64_t ts = t_ts[te];
      const PartEv ev{&t_w[0][te], t_nul[te]};
      const bool f1 = Spec::f1(k, q, ql, L, ev);
      int64_t idx = 0;  // emission index of this (instance, event): the pending-list order

      if constexpr (KIND == PK_OR || KIND == PK_AND) {
        const bool fb = Spec::fb(k, q, ql, L, ev), fa = Spec::fa(k, q, ql, L, ev);
        // expiry of every partial (both sides' isExpired see the same event timestamp)
        if (within >= 0) {
          int w = 0, Fw = 0;
          tab.each(n, [&](int kk, const auto& e) {
            if (dev::expired(e.get(0), ts, within)) return;
            if (w != kk) tab.put(w, e, 3);
            if (kk < F) ++Fw;
            ++w;
          });
          n = w;
          F = Fw;
          if (F == 0) side = 0;
        }
        // one match record at r: [words, qid, key, ts, seq, idx, 3 | stream, (1, seq) | (0) per slot]
        // (a_seq / b_seq -1: empty slot)
        auto put_rec = [&](auto r, int words, int64_t my_idx, int64_t e1seq, int64_t a_seq, int64_t b_seq) {
          r[0] = words;
          r[1] = qid;
          r[2] = key;
          r[3] = ts;
          r[4] = seq;
          r[5] = my_idx;
          r[6] = 3 | (stream << 16);
          int p = 7;
          for (int s = 0; s < 3; ++s) {
            const int64_t v = s == 0 ? e1seq : s == sA ? a_seq : b_seq;
            if (v >= 0) {
              r[p++] = 1;
              r[p++] = v;
            } else {
              r[p++] = 0;
            }
          }
        };
        // the narrow record (nfa_types.h): slots by state id, 0 = e1, sA = side A, the other side B
        auto put_nrec = [&](auto r, int64_t e1seq, int64_t a_seq, int64_t b_seq) {
          const int64_t s1 = sA == 1 ? a_seq : b_seq, s2 = sA == 1 ? b_seq : a_seq;
          r[0] = nrec_pack(-NREC_ORAND_WORDS, qid);
          r[1] = nrec_pack(seq - L.b.seq_base, (int64_t)kid);
          r[2] = nrec_pack(seq - e1seq, s1 >= 0 ? seq - s1 : (int64_t)INT32_MIN);
          r[3] = nrec_pack(s2 >= 0 ? seq - s2 : (int64_t)INT32_MIN, 0);
        };
        // narrow unless a lane's oldest partial is 2^31 events back (one record width per call: the
        // collective emit is uniform)
        auto narrow_ok = [&](int c) {
          return !__ballot(c > 0 && !(nb_ok && seq - tab.get(0, 1) <= (int64_t)INT32_MAX));
        };
        // The lane's matches of this event are the first c partials of its list (see the two cases
        // below): their records go out in one collective reservation, record kk at r0 + kk * words
        // with emission index kk (the pending-list order; the narrow form's index is e1's seq, the
        // same order)
        (void)idx;
        if constexpr (KIND == PK_OR) {
          // side B first (its processor runs first), then side A; either empties the list
          if (fb || fa) {
            nrec += n;
            if (L.write_records) {
              const int64_t as = fb ? -1 : seq, bs = fb ? seq : -1;  // words: 7 + 2 + 2 + 1
              if (narrow_ok(n))
                o.emit_n(n, NREC_ORAND_WORDS, [&](auto r0) {
                  tab.each(n, [&](int kk, const auto& e) { put_nrec(r0 + kk * NREC_ORAND_WORDS, e.get(1), as, bs); });
                }, true);
              else
                o.emit_n(n, 12, [&](auto r0) {
                  tab.each(n, [&](int kk, const auto& e) { put_rec(r0 + kk * 12, 12, kk, e.get(1), as, bs); });
                }, true);
            }
            n = 0;
          }
        } else if (fb || fa) {
          // AND. B pass: partials filled on A complete (a = fill, b = x); empty ones get b = x.
          // A pass: partials filled on B (old and new) complete (a = x). Both passes walk the list
          // in creation order and every completed partial precedes every surviving one: with both
          // sides passing all n complete, with one side the F partials filled on the other side.
          const int c = (fa && fb) ? n : ((fb && side == 1) || (fa && side == 2)) ? F : 0;
          nrec += c;
          if (L.write_records) {
            const bool nar = narrow_ok(c);
            const int words = nar ? NREC_ORAND_WORDS : 13;  // (wide: 7 + 2 + 2 + 2)
            o.emit_n(c, words, [&](auto r0) {
              tab.each(c, [&](int kk, const auto& e) {
                const bool filled = kk < F;
                const int64_t aseq = (filled && side == 1) ? e.get(2) : seq;
                const int64_t bseq = (filled && side == 2) ? e.get(2) : seq;
                if (nar) put_nrec(r0 + kk * NREC_ORAND_WORDS, e.get(1), aseq, bseq);
                else put_rec(r0 + kk * 13, 13, kk, e.get(1), aseq, bseq);
              });
            }, true);
          }
          int w = 0;
          tab.each(n, [&](int kk, const auto& e) {
            if (kk < c) return;
            const bool filled = kk < F;
            int64_t aseq = -1, bseq = -1;
            if (filled && side == 1) aseq = e.get(2);
            if (filled && side == 2) bseq = e.get(2);
            if (fb && bseq < 0) bseq = seq;  // B pass: the partials whose B slot is empty
            if (fa && aseq < 0) aseq = seq;  // A pass: those whose A slot is empty (B-filled too)
            // survivor: exactly one side filled
            e.set(2, aseq >= 0 ? aseq : bseq);
            if (w != kk) tab.put(w, e, 3);
            ++w;
          });
          n = w;
          F = w;
          side = n == 0 ? 0 : (fb ? 2 : 1);
        }
        if (f1) {  // e1 opens a partial; it joins both sides' lists at the next event
          if (n < L.cap) {
            tab.set(n, 0, ts);
            tab.set(n, 1, seq);
            tab.set(n, 2, -1);
            ++n;
          } else {
            cap_over = true;
          }
        }
      }
    }
    }
    __syncthreads();  // the tile is rewritten next
    PPROF_T(c_t2);
    PPROF_ADD(2, c_t2 - c_t1);
    PPROF_ADD(4, cnt);
  }
  PPROF_T(c_loop);
  // register entries back to the output block
  if constexpr (RC > 0 && KIND != PK_COUNT) {
#pragma unroll
    for (int kk = 0; kk < RC; ++kk)
      if (kk < n)
        for (int w = 0; w < ew; ++w) tab.gref(kk).set(w, tab.r[kk][w]);
  }
  st[0] = n;
  st[64] = (int64_t)(uint32_t)F | ((int64_t)side << 32);
  o.close();
  if (nrec) atomicAdd(L.rec_count, nrec);
  if (cap_over) atomicOr(&L.err[0], 1);
  if (o.over) atomicOr(&L.err[2], 1);
#ifdef SDH_PART_PROF
  PPROF_T(c_end);
  PPROF_ADD(3, c_end - c_loop);
  PPROF_ADD(5, 1);
  if (lane == 0 && L.prof)
    for (int i = 0; i < 6; ++i) atomicAdd(&L.prof[i], prof_acc[i]);
#endif
}

}  // namespace sdh
