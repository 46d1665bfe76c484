// seq_body.h -- K_seq: sequences as windows of consecutive events (kg::seq_window / kg::seq_match).
//
// A lane is a query; the wave's 64 queries share one shape (template q, scalar loads). Window
// starts are tiled by 64: the tile's events (64 + S - 1, tail rows first) are staged once in LDS,
// then every lane tests every start of the tile against its own constants -- all lanes read the
// same LDS word at a time (a broadcast). No per-query state exists beyond the stream's tail.
//
// The window test is the Spec's: SeqInterp (nfa_gen.hip) walks the shape's atoms / bytecode, a
// shape-compiled Spec (spec.hip, generated and compiled with hiprtc when the engine is created) is
// the same test as straight-line code with the lane's constants in registers.
#pragma once
#include "dev_common.h"

namespace sdh {

constexpr int SEQ_TILE = 64;
constexpr int SEQ_ROW = 3 + kg::GMAXNA;  // ts, seq, null bits, raw words (the widest row)

// a window over LDS rows of ROW words; a Spec sets kRow = 3 + the attributes its shape captures (the
// LDS a wave takes bounds the resident waves: C4's rows are 5 words, not 11).
// CLEAN: the tile has no null attribute and its timestamps are ordered and span no more than any
// lane's `within` -- no null test and no expiry test can fail, so both fold away. The window rows
// are wave-uniform, so those tests ran on the scalar unit (per start: a 64-bit |ts_i - ts_0| and a
// bit test per attribute read), which bound K_seq at ~78 % SALU issue.
template <int ROW, bool CLEAN = false>
struct LdsWinT {
  static constexpr bool kStagedConsts = false;
  const int64_t* base;  // row of window event 0
  __device__ int64_t lane_const(int) const { return 0; }
  __device__ int64_t ts(int p) const { return base[p * ROW]; }
  __device__ int64_t raw(int p, int j, bool = false) const { return base[p * ROW + 3 + j]; }
  __device__ bool null(int p, int j, bool = false) const {
    if constexpr (CLEAN) return false;
    else return (base[p * ROW + 2] >> j) & 1;
  }
  // state i's event more than `within` from the start event (StreamPreStateProcessor.isExpired)
  __device__ bool exp(int i, int64_t within) const {
    if constexpr (CLEAN) return false;
    else return dev::expired(ts(0), ts(i), within);
  }
};
using LdsWin = LdsWinT<SEQ_ROW>;
template <bool B>
struct SeqClean {
  static constexpr bool value = B;
};

template <class Spec>
__device__ __forceinline__ void seq_body(const SeqLaunch& L) {
  constexpr int ROW = Spec::kRow;
  using Win = LdsWinT<ROW>;
  __shared__ int64_t win[(SEQ_TILE + 8 + kg::GMAXS) * ROW];  // (+8: masked starts of the last group)
  const int lane = threadIdx.x;
  const int64_t it = dev::grid_item(L.xcd);  // (chunk-major: one chunk's groups are neighbours)
  if (it >= (int64_t)L.n_glist * L.n_chunks) return;
  const int gi = L.glist[it % L.n_glist];
  const int chunk = (int)(it / L.n_glist);
  const int qi = L.lane_q[(int64_t)gi * 64 + lane];
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[gi];
  const kg::GQuery* __restrict__ ql = L.queries + (qi >= 0 ? qi : L.group_tmpl[gi]);
  typename Spec::K k;
  Spec::load(k, ql);
  const int S = q->n_states;
  const int stream = L.b.stream;
  const int na = q->n_cap[stream];
  const int64_t within = ql->within;
  const int64_t qid = ql->qid;  // (a per-lane load in the loop would wait for the record stores)
  // the smallest `within` of the wave's live lanes (none: INT64_MAX), for the clean-tile test
  int64_t wmin = (qi >= 0 && within >= 0) ? within : INT64_MAX;
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t y = __shfl_xor(wmin, o);
    wmin = y < wmin ? y : wmin;
  }
  // window index w: tail rows 0 .. tail_len-1, then batch event w - tail_len. Start s is evaluated
  // by the batch holding its last event s + S - 1.
  const int64_t W = L.tail_len + L.b.n;
  const int64_t s_begin = L.tail_len - (S - 1) > 0 ? L.tail_len - (S - 1) : 0;
  const int64_t s_end = W - S + 1;
  int64_t lo = s_begin + (int64_t)chunk * L.chunk_len;
  int64_t hi = lo + L.chunk_len < s_end ? lo + L.chunk_len : s_end;
  using Out = dev::WaveOutT<Spec::kOutW>;
  __shared__ typename Out::Shared out_sh;
  Out o;
  o.g = dev::LaneOut{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  o.sh = &out_sh;
  o.init();
  unsigned long long nrec = 0;
  // one window row (event w of tail ++ batch) into registers: the next tile's rows are loaded
  // while the current tile is tested, and written to LDS after it
  struct Row {
    int64_t ts, seq, nb, v[kg::GMAXNA];
  };
  auto fetch = [&](int64_t w, Row& r) {
    r.nb = 0;
    if (w < L.tail_len) {
      const int64_t* tr = L.tail + w * SEQ_TW;
      r.ts = tr[0];
      r.seq = tr[1];
#pragma unroll
      for (int j = 0; j < kg::GMAXNA; ++j) {  // (constant indices: the row stays in registers)
        if (j >= na) break;
        const int a = q->cap_attr[stream][j];
        r.v[j] = tr[2 + a];
        r.nb |= (tr[2 + MAXATTR + a] != 0 ? 1ll : 0ll) << j;
      }
    } else {
      const int64_t e = w - L.tail_len;
      r.ts = L.b.ts[e];
      r.seq = L.b.seq_base + e;
#pragma unroll
      for (int j = 0; j < kg::GMAXNA; ++j) {
        if (j >= na) break;
        bool nl;
        r.v[j] = dev::raw_word(L.b, q->cap_attr[stream][j], e, nl);
        r.nb |= (nl ? 1ll : 0ll) << j;
      }
    }
  };
  auto put = [&](int p, const Row& r) {
    int64_t* row = win + p * ROW;
    row[0] = r.ts;
    row[1] = r.seq;
    row[2] = r.nb;
#pragma unroll
    for (int j = 0; j < kg::GMAXNA; ++j)
      if (j < na && j < ROW - 3) row[3 + j] = r.v[j];
  };
  // rows t0 + p for p = lane (and lane + 64 for the S - 1 rows past the tile) that exist
  const int64_t rows_end = hi + S - 1;  // one past the last window row any start of the chunk reads
  Row ra, rb;
  if (lo + lane < rows_end) fetch(lo + lane, ra);
  if (lane < S - 1 && lo + 64 + lane < rows_end) fetch(lo + 64 + lane, rb);
  const int words = 7 + 2 * S;  // (the wave's shape's)
  auto put_rec = [&](auto r, int s) {
    const Win wv{win + s * ROW};
    r[0] = words;
    r[1] = qid;
    r[2] = -1;
    r[3] = wv.base[(S - 1) * ROW];      // ts of the last event
    r[4] = wv.base[(S - 1) * ROW + 1];  // the triggering event's seq
    r[5] = 0;                               // one match per event per query
    r[6] = S | (stream << 16);
    for (int i = 0; i < S; ++i) {
      r[7 + 2 * i] = 1;
      r[8 + 2 * i] = wv.base[i * ROW + 1];
    }
  };
  // the narrow record (nfa_types.h, 24 B at S = 3 instead of 104) unless an offset or a distance
  // does not fit int32 (one record width per collective call: the emit is uniform)
  const bool nb_ok = L.b.n < (int64_t)INT32_MAX;
  const int nwords = nrec_seq_words(S);
  auto nar_ok = [&](int s) {
    const Win wv{win + s * ROW};
    return nb_ok && wv.base[(S - 1) * ROW + 1] - wv.base[1] <= (int64_t)INT32_MAX;
  };
  auto put_nrec = [&](auto r, int s) {
    const Win wv{win + s * ROW};
    const int64_t sq = wv.base[(S - 1) * ROW + 1];
    r[0] = nrec_pack(-(nwords + (NREC_KIND_SEQ << 16)), qid);
    r[1] = nrec_pack(sq - L.b.seq_base, S);
    for (int i = 0; i < S - 1; i += 2)
      r[2 + i / 2] = nrec_pack(sq - wv.base[i * ROW + 1], i + 1 < S - 1 ? sq - wv.base[(i + 1) * ROW + 1] : 0);
  };
  auto emit = [&](int s) {
    ++nrec;
    if (!L.write_records) return;
    if (!__ballot(!nar_ok(s))) o.emit_u(nwords, [&](auto r) { put_nrec(r, s); });
    else o.emit_u(words, [&](auto r) { put_rec(r, s); });
  };
  // a lane's matches among the tile's starts (mask m) in one collective call: its records are
  // contiguous, start order; the record counts take 7 ballots. (One call per 64 starts instead of per
  // 8: the call's wave-uniform bookkeeping -- ballots, the LDS buffer's counters, placement rounds --
  // ran on the scalar unit once per 8 starts, which bound C4 at 78 % SALU issue.)
  auto emit_tile = [&](uint64_t m) {
    const int nl = __popcll(m);
    nrec += nl;
    if (!L.write_records || __ballot(nl > 0) == 0) return;
    bool ok = true;
    for (uint64_t mm = m; mm; mm &= mm - 1) ok = ok && nar_ok(__builtin_ctzll(mm));
    if (!__ballot(!ok))
      o.emit_n(nl, nwords, [&](auto r0) {
        int kk = 0;
        for (uint64_t mm = m; mm; mm &= mm - 1, ++kk) put_nrec(r0 + kk * nwords, __builtin_ctzll(mm));
      }, true, 7);
    else
      o.emit_n(nl, words, [&](auto r0) {
        int kk = 0;
        for (uint64_t mm = m; mm; mm &= mm - 1, ++kk) put_rec(r0 + kk * words, __builtin_ctzll(mm));
      }, true, 7);
  };
  for (int64_t t0 = lo; t0 < hi; t0 += SEQ_TILE) {
    const int cnt = hi - t0 < SEQ_TILE ? (int)(hi - t0) : SEQ_TILE;
    if (t0 + lane < rows_end) put(lane, ra);
    if (lane < S - 1 && t0 + 64 + lane < rows_end) put(64 + lane, rb);
    // a clean tile (LdsWinT): no null bit in the rows its starts read, timestamps ordered, span <= wmin
    const bool nulls = __ballot((t0 + lane < rows_end && ra.nb != 0) ||
                                (lane < S - 1 && t0 + 64 + lane < rows_end && rb.nb != 0)) != 0;
    __syncthreads();
    const int nrows = cnt + S - 1;  // (rows_end bounds them: the chunk's starts read up to hi + S - 2)
    bool clean = false;
    if (!nulls) {
      bool bad = false;
      for (int p = lane; p + 1 < nrows; p += 64) bad |= win[(p + 1) * ROW] < win[p * ROW];
      // (ordered rows: last >= first, so the difference is exact as unsigned)
      clean = __ballot(bad) == 0 && (uint64_t)win[(nrows - 1) * ROW] - (uint64_t)win[0] <= (uint64_t)wmin;
    }
    const int64_t t1 = t0 + SEQ_TILE;  // prefetch the next tile's rows
    if (t1 < hi) {
      if (t1 + lane < rows_end) fetch(t1 + lane, ra);
      if (lane < S - 1 && t1 + 64 + lane < rows_end) fetch(t1 + 64 + lane, rb);
    }
    if (qi >= 0) {
      if constexpr (Spec::kBranchFree) {
        // 8 starts at a time, every state of each evaluated: their LDS reads overlap; starts past
        // cnt read rows of the LDS window that are stale or unset, and are masked off
        auto tile = [&](auto c) {
          using W = LdsWinT<ROW, decltype(c)::value>;
          uint64_t m = 0;
          for (int s0 = 0; s0 < cnt; s0 += 8) {
            uint32_t m8 = 0;
#pragma unroll
            for (int u = 0; u < 8; ++u)
              m8 |= (Spec::match(k, q, ql, within, W{win + (s0 + u) * ROW}) ? 1u : 0u) << u;
            m |= (uint64_t)m8 << s0;
          }
          if (cnt < 64) m &= (1ull << cnt) - 1ull;
          return m;
        };
        emit_tile(clean ? tile(SeqClean<true>{}) : tile(SeqClean<false>{}));
      } else {
        for (int s = 0; s < cnt; ++s)
          if (Spec::match(k, q, ql, within, Win{win + s * ROW})) emit(s);
      }
    }
    __syncthreads();
  }
  if (nrec) atomicAdd(L.rec_count, nrec);
  o.close();
  if (o.over) atomicOr(&L.err[2], 1);
}

}  // namespace sdh
