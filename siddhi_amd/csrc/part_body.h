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

// a count partial as f3 sees it: e1's words, the chain's first and last event words (entry words
// o_e1.., o_first.., o_last..) and their null bits in the flags word (16 / 24 / 32 + j)
struct PartEnt {
  const int64_t* p;  // entry word 0 of this lane (stride 64)
  int64_t fl;
  int o_e1, o_first, o_last;
  __device__ int64_t word(int x) const { return p[(int64_t)x * 64]; }
  __device__ int64_t e1(int j) const { return word(o_e1 + j); }
  __device__ int64_t first(int j) const { return word(o_first + j); }
  __device__ int64_t last(int j) const { return word(o_last + j); }
  __device__ bool e1_null(int j) const { return (fl >> (16 + j)) & 1; }
  __device__ bool first_null(int j) const { return (fl >> (24 + j)) & 1; }
  __device__ bool last_null(int j) const { return (fl >> (32 + j)) & 1; }
};

template <int KIND, class Spec>
__device__ __forceinline__ void part_body(const PartLaunch& L) {
  const int lane = threadIdx.x;
  const int item = blockIdx.x;
  if (item >= L.n_items) return;
  const int seg = item / L.gn, g = L.g0 + item % L.gn;
  const uint32_t kid = L.seg_kid[seg];
  if (kid == 0xFFFFFFFFu) return;  // null / foreign partition keys
  const int64_t e0 = L.seg_begin[seg], e1 = e0 + L.seg_len[seg];
  const int qi = L.lane_q[(int64_t)(L.group_base + g) * 64 + lane];
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[L.group_base + g];  // wave-uniform shape
  const kg::GQuery* __restrict__ ql = L.queries + (qi >= 0 ? qi : L.group_tmpl[L.group_base + g]);
  typename Spec::K k;
  Spec::load(k, ql, L);
  const int stream = L.b.stream;
  const int ncap = q->n_cap[stream];
  const int64_t within = ql->within;
  const int64_t key = L.key_of_id[kid];
  const int64_t bw = PK_HDR + (int64_t)L.cap * L.ew;
  const int64_t block = (int64_t)kid * L.groups + g;
  const int cb = L.cur[kid];
  const int64_t* __restrict__ in = L.st + ((int64_t)cb * L.blocks + block) * bw * 64 + lane;
  int64_t* __restrict__ st = L.st + ((int64_t)(1 - cb) * L.blocks + block) * bw * 64 + lane;
  if (g == 0 && lane == 0) L.nxt[kid] = 1 - cb;
  const int ew = L.ew;
  auto W = [&](int64_t i) -> int64_t& { return st[i * 64]; };
  auto E = [&](int kk, int w) -> int64_t& { return st[(PK_HDR + (int64_t)kk * ew + w) * 64]; };

  // the lane's table: input buffer -> output block (the working copy)
  int n = (int)in[0];
  int64_t hdr1 = in[64];
  for (int kk = 0; kk < n; ++kk)
    for (int w = 0; w < ew; ++w) E(kk, w) = in[(PK_HDR + (int64_t)kk * ew + w) * 64];

  // the key's events, staged 64 at a time (one coalesced index load and one gather per lane), then
  // read by broadcast: ts, seq, null bits and the captured words
  __shared__ int64_t t_ts[64], t_seq[64], t_w[kg::GMAXNA][64];
  __shared__ uint32_t t_nul[64];
  __shared__ dev::WaveOut::Shared out_sh;
  dev::WaveOut o;
  o.g = dev::LaneOut{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  o.sh = &out_sh;
  o.init();
  unsigned long long nrec = 0;
  bool cap_over = false;
  const bool live = qi >= 0;
  const int sA = L.sA;
  int F = (int)(hdr1 & 0xffffffff), side = (int)(hdr1 >> 32);  // logical: filled prefix and its side

  for (int64_t t0 = e0; t0 < e1; t0 += 64) {
    const int cnt = e1 - t0 < 64 ? (int)(e1 - t0) : 64;
    if (lane < cnt) {
      const int64_t e = L.ev_idx[t0 + lane];
      t_ts[lane] = L.b.ts[e];
      t_seq[lane] = L.b.seq_base + e;
      uint32_t nb = 0;
      for (int j = 0; j < ncap; ++j) {
        bool nl;
        t_w[j][lane] = dev::raw_word(L.b, q->cap_attr[stream][j], e, nl);
        if (nl) nb |= 1u << j;
      }
      t_nul[lane] = nb;
    }
    __syncthreads();
    for (int te = 0; te < cnt && live; ++te) {
      const int64_t seq = t_seq[te];
      const int64_t ts = t_ts[te];
      const PartEv ev{&t_w[0][te], t_nul[te]};
      const bool f1 = Spec::f1(k, q, ql, L, ev);
      int64_t idx = 0;  // emission index of this (instance, event): the pending-list order

      if (KIND == PK_OR || KIND == PK_AND) {
        const bool fb = Spec::fb(k, q, ql, L, ev), fa = Spec::fa(k, q, ql, L, ev);
        // expiry of every partial (both sides' isExpired see the same event timestamp)
        if (within >= 0) {
          int w = 0, Fw = 0;
          for (int kk = 0; kk < n; ++kk) {
            if (dev::expired(E(kk, 0), ts, within)) continue;
            if (w != kk)
              for (int x = 0; x < ew; ++x) E(w, x) = E(kk, x);
            if (kk < F) ++Fw;
            ++w;
          }
          n = w;
          F = Fw;
          if (F == 0) side = 0;
        }
        auto emit = [&](int kk, int64_t a_seq, int64_t b_seq) {  // a_seq / b_seq: -1 = empty slot
          ++nrec;
          if (!L.write_records) return;
          const int words = 7 + 2 + (a_seq >= 0 ? 2 : 1) + (b_seq >= 0 ? 2 : 1);
          int64_t* r = o.reserve(words);
          if (!r) return;
          r[0] = words;
          r[1] = ql->qid;
          r[2] = key;
          r[3] = ts;
          r[4] = seq;
          r[5] = idx++;
          r[6] = 3 | (stream << 16);
          int p = 7;
          for (int s = 0; s < 3; ++s) {
            const int64_t v = s == 0 ? E(kk, 1) : s == sA ? a_seq : b_seq;
            if (v >= 0) {
              r[p++] = 1;
              r[p++] = v;
            } else {
              r[p++] = 0;
            }
          }
        };
        if (KIND == PK_OR) {
          // side B first (its processor runs first), then side A; either empties the list
          if (fb || fa) {
            for (int kk = 0; kk < n; ++kk) emit(kk, fb ? -1 : seq, fb ? seq : -1);
            n = 0;
          }
        } else if (fb || fa) {
          // AND. B pass: partials filled on A complete (a = fill, b = x); empty ones get b = x.
          // A pass: partials filled on B (old and new) complete (a = x). Both passes walk the list
          // in creation order and every completed partial precedes every surviving one, so one walk
          // in list order emits in the reference's order.
          int w = 0;
          for (int kk = 0; kk < n; ++kk) {
            const bool filled = kk < F;
            int64_t aseq = -1, bseq = -1;
            if (filled && side == 1) aseq = E(kk, 2);
            if (filled && side == 2) bseq = E(kk, 2);
            if (fb && bseq < 0) bseq = seq;  // B pass: the partials whose B slot is empty
            if (fa && aseq < 0) aseq = seq;  // A pass: those whose A slot is empty (B-filled too)
            if (aseq >= 0 && bseq >= 0) {
              emit(kk, aseq, bseq);
              continue;
            }
            // survivor: exactly one side filled
            if (w != kk)
              for (int x = 0; x < ew; ++x) E(w, x) = E(kk, x);
            E(w, 2) = aseq >= 0 ? aseq : bseq;
            ++w;
          }
          n = w;
          F = w;
          side = n == 0 ? 0 : (fb ? 2 : 1);
        }
        if (f1) {  // e1 opens a partial; it joins both sides' lists at the next event
          if (n < L.cap) {
            E(n, 0) = ts;
            E(n, 1) = seq;
            E(n, 2) = -1;
            ++n;
          } else {
            cap_over = true;
          }
        }
      } else {  // PK_COUNT
        const bool f2 = Spec::f2(k, q, ql, L, ev);
        const int cmin = q->st[1].min, cmax = q->st[1].max;  // this shape's <min:max>
        const int o_e1 = 3 + L.cmax, o_first = o_e1 + L.n_e1, o_last = o_first + L.n_first;
        int w = 0;
        for (int kk = 0; kk < n; ++kk) {
          int64_t fl = E(kk, 2);
          int len = (int)(fl & 0xff);
          bool inL3 = (fl >> 8) & 1;
          bool done = false;
          // e3 (processed first): expiry, then f3 over the partial as it is now
          if (inL3) {
            if (dev::expired(E(kk, 0), ts, within)) {
              inL3 = false;
            } else if (Spec::f3(k, q, ql, L, ev, PartEnt{&E(kk, 0), fl, o_e1, o_first, o_last})) {
              done = true;  // completed: removed from e3's list now, from the count list at this event
              ++nrec;
              if (L.write_records) {
                const int words = 7 + 2 + 1 + len + 2;
                int64_t* r = o.reserve(words);
                if (r) {
                  r[0] = words;
                  r[1] = ql->qid;
                  r[2] = key;
                  r[3] = ts;
                  r[4] = seq;
                  r[5] = idx++;
                  r[6] = 3 | (stream << 16);
                  r[7] = 1;
                  r[8] = E(kk, 1);
                  r[9] = len;
                  for (int c = 0; c < len; ++c) r[10 + c] = E(kk, 3 + c);
                  r[10 + len] = 1;
                  r[11 + len] = seq;
                }
              }
            }
          }
          if (done) continue;
          // count state: a partial with len < max appends every f2-passing event
          if (len < cmax && f2) {
            E(kk, 3 + len) = seq;
            const int64_t nb = (int64_t)(ev.nul & 0xff);
            if (len == 0) {
              for (int j = 0; j < L.n_first; ++j) E(kk, o_first + j) = ev.word(j);
              fl = (fl & ~(0xffll << 24)) | (nb << 24);
            }
            for (int j = 0; j < L.n_last; ++j) E(kk, o_last + j) = ev.word(j);
            fl = (fl & ~(0xffll << 32)) | (nb << 32);
            ++len;
            if (len == cmin) inL3 = true;  // CountPost: next.addState at n == min (visible next event)
          }
          if (!inL3 && len >= cmax) continue;  // in neither list any more
          fl = (fl & ~0x1ffll) | (int64_t)len | ((int64_t)inL3 << 8);
          if (w != kk)
            for (int x = 0; x < ew; ++x) E(w, x) = E(kk, x);
          E(w, 2) = fl;
          ++w;
        }
        n = w;
        if (f1) {
          if (n < L.cap) {
            E(n, 0) = ts;
            E(n, 1) = seq;
            for (int j = 0; j < L.n_e1; ++j) E(n, o_e1 + j) = ev.word(j);
            E(n, 2) = (int64_t)(ev.nul & 0xff) << 16;  // e1's null bits
            ++n;
          } else {
            cap_over = true;
          }
        }
      }
    }
    __syncthreads();  // the tile is rewritten next
  }
  W(0) = n;
  W(1) = (int64_t)(uint32_t)F | ((int64_t)side << 32);
  if (nrec) atomicAdd(L.rec_count, nrec);
  if (cap_over) atomicOr(&L.err[0], 1);
  o.close();
  if (o.over) atomicOr(&L.err[2], 1);
}

}  // namespace sdh
