// nfa_part.hip -- K_part: shape-specialised kernels for partitioned count / logical patterns (the C3
// family), on compact per-(query, key) partial tables instead of K_gen's object arenas.
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
// wave-uniform: one event's captured words staged in LDS, read by broadcast); one lane = one
// (query, key) instance; its partials live in the output state block (lane-interleaved, so the
// k-th partial of every lane is one coalesced 512-B access per word). The state is double-buffered
// across pushes: an entry-capacity overflow re-runs the push exactly with a larger table.
#include <hip/hip_runtime.h>

#include "kgen.h"
#include "nfa_types.h"

namespace sdh {

namespace {

__device__ __forceinline__ int64_t event_word(const StreamBatch& b, int attr, int64_t e, bool& isnull) {
  const void* p = nullptr;
  const uint8_t* nl = nullptr;
  int w = 4;
#pragma unroll
  for (int c = 0; c < MAXATTR; ++c)
    if (c == attr) {
      p = b.col[c];
      nl = b.nul[c];
      w = b.width[c];
    }
  isnull = nl && nl[e];
  if (w == 8) return ((const int64_t*)p)[e];
  if (w == 4) return (int64_t)((const int32_t*)p)[e];
  return (int64_t)((const uint8_t*)p)[e];
}

__device__ __forceinline__ bool expired(int64_t ts1, int64_t ts, int64_t within) {
  if (within < 0) return false;
  const int64_t d = (int64_t)((uint64_t)ts1 - (uint64_t)ts);
  const int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

__device__ __forceinline__ kg::Val typed(const kg::GInsn& in, int64_t raw, bool isnull) {
  kg::Val v{in.res, 1, 0};
  if (!isnull) {
    v.null = 0;
    v.bits = in.res == kg::T_INT ? (int64_t)(int32_t)raw : in.res == kg::T_FLOAT ? (int64_t)(uint32_t)raw : raw;
  }
  return v;
}

// K_gen-format match records + record index (as nfa_gen.hip LaneOut)
struct POut {
  int64_t* out;
  int64_t cap;
  unsigned long long* next;
  bool ring;
  int64_t* rec_off;
  int64_t rec_cap;
  unsigned long long* rec_next;
  bool over = false;
  __device__ int64_t* reserve(int words) {
    const unsigned long long o = atomicAdd(next, (unsigned long long)words);
    if (ring) return out + (int64_t)(o % (unsigned long long)(cap - GEN_RING_MARGIN));
    if ((int64_t)(o + words) > cap) {
      over = true;
      return nullptr;
    }
    const unsigned long long r = atomicAdd(rec_next, 1ull);
    if ((int64_t)r >= rec_cap) {
      over = true;
      return nullptr;
    }
    rec_off[r] = (int64_t)o;
    return out + o;
  }
};

}  // namespace

template <int KIND>
__global__ __launch_bounds__(64) void nfa_part_kernel(PartLaunch L) {
  const int lane = threadIdx.x;
  const int item = blockIdx.x;
  if (item >= L.n_items) return;
  const int seg = item / L.groups, g = item % L.groups;
  const uint32_t kid = L.seg_kid[seg];
  if (kid == 0xFFFFFFFFu) return;  // null / foreign partition keys
  const int64_t e0 = L.seg_begin[seg], e1 = e0 + L.seg_len[seg];
  const int qi = L.lane_q[(int64_t)(L.group_base + g) * 64 + lane];
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[L.group_base + g];  // wave-uniform shape
  const kg::GQuery* __restrict__ ql = L.queries + (qi >= 0 ? qi : L.group_tmpl[L.group_base + g]);
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
  // the lane's table works in LDS for its first `cl` entries ([entry][word][lane]: conflict-free,
  // one bank per lane) and in the output block beyond them
  extern __shared__ int64_t part_lds[];
  const int cl = L.cl;
  auto W = [&](int64_t i) -> int64_t& { return st[i * 64]; };
  auto E = [&](int k, int w) -> int64_t& {
    return k < cl ? part_lds[((int64_t)k * ew + w) * 64 + lane] : st[(PK_HDR + (int64_t)k * ew + w) * 64];
  };

  // the lane's table: input buffer -> working copy (LDS, then the output block)
  int n = (int)in[0];
  int64_t hdr1 = in[64];
  for (int k = 0; k < n; ++k)
    for (int w = 0; w < ew; ++w) E(k, w) = in[(PK_HDR + (int64_t)k * ew + w) * 64];

  // the key's events, staged 64 at a time (one coalesced index load and one gather per lane), then
  // read by broadcast: ts, seq, null bits and the captured words
  __shared__ int64_t t_ts[64], t_seq[64], t_w[kg::GMAXNA][64];
  __shared__ uint32_t t_nul[64];
  POut o{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  unsigned long long nrec = 0;
  bool cap_over = false;
  const bool live = qi >= 0;
  const kg::GState& s0 = q->st[0];
  // logical: the sides' states; count: the count state 1 and e3 = 2
  const int sA = L.sA, sB = L.sB;
  const kg::GState& sa = q->st[KIND == PK_COUNT ? 1 : sA];
  const kg::GState& sb = q->st[KIND == PK_COUNT ? 2 : sB];
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
      t_w[j][lane] = event_word(L.b, q->cap_attr[stream][j], e, nl);
      if (nl) nb |= 1u << j;
    }
    t_nul[lane] = nb;
  }
  __syncthreads();
  for (int te = 0; te < cnt && live; ++te) {
    const int64_t seq = t_seq[te];
    const int64_t ts = t_ts[te];
    const uint32_t ev_null = t_nul[te];
    auto evw = [&](int j) -> int64_t { return t_w[j][te]; };
    // an event-only filter of state `st` (FilterProcessor.java:55-66 over the typed bytecode)
    auto ev_filter = [&](const kg::GState& gs, int sid) -> bool {
      for (int f = 0; f < gs.n_filt; ++f) {
        const kg::Val v = kg::eval_code<kg::RegStack>(
            q, ql, gs.fb[f], gs.fe[f],
            [&](const kg::GInsn& in) {  // the state's own one-event slot: index 0 / CURRENT only
              const bool here = in.a == sid && (in.b == 0 || in.b == -1);
              return typed(in, here ? evw(in.imm) : 0, !here || ((ev_null >> in.imm) & 1u));
            },
            [&](const kg::GInsn& in) { return !(in.a == sid && (in.b == 0 || in.b == -1)); });
        if (v.null || !v.bits) return false;
      }
      return true;
    };
    const bool f1 = ev_filter(s0, 0);
    int64_t idx = 0;  // emission index of this (instance, event): the pending-list order

    if (KIND == PK_OR || KIND == PK_AND) {
      const bool fb = ev_filter(sb, sB), fa = ev_filter(sa, sA);
      // expiry of every partial (both sides' isExpired see the same event timestamp)
      if (within >= 0) {
        int w = 0, Fw = 0;
        for (int kk = 0; kk < n; ++kk) {
          if (expired(E(kk, 0), ts, within)) continue;
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
        // A pass: partials filled on B (old and new) complete (a = x). Both passes walk the list in
        // creation order and every completed partial precedes every surviving one, so one walk in
        // list order emits in the reference's order.
        int w = 0;
        for (int kk = 0; kk < n; ++kk) {
          const bool filled = kk < F;
          int64_t aseq = -1, bseq = -1;
          if (filled && side == 1) aseq = E(kk, 2);
          if (filled && side == 2) bseq = E(kk, 2);
          if (fb && bseq < 0) bseq = seq;  // B pass: the partials whose B slot is empty
          if (fa && aseq < 0) aseq = seq;  // A pass: those whose A slot is empty (B-filled ones too)
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
      const bool f2 = ev_filter(sa, 1);
      const kg::GState& s3 = sb;
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
          if (expired(E(kk, 0), ts, within)) {
            inL3 = false;
          } else {
            bool pass = true;
            for (int f = 0; f < s3.n_filt && pass; ++f) {
              const kg::Val v = kg::eval_code<kg::RegStack>(
                  q, ql, s3.fb[f], s3.fe[f],
                  [&](const kg::GInsn& in) {
                    if (in.a == 2) {  // the current event
                      const bool here = in.b == 0 || in.b == -1;
                      return typed(in, here ? evw(in.imm) : 0, !here || ((ev_null >> in.imm) & 1u));
                    }
                    if (in.a == 0) {  // e1
                      const bool here = in.b == 0 || in.b == -1;
                      return typed(in, here ? E(kk, o_e1 + in.imm) : 0, !here || ((fl >> (16 + in.imm)) & 1));
                    }
                    // e2: the chain's first (0) or last (CURRENT) event
                    const bool first = in.b == 0;
                    return typed(in, first ? E(kk, o_first + in.imm) : E(kk, o_last + in.imm),
                                 ((fl >> ((first ? 24 : 32) + in.imm)) & 1));
                  },
                  [&](const kg::GInsn&) { return false; });  // e1, e2 (len >= min >= 1), cur exist
              pass = !v.null && v.bits;
            }
            if (pass) {
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
        }
        if (done) continue;
        // count state: a partial with len < max appends every f2-passing event
        if (len < cmax && f2) {
          E(kk, 3 + len) = seq;
          const int64_t nb = (int64_t)(ev_null & 0xff);
          if (len == 0) {
            for (int j = 0; j < L.n_first; ++j) E(kk, o_first + j) = evw(j);
            fl = (fl & ~(0xffll << 24)) | (nb << 24);
          }
          for (int j = 0; j < L.n_last; ++j) E(kk, o_last + j) = evw(j);
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
          int64_t fl = (int64_t)(ev_null & 0xff) << 16;  // e1's null bits
          for (int j = 0; j < L.n_e1; ++j) E(n, o_e1 + j) = evw(j);
          E(n, 2) = fl;
          ++n;
        } else {
          cap_over = true;
        }
      }
    }
  }
  __syncthreads();  // the tile is rewritten next
  }
  for (int k = 0; k < n && k < cl; ++k)  // LDS-resident entries back to the output block
    for (int w = 0; w < ew; ++w) st[(PK_HDR + (int64_t)k * ew + w) * 64] = part_lds[((int64_t)k * ew + w) * 64 + lane];
  W(0) = n;
  W(1) = (int64_t)(uint32_t)F | ((int64_t)side << 32);
  if (nrec) atomicAdd(L.rec_count, nrec);
  if (cap_over) atomicOr(&L.err[0], 1);
  if (o.over) atomicOr(&L.err[2], 1);
}

}  // namespace sdh

extern "C" hipError_t sdh_launch_part(const sdh::PartLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  const size_t lds = (size_t)L->cl * L->ew * 64 * 8;  // dynamic: the LDS-resident table entries
  switch (L->kind) {
    case sdh::PK_OR: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_OR>, dim3(L->n_items), dim3(64), lds, s, *L); break;
    case sdh::PK_AND: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_AND>, dim3(L->n_items), dim3(64), lds, s, *L); break;
    default: hipLaunchKernelGGL(sdh::nfa_part_kernel<sdh::PK_COUNT>, dim3(L->n_items), dim3(64), lds, s, *L);
  }
  return hipGetLastError();
}
