// nfa_gen.hip -- K_gen: the general NFA step, one lane per query instance (query, partition key),
// plus the device-side partition routing that feeds it.
//
// Mapping to CDNA4: a wave is 64 instances that see the SAME event sequence -- 64 queries of one
// partition for one key (or 64 unpartitioned queries of one stream) -- so every event is read at
// one uniform address by the whole wave. Each lane runs the reference's processor logic
// (kgen.h: pending / newAndEvery lists, StateEvent + StreamEvent-chain pools, mark/sweep) over its
// instance arena in HBM. Arenas are lane-interleaved ([block][word][lane]) so that lanes touching the
// same logical field coalesce into one 256-B access. Matches go to lane-private output chunks
// (one atomic per 4 KiB chunk) and are ordered by the host (R18 sort key).
//
// Partition routing (PartitionStreamReceiver.java:80-281, R19): key = the partition attribute's
// value (String.valueOf identity on raw words, NaN canonical); null keys drop the event. Keys get
// dense ids from a device hash table (open addressing, CAS on the key word); events are grouped by
// key with a stable radix sort of (key id, event index), so each key's events keep their order.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "dev_common.h"
#include "seq_body.h"

namespace sdh {

using dev::gpick;
using dev::LaneOut;
using dev::raw_word;

template <int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void nfa_gen_kernel(GenLaunch L) {
  const int lane = threadIdx.x;
  const int item = (int)dev::grid_item(L.xcd);
  if (item >= L.n_items) return;
  int seg = item / L.groups, g = item % L.groups;
  if (L.glist) {  // unpartitioned: a subset of the set's groups (K_seq runs the others)
    seg = item / L.n_glist;
    g = L.glist[item % L.n_glist];
  }
  int64_t e0 = 0, e1 = L.b.n;
  uint32_t kid = 0;
  if (L.sweep) {  // every known key's clone walks the whole batch (timers), processing its own events
    kid = (uint32_t)seg;
    if ((int64_t)kid >= L.n_keys) return;
  } else if (L.seg_begin) {
    kid = L.seg_kid[seg];
    if (kid == 0xFFFFFFFFu) return;  // events with a null partition key
    e0 = L.seg_begin[seg];
    e1 = e0 + L.seg_len[seg];
  }
  const int qi = L.lane_q[(int64_t)(L.group_base + g) * 64 + lane];
  if (qi < 0) return;
  // wave-uniform shape template (scalar loads) + the lane's own query (constants)
  const kg::GQuery* __restrict__ q = L.queries + L.group_tmpl[L.group_base + g];
  const kg::GQuery* __restrict__ ql = L.queries + qi;
  // a query that does not read the stream still sees time pass if it has absent states
  const bool reads = q->recv_n[L.b.stream] != 0;
  if (!reads && q->lay.TQ == 0) return;
  int64_t block = L.block_base + (int64_t)kid * L.groups + g;
  int32_t* a32 = L.a32;
  int64_t* a64 = L.a64;
  int64_t w0 = e0;  // first event replayed (w0 < e0: look-back, nothing emitted)
  if (L.ev_chunks > 1) {
    e0 = (int64_t)seg * L.chunk_len;
    e1 = e0 + L.chunk_len < L.b.n ? e0 + L.chunk_len : L.b.n;
    w0 = e0;
    if (seg > 0) {  // fresh instance in scratch, rebuilt from the look-back window
      block = (int64_t)(seg - 1) * L.groups + g;
      a32 = L.s32;
      a64 = L.s64;
      w0 = e0 - (q->n_states - 1);
      for (int w = 0; w < q->lay.n32; ++w) a32[(block * L.B32 + w) * 64 + lane] = 0;
      for (int w = 0; w < q->lay.n64; ++w) a64[(block * L.B64 + w) * 64 + lane] = 0;
    }
  }
  kg::Ctx c;
  c.bind(q, ql);
  c.w32 = a32 + block * L.B32 * 64 + lane;
  c.w64 = a64 + block * L.B64 * 64 + lane;
  c.stride = 64;
  // dynamic LDS (sized in sdh_launch_gen): the current event's captured words (wave-uniform), the hot
  // words of the item (kgen.h Ctx::h32/h64), [word][lane] -- sized to the launch's largest shape so
  // LDS does not cap occupancy
  extern __shared__ int64_t gen_lds[];
  int64_t* evv = gen_lds;
  c.h64 = gen_lds + kg::GMAXNA + lane;
  c.h32 = (int32_t*)(gen_lds + kg::GMAXNA + (1 + L.hot_nu) * 64) + lane;
  c.hstride = 64;
  c.hs = L.hot_s;
  c.load_hot();
  c.ev_val = evv;
  c.pins = c.h32 + (int64_t)3 * L.hot_s * 64;  // [4][lane] after the hot words
  c.err = kg::GE_OK;
  c.capk = 0;
  c.npin = 0;
  c.n_ret = 0;
  c.stream = L.b.stream;
  const int64_t key = L.key_of_id ? L.key_of_id[kid] : -1;
  // PartitionRuntime.cloneIfNotExist / QueryRuntime.init: seed (a sweep seeds a clone at its key's
  // first event); only top-level runtimes are start()ed (SiddhiAppRuntime.start)
  auto seed = [&]() {
    c.init_instance();
    if (!L.key_of_id) c.start_instance(L.start_ts);
    c.i32(q->lay.o_init) = 1;
  };
  if (!L.sweep && c.i32(q->lay.o_init) == 0) seed();
  LaneOut o{L.out, L.out_cap, L.out_next, L.write_records == 2, L.rec_off, L.rec_cap, L.rec_next};
  const int S = q->n_states;
  const int ncap = q->n_cap[c.stream];
  unsigned long long nrec = 0;
  int64_t idx = 0;
  const int64_t fpos = L.fan_pos ? (int64_t)L.fan_pos[kid] << 32 : 0;
  bool live = true;
  // a match record [len, qid, key, ts, trigger seq, idx, S | stream << 16, (count, seqs...) x S];
  // a timer's record carries stream 0xFFFF and its sort time (kgen.h fire_timers) in idx
  auto emit = [&](const kg::Ctx& cx, int se) {
    if (!live) return;
    int words = 7;
    for (int i = 0; i < S; ++i) {
      words += 1;
      for (int n = cx.slot(se, i); n >= 0; n = cx.nd_next(n)) ++words;
    }
    ++nrec;
    if (!L.write_records) return;
    int64_t* r = o.reserve(words);
    if (!r) return;
    r[0] = words;
    r[1] = ql->qid;
    r[2] = key;
    r[3] = cx.se_ts(se);
    r[4] = cx.seq;
    if (cx.in_timer) {
      r[5] = cx.timer_ts;
      r[6] = S | (0xFFFFll << 16);
    } else {
      r[5] = fpos | idx++;
      r[6] = S | (c.stream << 16);
    }
    int w = 7;
    for (int i = 0; i < S; ++i) {
      const int cw = w++;
      int64_t cnt = 0;
      for (int n = cx.slot(se, i); n >= 0; n = cx.nd_next(n)) {
        r[w++] = cx.nd_seq(n);
        ++cnt;
      }
      r[cw] = cnt;
    }
  };
  // One walk, one call site each for the timers and the interpreter (the interpreter is inlined per
  // call site). Plain: the key's events [w0, e1). Whole-batch sweep: every batch event passes time,
  // the key's own events are received. Indexed sweep (ordered batch, pm = ts): only the key's own
  // events and the timer stops -- a timer due at d fires at the first batch event whose time reaches
  // d (binary search of pm), with that event's seq and time, exactly where the whole walk fires it.
  const bool indexed = L.sweep && L.pm;
  const bool timers = !L.no_timers;  // (a chunk push fired its timers before its first event)
  const int32_t sg = indexed && L.kseg ? L.kseg[kid] : -1;
  const int64_t sb = sg >= 0 ? L.seg_begin[sg] : 0, sl = sg >= 0 ? L.seg_len[sg] : 0;
  int64_t j = 0, pos = 0;  // indexed: next own event, first batch event whose timers may still fire
  for (int64_t k = w0; c.err == kg::GE_OK;) {
    int64_t e;
    bool own;
    const bool inited = !L.sweep || c.i32(q->lay.o_init) != 0;
    if (indexed) {
      const int64_t eo = j < sl ? L.ev_idx[sb + j] : L.b.n - 1;
      if (eo < 0) break;  // (an empty batch)
      const int64_t d = inited && timers ? c.next_due() : 0x7fffffffffffffffLL;
      if (d <= L.b.ts[eo] && pos <= eo) {  // a timer stop at or before the next own event
        int64_t lo = pos, hi = eo;
        while (lo < hi) {
          const int64_t m = (lo + hi) >> 1;
          if (L.pm[m] < d) lo = m + 1;
          else hi = m;
        }
        e = lo;
        own = false;
        pos = e;
      } else if (j < sl) {
        e = eo;
        own = true;
        ++j;
        // a timer the event itself schedules fires at a later event (the whole-batch walk fires
        // timers before it receives), never at this one
        pos = e + 1;
      } else {
        break;
      }
    } else {
      if (k >= e1) break;
      live = k >= e0;
      e = L.ev_idx ? L.ev_idx[k] : k;
      ++k;
      // a sweep passes time at other keys' events; a fan-out stream's events are every key's
      own = !L.sweep || L.fan_pos || (L.ev_kid && L.ev_kid[e] == kid);
    }
    c.seq = L.b.seq_base + e;
    c.ts = L.b.ts[e];
    idx = 0;
    if (inited && timers) c.fire_timers(c.ts, L.playback != 0, emit);  // timers due by this event fire before it
    if (!own) continue;
    if (!inited) seed();
    if (!reads) continue;
    c.ev_null = 0;
    for (int jj = 0; jj < ncap; ++jj) {  // the event is the same for every lane: identical LDS stores
      bool nl;
      evv[jj] = raw_word(L.b, q->cap_attr[c.stream][jj], e, nl);
      if (nl) c.ev_null |= 1u << jj;
    }
    c.receive(emit);
  }
  if (L.advance_to != INT64_MIN && c.err == kg::GE_OK && c.i32(q->lay.o_init) != 0) {  // time passes after the batch
    live = true;
    c.seq = L.timer_seq;
    c.fire_timers(L.advance_to, L.playback != 0, emit);
  }
  o.close();
  c.store_hot();
  if (nrec) atomicAdd(L.rec_count, nrec);
  if (c.err == kg::GE_CAPACITY) atomicOr(&L.err[0], c.capk);  // which limits (kg::CAP_*)
  if (c.err == kg::GE_REFERENCE) atomicOr(&L.err[1], 1);
  if (o.over) atomicOr(&L.err[2], 1);
}


// ---- K_seq (seq_body.h) with the interpreted window test: the shape's atoms, else its bytecode ----
struct SeqInterp {
  static constexpr bool kBranchFree = false;
  static constexpr int kRow = SEQ_ROW, kOutW = 1024;
  struct K {};
  __device__ static void load(K&, const kg::GQuery*) {}
  template <class Win>
  __device__ static bool match(const K&, const kg::GQuery* q, const kg::GQuery* ql, int64_t within, const Win& w) {
    return kg::seq_match(q, ql, within, w);
  }
};

__global__ __launch_bounds__(64) void nfa_seq_kernel(SeqLaunch L) { seq_body<SeqInterp>(L); }

// the stream's tail after this batch: the last min(SEQ_TMAX, tail_len + n) events of tail ++ batch
// (rows move towards 0 only, so increasing order is safe in place)
__global__ void seq_tail_kernel(StreamBatch b, int64_t* tail, int32_t tail_len, int32_t new_len) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int64_t W = tail_len + b.n;
  for (int r = 0; r < new_len; ++r) {
    const int64_t w = W - new_len + r;
    int64_t* dst = tail + (int64_t)r * SEQ_TW;
    if (w < tail_len) {
      const int64_t* src = tail + w * SEQ_TW;
      for (int k = 0; k < SEQ_TW; ++k) dst[k] = src[k];
    } else {
      const int64_t e = w - tail_len;
      dst[0] = b.ts[e];
      dst[1] = b.seq_base + e;
      for (int a = 0; a < MAXATTR; ++a) {
        bool nl = false;
        dst[2 + a] = a < b.n_attr ? raw_word(b, a, e, nl) : 0;
        dst[2 + MAXATTR + a] = nl ? 1 : 0;
      }
    }
  }
}

// ---- indexed timer sweep inputs: the batch's timestamp prefix max (and whether it is ordered), and
// each known key's routed segment ----
__global__ void ts_order_kernel(const int64_t* __restrict__ ts, int64_t n, int32_t* unordered) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > 0 && i < n && ts[i] < ts[i - 1]) atomicOr(unordered, 1);
}
__global__ void key_segment_kernel(const uint32_t* __restrict__ uniq, const int32_t* __restrict__ nruns,
                                   int64_t n_keys, int32_t* __restrict__ kseg) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= *nruns) return;
  const uint32_t kid = uniq[s];
  if (kid != 0xFFFFFFFFu && (int64_t)kid < n_keys) kseg[kid] = (int32_t)s;
}

// ---- keys created by this batch (ids [old_n, new_n)): their first event and value, for the
// creation order of the fan-out junction maps (PartitionRuntime.clonePartition at the key's first
// event) ----
__global__ void new_keys_kernel(const uint32_t* __restrict__ uniq, const int32_t* __restrict__ nruns,
                                const int32_t* __restrict__ off, const int32_t* __restrict__ idx_s,
                                const int64_t* __restrict__ key_of_id, int64_t old_n, int64_t new_n,
                                int64_t* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= *nruns) return;
  const uint32_t kid = uniq[s];
  if (kid == 0xFFFFFFFFu || (int64_t)kid < old_n || (int64_t)kid >= new_n) return;
  out[2 * (kid - old_n)] = idx_s[off[s]];  // segments list a key's events in batch order
  out[2 * (kid - old_n) + 1] = key_of_id[kid];
}

// ---- exact re-runs: the arena blocks a pass is about to modify, journaled just before it runs ----
// Slot x journals block: mode 0, glist[x] (an unpartitioned set's groups); mode 1, seg_kid[x /
// groups] * groups + x % groups (a partition's key segments; dropped events have no block); mode 2,
// x (a timer sweep over every known key). restore != 0 copies the journaled blocks back.
__global__ void gen_journal_kernel(int32_t* __restrict__ a32, int64_t* __restrict__ a64, int64_t B32, int64_t B64,
                                   int mode, const int32_t* __restrict__ glist, const uint32_t* __restrict__ seg_kid,
                                   int groups, int32_t* __restrict__ j32, int64_t* __restrict__ j64,
                                   int64_t* __restrict__ jidx, int restore) {
  const int64_t x = blockIdx.x;
  int64_t b;
  if (restore) {
    b = jidx[x];
  } else {
    if (mode == 0) {
      b = glist[x];
    } else if (mode == 1) {
      const uint32_t kid = seg_kid[x / groups];
      b = kid == 0xFFFFFFFFu ? -1 : (int64_t)kid * groups + x % groups;
    } else {
      b = x;
    }
    if (threadIdx.x == 0) jidx[x] = b;
  }
  if (b < 0) return;
  int32_t* s32 = a32 + b * B32 * 64;
  int32_t* d32 = j32 + x * B32 * 64;
  int64_t* s64 = a64 + b * B64 * 64;
  int64_t* d64 = j64 + x * B64 * 64;
  for (int64_t i = threadIdx.x; i < B32 * 64; i += blockDim.x) {
    if (restore) s32[i] = d32[i];
    else d32[i] = s32[i];
  }
  for (int64_t i = threadIdx.x; i < B64 * 64; i += blockDim.x) {
    if (restore) s64[i] = d64[i];
    else d64[i] = s64[i];
  }
}

// ---- live partials (sdh_engine_stats): entries of the pending lists of non-start states ----
__device__ __forceinline__ void acc_wave(unsigned long long v, unsigned long long* acc) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(acc, v);
}

// K_gen arenas: one thread per (block, lane); blocks [key][group] or [group]; K_seq groups skipped
__global__ void gen_live_kernel(const int32_t* __restrict__ a32, int64_t B32, int64_t blocks, int n_groups, int group_base,
                                const int32_t* __restrict__ lane_q, const int32_t* __restrict__ group_seq,
                                const kg::GQuery* __restrict__ queries, unsigned long long* acc) {
  const int64_t block = blockIdx.x;
  const int lane = threadIdx.x;
  unsigned long long v = 0;
  const int g = (int)(block % n_groups);
  const int qi = block < blocks ? lane_q[(int64_t)(group_base + g) * 64 + lane] : -1;
  if (qi >= 0 && group_seq[group_base + g] == 0) {
    const kg::GQuery& q = queries[qi];
    const int32_t* w = a32 + block * B32 * 64 + lane;
    if (w[(int64_t)q.lay.o_init * 64] != 0)
      for (int s = 0; s < q.n_states; ++s)
        if (!q.st[s].is_start) v += (unsigned long long)w[(int64_t)(q.lay.o_pn + s) * 64];
  }
  acc_wave(v, acc);
}

// K_seq: a sequence partial waits at state j (1 <= j < S) iff states 0 .. j-1 passed (with their
// `within` checks) over the stream's last j events (seq_body.h: the window argument); one wave per
// group of the stream, lane = query, over the carried tail
struct TailWin {
  static constexpr bool kStagedConsts = false;
  const int64_t* base;  // row of window event 0
  const int32_t* cap;   // the stream's captured attribute per capture index
  __device__ int64_t lane_const(int) const { return 0; }
  __device__ int64_t ts(int p) const { return base[p * SEQ_TW]; }
  __device__ int64_t raw(int p, int j, bool = false) const { return base[p * SEQ_TW + 2 + cap[j]]; }
  __device__ bool null(int p, int j, bool = false) const { return base[p * SEQ_TW + 2 + MAXATTR + cap[j]] != 0; }
};
__global__ void seq_live_kernel(const int64_t* __restrict__ tail, int tail_len, int stream,
                                const int32_t* __restrict__ groups, const int32_t* __restrict__ lane_q,
                                const int32_t* __restrict__ group_tmpl, const kg::GQuery* __restrict__ queries,
                                unsigned long long* acc) {
  const int g = groups[blockIdx.x];
  const int lane = threadIdx.x;
  const int qi = lane_q[(int64_t)g * 64 + lane];
  unsigned long long v = 0;
  if (qi >= 0) {
    const kg::GQuery* q = queries + group_tmpl[g];
    const kg::GQuery* ql = queries + qi;
    for (int j = 1; j < q->n_states && j <= tail_len; ++j)
      if (kg::seq_match(q, ql, ql->within, TailWin{tail + (int64_t)(tail_len - j) * SEQ_TW, q->cap_attr[stream]}, j))
        ++v;
  }
  acc_wave(v, acc);
}

// ---- pool growth: one instance arena re-laid from layout `a` to layout `b` (kgen.h make_layout) ----
// Pools and lists only grow, so every index an arena holds (StateEvent, node, list entry) stays
// valid: each field is copied entry by entry to its new offset and the new entries stay zero (free
// pool bits, empty list slots). One thread per (block, lane); blocks are [key][group] (partitioned)
// or [group].
__global__ void gen_remap_kernel(const int32_t* __restrict__ lane_q, int group_base, int n_groups, int64_t blocks,
                                 const kg::GLayout* __restrict__ oldL, const kg::GLayout* __restrict__ newL,
                                 const int32_t* __restrict__ o32, const int64_t* __restrict__ o64, int64_t oB32,
                                 int64_t oB64, int32_t* __restrict__ n32, int64_t* __restrict__ n64, int64_t nB32,
                                 int64_t nB64) {
  const int64_t block = blockIdx.x;
  const int lane = threadIdx.x;
  if (block >= blocks) return;
  const int g = (int)(block % n_groups);
  const int qi = lane_q[(int64_t)(group_base + g) * 64 + lane];
  if (qi < 0) return;
  const kg::GLayout a = oldL[qi], b = newL[qi];
  const int32_t* s32 = o32 + block * oB32 * 64 + lane;
  const int64_t* s64 = o64 + block * oB64 * 64 + lane;
  int32_t* d32 = n32 + block * nB32 * 64 + lane;
  int64_t* d64 = n64 + block * nB64 * 64 + lane;
  auto c32 = [&](int from, int to, int n) {
    for (int k = 0; k < n; ++k) d32[(int64_t)(to + k) * 64] = s32[(int64_t)(from + k) * 64];
  };
  auto c64 = [&](int from, int to, int n) {
    for (int k = 0; k < n; ++k) d64[(int64_t)(to + k) * 64] = s64[(int64_t)(from + k) * 64];
  };
  const int S = a.S;
  c32(a.o_flags, b.o_flags, S);
  c32(a.o_pn, b.o_pn, S);
  c32(a.o_nn, b.o_nn, S);
  for (int i = 0; i < S; ++i) {
    c32(a.o_plist + i * a.LC, b.o_plist + i * b.LC, a.LC);
    c32(a.o_nlist + i * a.LC, b.o_nlist + i * b.LC, a.LC);
  }
  c32(a.o_seslot, b.o_seslot, a.R * S);  // [StateEvent][state]: same stride S
  c32(a.o_ndnext, b.o_ndnext, a.N);
  c32(a.o_ndnull, b.o_ndnull, a.N);
  c32(a.o_init, b.o_init, 1);
  c64(a.o_seused, b.o_seused, a.SU);
  c64(a.o_ndused, b.o_ndused, a.NU);
  c64(a.o_sets, b.o_sets, a.R);
  c64(a.o_ndseq, b.o_ndseq, a.N);
  c64(a.o_ndts, b.o_ndts, a.N);
  if (a.v32) c32(a.o_ndval, b.o_ndval, a.N * a.NA);  // [node][attr]: same stride NA
  else c64(a.o_ndval, b.o_ndval, a.N * a.NA);
  if (a.TQ > 0) {  // absent schedulers: each FIFO ring is written out from its head (head 0)
    c64(a.o_lst, b.o_lst, S);
    for (int i = 0; i < S; ++i) {
      const int h = s32[(int64_t)(a.o_tqh + 2 * i) * 64], n = s32[(int64_t)(a.o_tqh + 2 * i + 1) * 64];
      for (int k = 0; k < n; ++k) d64[(int64_t)(b.o_tq + i * b.TQ + k) * 64] = s64[(int64_t)(a.o_tq + i * a.TQ + (h + k) % a.TQ) * 64];
      d32[(int64_t)(b.o_tqh + 2 * i) * 64] = 0;
      d32[(int64_t)(b.o_tqh + 2 * i + 1) * 64] = n;
    }
  }
}

// ---- partition routing ----
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Key-sharding rule of a multi-GPU engine: rank = |h % world| (Java int remainder), the reference's
// PartitionedDistributionStrategy destination (PartitionedDistributionStrategy.java:98-109) with h
// = String.valueOf(key).hashCode() for int / long / bool keys (the partition key IS that string,
// ValuePartitionExecutor.java:34-40); float / double keys (Java's shortest-repr formatting) and
// string dictionary ids hash their raw word instead. siddhi_amd/dist.py key_shard mirrors this.
__device__ int key_shard(int64_t raw, int type, int world) {
  int32_t h = 0;
  if (type == kg::T_INT || type == kg::T_LONG) {
    const int64_t v = type == kg::T_INT ? (int64_t)(int32_t)raw : raw;
    uint64_t mag = v < 0 ? 0ull - (uint64_t)v : (uint64_t)v;
    char dig[20];
    int nd = 0;
    do {
      dig[nd++] = (char)('0' + mag % 10);
      mag /= 10;
    } while (mag);
    uint32_t u = v < 0 ? 45u : 0u;  // '-'
    for (int i = nd - 1; i >= 0; --i) u = u * 31u + (uint32_t)dig[i];
    h = (int32_t)u;
  } else if (type == kg::T_BOOL) {
    h = raw ? 3569038 : 97196323;  // "true".hashCode(), "false".hashCode()
  } else {
    h = (int32_t)(mix64((uint64_t)raw) >> 33);
  }
  const int32_t r = h % world;
  return r < 0 ? -r : r;
}

// shard_world > 1: events whose key another rank owns are dropped here, like null keys
__global__ void gen_keys_kernel(StreamBatch b, int attr, int type, int64_t* key, uint32_t* kid, int shard_rank,
                                int shard_world) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= b.n) return;
  bool nl;
  int64_t raw = raw_word(b, attr, e, nl);
  if (type == kg::T_FLOAT) {
    const float f = __uint_as_float((uint32_t)raw);
    raw = (f != f) ? 0x7fc00000 : (int64_t)(uint32_t)raw;
  } else if (type == kg::T_DOUBLE) {
    const double d = __longlong_as_double(raw);
    if (d != d) raw = 0x7ff8000000000000LL;
  }
  key[e] = raw;
  const bool foreign = shard_world > 1 && !nl && key_shard(raw, type, shard_world) != shard_rank;
  kid[e] = (nl || foreign) ? 0xFFFFFFFFu : 0u;  // 0 = valid, resolved by the lookup
}

constexpr long long KEY_EMPTY = (long long)0x8000000000000000ull;  // INT64_MIN keys use slot `cap`

__global__ void gen_insert_kernel(int64_t n, const int64_t* key, const uint32_t* kid, unsigned long long* tkey,
                                  int64_t mask, int32_t* err) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n || kid[e] == 0xFFFFFFFFu) return;
  const long long k = key[e];
  if (k == KEY_EMPTY) {  // the INT64_MIN key lives in the extra slot mask+1 (1 = present)
    tkey[mask + 1] = 1ull;
    return;
  }
  int64_t h = (int64_t)(mix64((uint64_t)k) & (uint64_t)mask);
  for (int64_t p = 0; p <= mask; ++p) {
    const unsigned long long cur = atomicCAS(&tkey[h], (unsigned long long)KEY_EMPTY, (unsigned long long)k);
    if (cur == (unsigned long long)KEY_EMPTY || cur == (unsigned long long)k) return;
    h = (h + 1) & mask;
  }
  atomicOr(err, 1);
}

__global__ void gen_assign_kernel(const unsigned long long* tkey, int32_t* tid, int64_t slots, int32_t* n_keys,
                                  int64_t* key_of_id, int64_t key_cap, int32_t* err) {
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h >= slots) return;
  const bool special = h == slots - 1;  // INT64_MIN key slot (initialized to 0, 1 = present)
  const bool used = special ? tkey[h] == 1ull : tkey[h] != (unsigned long long)KEY_EMPTY;
  if (!used || tid[h] >= 0) return;
  const int32_t id = atomicAdd(n_keys, 1);
  if (id >= key_cap) {
    atomicOr(err, 1);
    return;
  }
  tid[h] = id;
  key_of_id[id] = special ? INT64_MIN : (int64_t)tkey[h];
}

__global__ void gen_lookup_kernel(int64_t n, const int64_t* key, uint32_t* kid, int32_t* idx,
                                  const unsigned long long* tkey, const int32_t* tid, int64_t mask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  idx[e] = (int32_t)e;
  if (kid[e] == 0xFFFFFFFFu) return;
  const long long k = key[e];
  if (k == KEY_EMPTY) {
    kid[e] = (uint32_t)tid[mask + 1];
    return;
  }
  int64_t h = (int64_t)(mix64((uint64_t)k) & (uint64_t)mask);
  while (tkey[h] != (unsigned long long)k) h = (h + 1) & mask;
  kid[e] = (uint32_t)tid[h];
}

}  // namespace sdh

extern "C" hipError_t sdh_launch_gen(const sdh::GenLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  // 4 waves/SIMD (116 VGPRs, no spills): on C3, 5 (96 VGPRs + spills) is level and 6 / 8 are
  // 10-30 % slower
  const size_t lds = (size_t)(sdh::kg::GMAXNA + (1 + L->hot_nu) * 64) * 8 + (size_t)(3 * L->hot_s + 4) * 64 * 4;
  hipLaunchKernelGGL(sdh::nfa_gen_kernel<4>, dim3(L->xcd ? (L->n_items + 7) & ~7 : L->n_items), dim3(64), lds, s, *L);
  return hipGetLastError();
}

extern "C" hipError_t sdh_launch_seq(const sdh::SeqLaunch* L, hipStream_t s) {
  if (L->n_glist > 0 && L->n_chunks > 0)
    hipLaunchKernelGGL(sdh::nfa_seq_kernel, dim3(L->xcd ? (L->n_glist * L->n_chunks + 7) & ~7 : L->n_glist * L->n_chunks),
                       dim3(64), 0, s, *L);
  return hipGetLastError();
}

// pm = inclusive prefix max of ts; *unordered (device) = 1 when ts decreases somewhere
extern "C" size_t sdh_prefix_max_temp_bytes(int64_t n) {
  size_t b = 0;
  (void)hipcub::DeviceScan::InclusiveScan((void*)nullptr, b, (const int64_t*)nullptr, (int64_t*)nullptr,
                                          hipcub::Max(), (int)n);
  return b + 256;
}
extern "C" hipError_t sdh_prefix_max(const int64_t* ts, int64_t n, int64_t* pm, int32_t* unordered, void* temp,
                                     size_t temp_bytes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(unordered, 0, 4, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(sdh::ts_order_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ts, n, unordered);
  size_t tb = temp_bytes;
  e = hipcub::DeviceScan::InclusiveScan(temp, tb, ts, pm, hipcub::Max(), (int)n, s);
  if (e != hipSuccess) return e;
  return hipGetLastError();
}
extern "C" hipError_t sdh_new_keys(const uint32_t* uniq, const int32_t* nruns, int64_t max_runs, const int32_t* off,
                                   const int32_t* idx_s, const int64_t* key_of_id, int64_t old_n, int64_t new_n,
                                   int64_t* out, hipStream_t s) {
  if (max_runs <= 0 || new_n <= old_n) return hipSuccess;
  hipLaunchKernelGGL(sdh::new_keys_kernel, dim3((unsigned)((max_runs + 255) / 256)), dim3(256), 0, s, uniq, nruns, off,
                     idx_s, key_of_id, old_n, new_n, out);
  return hipGetLastError();
}
// kseg[kid] = the routed segment of key kid in this batch, -1 without events
extern "C" hipError_t sdh_key_segments(const uint32_t* uniq, const int32_t* nruns, int64_t max_runs, int64_t n_keys,
                                       int32_t* kseg, hipStream_t s) {
  if (n_keys <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(kseg, 0xFF, (size_t)n_keys * 4, s);
  if (e != hipSuccess) return e;
  if (max_runs > 0)
    hipLaunchKernelGGL(sdh::key_segment_kernel, dim3((unsigned)((max_runs + 255) / 256)), dim3(256), 0, s, uniq, nruns,
                       n_keys, kseg);
  return hipGetLastError();
}

extern "C" hipError_t sdh_gen_journal(int32_t* a32, int64_t* a64, int64_t B32, int64_t B64, int mode,
                                       const int32_t* glist, const uint32_t* seg_kid, int groups, int64_t slots,
                                       int32_t* j32, int64_t* j64, int64_t* jidx, int restore, hipStream_t s) {
  if (slots <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::gen_journal_kernel, dim3((unsigned)slots), dim3(256), 0, s, a32, a64, B32, B64, mode, glist,
                     seg_kid, groups, j32, j64, jidx, restore);
  return hipGetLastError();
}

extern "C" hipError_t sdh_live_gen(const int32_t* a32, int64_t B32, int64_t blocks, int n_groups, int group_base,
                                    const int32_t* lane_q, const int32_t* group_seq, const sdh::kg::GQuery* queries,
                                    unsigned long long* acc, hipStream_t s) {
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::gen_live_kernel, dim3((unsigned)blocks), dim3(64), 0, s, a32, B32, blocks, n_groups,
                     group_base, lane_q, group_seq, queries, acc);
  return hipGetLastError();
}

extern "C" hipError_t sdh_live_seq(const int64_t* tail, int tail_len, int stream, const int32_t* groups, int n_groups,
                                   const int32_t* lane_q, const int32_t* group_tmpl, const sdh::kg::GQuery* queries,
                                   unsigned long long* acc, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::seq_live_kernel, dim3((unsigned)n_groups), dim3(64), 0, s, tail, tail_len, stream, groups,
                     lane_q, group_tmpl, queries, acc);
  return hipGetLastError();
}

// roll a stream's K_seq tail over batch b (after the push's K_seq launches have succeeded)
extern "C" hipError_t sdh_seq_tail(const sdh::StreamBatch* b, int64_t* tail, int32_t tail_len, int32_t new_tail_len,
                                   hipStream_t s) {
  hipLaunchKernelGGL(sdh::seq_tail_kernel, dim3(1), dim3(64), 0, s, *b, tail, tail_len, new_tail_len);
  return hipGetLastError();
}

// re-lay `blocks` instance blocks of one K_gen set from the old to the new pool sizing (zeroed `n32`/`n64`)
extern "C" hipError_t sdh_gen_remap(const int32_t* lane_q, int group_base, int n_groups, int64_t blocks,
                                    const sdh::kg::GLayout* oldL, const sdh::kg::GLayout* newL, const int32_t* o32,
                                    const int64_t* o64, int64_t oB32, int64_t oB64, int32_t* n32, int64_t* n64,
                                    int64_t nB32, int64_t nB64, hipStream_t s) {
  if (blocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::gen_remap_kernel, dim3((unsigned)blocks), dim3(64), 0, s, lane_q, group_base, n_groups, blocks,
                     oldL, newL, o32, o64, oB32, oB64, n32, n64, nB32, nB64);
  return hipGetLastError();
}

// Route batch B of a partitioned stream: dense key ids (persistent hash table), then events grouped
// by key id (stable). Outputs: sorted kids/idx, run-length segments; *n_seg on the host.
// Scratch: key[n], kid[n], kid_sorted[n], idx[n], idx_sorted[n], uniq[n], cnt[n], off[n], temp.
extern "C" hipError_t sdh_route_partition(const sdh::StreamBatch* B, int attr, int type, unsigned long long* tkey,
                                          int32_t* tid, int64_t table_mask, int32_t* n_keys, int64_t* key_of_id,
                                          int64_t key_cap, int64_t* key, uint32_t* kid, uint32_t* kid_sorted,
                                          int32_t* idx, int32_t* idx_sorted, uint32_t* uniq, int32_t* cnt,
                                          int32_t* off, int32_t* n_runs_dev, void* temp, size_t temp_bytes,
                                          int32_t* err, int shard_rank, int shard_world, hipStream_t s) {
  const int64_t n = B->n;
  const int T = 256;
  const int nb = (int)((n + T - 1) / T);
  hipLaunchKernelGGL(sdh::gen_keys_kernel, dim3(nb), dim3(T), 0, s, *B, attr, type, key, kid, shard_rank, shard_world);
  hipLaunchKernelGGL(sdh::gen_insert_kernel, dim3(nb), dim3(T), 0, s, n, key, kid, tkey, table_mask, err);
  const int64_t slots = table_mask + 2;
  hipLaunchKernelGGL(sdh::gen_assign_kernel, dim3((int)((slots + T - 1) / T)), dim3(T), 0, s, tkey, tid, slots,
                     n_keys, key_of_id, key_cap, err);
  hipLaunchKernelGGL(sdh::gen_lookup_kernel, dim3(nb), dim3(T), 0, s, n, key, kid, idx, tkey, tid, table_mask);
  size_t tb = temp_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(temp, tb, kid, kid_sorted, idx, idx_sorted, (int)n, 0, 32, s);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  e = hipcub::DeviceRunLengthEncode::Encode(temp, tb, kid_sorted, uniq, cnt, n_runs_dev, (int)n, s);
  if (e != hipSuccess) return e;
  tb = temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(temp, tb, cnt, off, (int)n, s);
  return e == hipSuccess ? hipGetLastError() : e;
}

// temp storage the routing needs for n events
extern "C" size_t sdh_route_temp_bytes(int64_t n) {
  size_t a = 0, b = 0, c = 0;
  (void)hipcub::DeviceRadixSort::SortPairs((void*)nullptr, a, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                     (int32_t*)nullptr, (int)n, 0, 32);
  (void)hipcub::DeviceRunLengthEncode::Encode((void*)nullptr, b, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                        (int32_t*)nullptr, (int)n);
  (void)hipcub::DeviceScan::ExclusiveSum((void*)nullptr, c, (int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return std::max(a, std::max(b, c)) + 256;
}
