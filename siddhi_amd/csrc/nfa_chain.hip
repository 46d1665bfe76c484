// nfa_chain.hip -- NFA-step kernel (K1 + K2 + K3 of SURVEY §2) for chain-family queries:
//
//     every? e0=S[f0] -> e1=S[f1(e0)] -> ... -> e{n-1}=S[f{n-1}(...)] [within T]
//
// Semantics restated from the reference (state/ = siddhi-core .../query/input/stream/state/):
//   * one pending partial per (pattern, trigger) -- StreamPreStateProcessor.processAndReturn:292-337
//   * a partial added during event j becomes pending for event j+1 (two-phase newAndEvery ->
//     pending promotion, :203-227,281-289; multi-stream receivers process states in reverse
//     registration order, PatternMultiProcessStreamReceiver.java:38-44) -- here: states are swept
//     from the last to the first, so an advanced partial is never seen twice for one event
//   * lazy `within` expiry measured against the start slot (isExpired:102-113), checked before
//     the filter, only on non-start states
//   * start state with `every` keeps its (stateless) seed forever (StreamPostStateProcessor:66-68
//     re-arms a shallow clone); without `every` the seed is consumed by its first match (R3)
//   * the last state emits (isEventReturned, :310-313) and drops the partial (stateChanged)
//   * predicates: conjunctions of typed compares, null -> false (FilterProcessor:55-66,
//     CompareConditionExpressionExecutor:39-43), evaluated in Java's promotion domain
//
// Mapping to CDNA4: one 64-lane wave owns one (query instance, event chunk); each lane holds one
// partial match in registers (K register sets -> 64*K partials). Every 64 events the wave stages
// a tile in its private LDS region: one coalesced load per attribute column, converted once per
// event into compare-domain keys (f64 or i64), so the per-event predicate is a branch-free pair of
// compares read by wave-uniform (broadcast) LDS loads. New partials take the first free lane
// (ctz of the inverted live-lane ballot); matches are compacted with ballot + mbcnt into the
// wave's contiguous output segment. No MFMA: the step is compare/branch work.
//
// Exactness of event-chunk parallelism: for chunkable queries (every on the start
// state, within T, one input stream) chunk c > 0 re-derives its start state by replaying the
// events from w0 = lower_bound(ts, ts[c0-1] - T) without emitting; any partial older than w0
// has expired by event c0-1. Requires non-decreasing timestamps, which every wave verifies on
// the range it reads (err[1]); the host re-runs the batch unchunked otherwise.
#include <hip/hip_runtime.h>

#include "nfa_types.h"

namespace sdh {

__device__ __forceinline__ int wave_mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Number.floatValue()/doubleValue()/longValue() into the compare domain (see enum Conv)
__device__ __forceinline__ int64_t to_key(uint64_t raw, int conv) {
  switch (conv) {
    case CV_I64_INT: return (int64_t)(int32_t)(uint32_t)raw;
    case CV_I64_LONG: return (int64_t)raw;
    case CV_F32_INT: return __double_as_longlong((double)(float)(int32_t)(uint32_t)raw);
    case CV_F32_LONG: return __double_as_longlong((double)(float)(int64_t)raw);
    case CV_F32_FLOAT:
    case CV_F64_FLOAT: return __double_as_longlong((double)__uint_as_float((uint32_t)raw));
    case CV_F64_INT: return __double_as_longlong((double)(int32_t)(uint32_t)raw);
    case CV_F64_LONG: return __double_as_longlong((double)(int64_t)raw);
    default: return (int64_t)raw;  // CV_F64_DOUBLE, CV_RAW
  }
}

// typed compare of two keys: ((lt & b0) | (gt & b1) | (eq & b2)) ^ b3 -- IEEE semantics for f64
// keys (NaN: only != holds), exactly Java's primitive compares
__device__ __forceinline__ bool cmp_keys(int mask, int f64, int64_t l, int64_t r) {
  bool lt, gt, eq;
  if (f64) {
    const double a = __longlong_as_double(l), b = __longlong_as_double(r);
    lt = a < b;
    gt = b < a;
    eq = a == b;
  } else {
    lt = l < r;
    gt = r < l;
    eq = l == r;
  }
  const bool v = (lt && (mask & CM_LT)) || (gt && (mask & CM_GT)) || (eq && (mask & CM_EQ));
  return v != ((mask & CM_NOT) != 0);
}

// Math.abs(a - b) > within with Java long wrap-around (Math.abs(Long.MIN_VALUE) < 0)
__device__ __forceinline__ bool expired(int64_t t0, int64_t t, int64_t within) {
  int64_t d = (int64_t)((uint64_t)t0 - (uint64_t)t);
  int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

// one register set of partial matches: lane l of set k holds partial 64*k + l
struct PSet {
  int st;                  // state id the partial is pending at, -1 = free lane
  int64_t ts0;             // timestamp of the start-state event (within reference)
  int64_t sq[MAXS - 1];    // event sequence number per filled slot
  int64_t cp[MAXCAP];      // captured operand keys read by later filters
  uint32_t cn;             // captured-null bits
};

__device__ __forceinline__ int64_t cap_get(const PSet P, int idx) {
  int64_t v = P.cp[0];
#pragma unroll
  for (int c = 1; c < MAXCAP; ++c) v = (idx == c) ? P.cp[c] : v;
  return v;
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, k);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), k);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// one atom on per-lane operands (tile time: lane = event; step time: lane = partial)
__device__ __forceinline__ bool atom_eval(const Atom& A, int64_t l, bool ln, int64_t r, bool rn) {
  return !ln && !rn && cmp_keys(A.mask, A.f64, l, r);
}

// first index i in [0, c0) with ts[i] >= target (64-ary search, all lanes cooperate)
__device__ int64_t lower_bound_ts(const int64_t* ts, int64_t c0, int64_t target, int lane) {
  int64_t lo = 0, hi = c0;  // answer in [lo, hi]
  while (hi - lo > 1) {
    const int64_t span = hi - lo;
    const int64_t p = lo + (span * lane) / WAVE;  // probe positions, p < hi
    const uint64_t m = __ballot(ts[p] < target);
    const int nb = __popcll(m);                   // ts is sorted: the first nb probes are below
    const int64_t nlo = nb == 0 ? lo : lo + (span * (nb - 1)) / WAVE + 1;
    const int64_t nhi = nb == WAVE ? hi : lo + (span * nb) / WAVE;
    lo = rfl64(nlo);
    hi = rfl64(nhi);
    if (lo == hi) break;
  }
  if (lo < c0 && ts[lo] < target) lo = lo + 1;
  return lo;
}

// Per-state predicate/capture descriptor, resolved once per wave into SGPRs so that the event
// loop carries no data-dependent decisions about the query's shape.
struct StateDesc {
  int active;        // state fed by this launch's stream
  int has_x;         // state has a capture-reading atom (at most one, planner-enforced)
  int l_cap, r_cap;  // operand is a captured value (index in lcap/rcap)
  int l_cur, r_cur;  // operand is the current event (key in xcur)
  int lcap, rcap;
  int64_t lc, rc;    // constant keys (used when neither CAP nor CUR)
  int l_null, r_null;
  int f64, mask;
  uint32_t capmask;  // captures taken when a partial passes this state
};

template <int S, int K>
__global__ __launch_bounds__(256) void nfa_chain_kernel(ChainLaunch L) {
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + wv;
  if (wid >= L.n_work) return;
  const WorkItem W = L.work[wid];
  const ChainQuery* __restrict__ Q = L.queries + W.q;
  const int stream = L.b.stream;
  const int pcap = L.pcap;
  // ---- wave-uniform program, resolved into SGPRs for the whole chunk ----
  const int64_t within = Q->within < 0 ? INT64_MAX : Q->within;
  const int every = Q->every, n_cap = Q->n_cap, qid = Q->qid, n_col = Q->n_col;
  StateDesc D[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    StateDesc d{};
    d.active = Q->state_stream[s] == stream;
    d.has_x = Q->xa_count[s] > 0;
    if (d.has_x) {
      const Atom& A = Q->atoms[Q->xa_atom[Q->xa_first[s]]];
      d.l_cap = A.lk == OPK_CAP; d.r_cap = A.rk == OPK_CAP;
      d.l_cur = A.lk == OPK_CUR; d.r_cur = A.rk == OPK_CUR;
      d.lcap = d.l_cap ? A.li : 0; d.rcap = d.r_cap ? A.ri : 0;
      d.lc = A.lc; d.rc = A.rc;
      d.l_null = A.lk == OPK_NULL; d.r_null = A.rk == OPK_NULL;
      d.f64 = A.f64; d.mask = A.mask;
    }
    uint32_t cm = 0;
    for (int c = 0; c < n_cap; ++c) cm |= (Q->cap_slot[c] == s ? 1u : 0u) << c;
    d.capmask = cm;
    D[s] = d;
  }

  // ---- start state: persisted table (chunk 0 / window reaching the batch start) or replay ----
  int64_t w0 = 0;
  if (W.chunk > 0) w0 = lower_bound_ts(L.b.ts, W.c0, L.b.ts[W.c0 - 1] - within, lane);
  PSet P[K];
  int seed_alive = 1;
  if (w0 == 0) {
    const int64_t* pin = L.part[W.inb] + (size_t)W.q * NF * pcap;
    seed_alive = L.hdr[W.inb][W.q].seed_alive;
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      const int li = kk * WAVE + lane;
      P[kk].st = (int)pin[F_STATE * pcap + li];
      P[kk].ts0 = pin[F_TS0 * pcap + li];
#pragma unroll
      for (int s = 0; s < MAXS - 1; ++s) P[kk].sq[s] = pin[(F_SEQ0 + s) * pcap + li];
#pragma unroll
      for (int c = 0; c < MAXCAP; ++c) P[kk].cp[c] = pin[(F_CAP0 + c) * pcap + li];
      P[kk].cn = (uint32_t)pin[F_CAPNULL * pcap + li];
    }
  } else {
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      P[kk].st = -1;
      P[kk].ts0 = 0;
#pragma unroll
      for (int s = 0; s < MAXS - 1; ++s) P[kk].sq[s] = 0;
#pragma unroll
      for (int c = 0; c < MAXCAP; ++c) P[kk].cp[c] = 0;
      P[kk].cn = 0;
    }
  }

  int64_t nmatch = 0;
  int64_t* seg = L.match + W.seg_off * L.rec_words;
  const int RW = L.rec_words;
  bool unordered = false, overflow = false, seg_over = false;
  int64_t prev_tile_ts = (w0 == 0) ? L.b.prev_ts : L.b.ts[w0 - 1];

  for (int64_t t = w0; t < W.c1; t += WAVE) {
    // ---- stage 64 events, one per lane: coalesced column loads converted once into
    //      compare-domain keys; partial-independent atoms evaluated for the whole tile ----
    const int64_t e = t + lane;
    const bool live = e < W.c1;
    const int64_t ets = live ? L.b.ts[e] : INT64_MAX;
    int64_t ck[MAXCOL];
    uint32_t cnul = 0;
#pragma unroll
    for (int c = 0; c < MAXCOL; ++c) {
      ck[c] = 0;
      if (c < n_col && Q->col_stream[c] == stream) {
        const int a = Q->col_attr[c];
        uint64_t raw = 0;
        if (live) {
          const int wdt = L.b.width[a];
          if (wdt == 8) raw = ((const uint64_t*)L.b.col[a])[e];
          else if (wdt == 4) raw = ((const uint32_t*)L.b.col[a])[e];
          else raw = ((const uint8_t*)L.b.col[a])[e];
          if (L.b.nul[a] && ((const uint8_t*)L.b.nul[a])[e]) cnul |= 1u << c;
        }
        ck[c] = to_key(raw, Q->col_conv[c]);
      }
    }
    auto col_key = [&](int col) {
      int64_t v = ck[0];
#pragma unroll
      for (int c = 1; c < MAXCOL; ++c) v = (col == c) ? ck[c] : v;
      return v;
    };
    // per state: bit k set iff event k passes every atom of the state that reads no capture
    uint64_t smask[S];
    int64_t xcur[S];      // current-event operand of the state's capture-reading atom
    uint32_t xnul = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      bool ok = live && D[s].active;
      xcur[s] = 0;
      if (D[s].active) {
        const int a1 = Q->atom_begin[s + 1] - Q->xa_count[s];
        for (int a = Q->atom_begin[s]; a < a1; ++a) {
          const Atom& A = Q->atoms[a];
          const int64_t l = A.lk == OPK_CUR ? col_key(A.li) : A.lc;
          const int64_t r = A.rk == OPK_CUR ? col_key(A.ri) : A.rc;
          const bool ln = A.lk == OPK_NULL || (A.lk == OPK_CUR && ((cnul >> A.li) & 1u));
          const bool rn = A.rk == OPK_NULL || (A.rk == OPK_CUR && ((cnul >> A.ri) & 1u));
          ok = ok && atom_eval(A, l, ln, r, rn);
        }
        if (D[s].has_x) {
          const int col = Q->xa_col[Q->xa_first[s]];
          if (col >= 0) {
            xcur[s] = col_key(col);
            xnul |= ((cnul >> col) & 1u) << s;
          }
        }
      }
      smask[s] = __ballot(ok);
    }
    int64_t capv[MAXCAP];
    uint32_t capn = 0;
#pragma unroll
    for (int c = 0; c < MAXCAP; ++c) {
      capv[c] = 0;
      if (c < n_cap) {
        capv[c] = col_key(Q->cap_col[c]);
        capn |= ((cnul >> Q->cap_col[c]) & 1u) << c;
      }
    }
    // timestamps must be non-decreasing for chunk warm-up to be exact
    int64_t pred = __shfl_up(ets, 1, WAVE);
    if (lane == 0) pred = prev_tile_ts;
    if (live && ets < pred) unordered = true;
    prev_tile_ts = __shfl(ets, WAVE - 1, WAVE);

    const int cnt = (int)((W.c1 - t) < WAVE ? (W.c1 - t) : WAVE);
#pragma unroll 1
    for (int k = 0; k < cnt; ++k) {
      const int64_t j = t + k;
      const bool emit_ok = j >= W.c0;
      const int64_t cts = readlane64(ets, k);
      const int64_t cseq = L.b.seq_base + j;
      const uint32_t capn_k = __builtin_amdgcn_readlane(capn, k);
      const uint32_t xnul_k = __builtin_amdgcn_readlane(xnul, k);

      // ---- non-start states, last to first (reverse registration order) ----
#pragma unroll
      for (int s = S - 1; s >= 1; --s) {
        const StateDesc& d = D[s];
        if (!d.active) continue;
        const bool last = (s == S - 1);
        const bool cpass = (smask[s] >> k) & 1ull;
        const int64_t cur = readlane64(xcur[s], k);
        const bool curn = (xnul_k >> s) & 1u;
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          const bool in_s = P[kk].st == s;
          if (__ballot(in_s) == 0) continue;
          const bool exp = in_s && expired(P[kk].ts0, cts, within);
          bool pass = in_s && !exp && cpass;
          if (d.has_x) {
            const int64_t lcap = cap_get(P[kk], d.lcap), rcap = cap_get(P[kk], d.rcap);
            const int64_t l = d.l_cap ? lcap : d.l_cur ? cur : d.lc;
            const int64_t r = d.r_cap ? rcap : d.r_cur ? cur : d.rc;
            const bool ln = d.l_null || (d.l_cur && curn) || (d.l_cap && ((P[kk].cn >> d.lcap) & 1u));
            const bool rn = d.r_null || (d.r_cur && curn) || (d.r_cap && ((P[kk].cn >> d.rcap) & 1u));
            pass = pass && !ln && !rn && cmp_keys(d.mask, d.f64, l, r);
          }
          if (last) {
            const uint64_t m = __ballot(pass);
            if (m && emit_ok) {
              const int64_t rank = nmatch + wave_mbcnt(m);
              if (nmatch + __popcll(m) > W.seg_cap) {
                seg_over = true;
              } else if (pass) {
                int64_t* r = seg + rank * RW;
                r[0] = qid;
                r[1] = cts;
#pragma unroll
                for (int q2 = 0; q2 < S - 1; ++q2) r[2 + q2] = P[kk].sq[q2];
                r[2 + S - 1] = cseq;
              }
              nmatch += __popcll(m);
            }
            if (pass || exp) P[kk].st = -1;
          } else {
            if (exp) P[kk].st = -1;
            if (pass) {
              P[kk].st = s + 1;
              P[kk].sq[s] = cseq;
#pragma unroll
              for (int c = 0; c < MAXCAP; ++c) {
                const bool take = (d.capmask >> c) & 1u;
                const int64_t v = readlane64(capv[c], k);
                const uint32_t nb = (capn_k >> c) & 1u;
                P[kk].cp[c] = take ? v : P[kk].cp[c];
                P[kk].cn = take ? ((P[kk].cn & ~(1u << c)) | (nb << c)) : P[kk].cn;
              }
            }
          }
        }
      }

      // ---- start state: the seed (every re-arms it, otherwise one match consumes it) ----
      if (seed_alive && ((smask[0] >> k) & 1ull)) {
        if (S == 1) {
          if (emit_ok) {
            if (nmatch + 1 > W.seg_cap) {
              seg_over = true;
            } else if (lane == 0) {
              int64_t* r = seg + nmatch * RW;
              r[0] = qid;
              r[1] = cts;
              r[2] = cseq;
            }
            nmatch += 1;
          }
        } else {
          int slot_set = -1, slot_lane = 0;
#pragma unroll
          for (int kk = 0; kk < K; ++kk) {
            const uint64_t freem = ~__ballot(P[kk].st >= 0);
            if (slot_set < 0 && freem != 0) {
              slot_set = kk;
              slot_lane = __builtin_ctzll(freem);
            }
          }
          if (slot_set < 0) overflow = true;
          const uint32_t cm0 = D[0].capmask;
#pragma unroll
          for (int kk = 0; kk < K; ++kk) {
            if (kk != slot_set) continue;
            const bool mine = lane == slot_lane;
            P[kk].st = mine ? 1 : P[kk].st;
            P[kk].ts0 = mine ? cts : P[kk].ts0;
            P[kk].sq[0] = mine ? cseq : P[kk].sq[0];
            P[kk].cn = mine ? 0u : P[kk].cn;
#pragma unroll
            for (int c = 0; c < MAXCAP; ++c) {
              const bool take = mine && ((cm0 >> c) & 1u);
              const int64_t v = readlane64(capv[c], k);
              P[kk].cp[c] = take ? v : P[kk].cp[c];
              P[kk].cn = take ? (P[kk].cn | (((capn_k >> c) & 1u) << c)) : P[kk].cn;
            }
          }
        }
        if (!every) seed_alive = 0;
      }
    }
  }

  // ---- outputs ----
  const uint64_t any_unordered = __ballot(unordered);
  if (lane == 0) {
    L.seg_count[wid] = nmatch;
    if (overflow) atomicOr(&L.err[0], 1);
    if (any_unordered && W.n_chunks > 1) atomicOr(&L.err[1], 1);
    if (seg_over) atomicOr(&L.err[2], 1);
  }
  if (W.chunk == W.n_chunks - 1) {  // the last chunk owns the instance's final state
    int64_t* pout = L.part[1 - W.inb] + (size_t)W.q * NF * pcap;
    int nlive = 0;
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      const int li = kk * WAVE + lane;
      pout[F_STATE * pcap + li] = P[kk].st;
      pout[F_TS0 * pcap + li] = P[kk].ts0;
#pragma unroll
      for (int s = 0; s < MAXS - 1; ++s) pout[(F_SEQ0 + s) * pcap + li] = P[kk].sq[s];
#pragma unroll
      for (int c = 0; c < MAXCAP; ++c) pout[(F_CAP0 + c) * pcap + li] = P[kk].cp[c];
      pout[F_CAPNULL * pcap + li] = P[kk].cn;
      nlive += __popcll(__ballot(P[kk].st >= 0));
    }
    if (lane == 0) {
      InstHeader h;
      h.seed_alive = seed_alive;
      h.n_live = nlive;
      h.overflow = overflow;
      h.unordered = any_unordered != 0;
      L.hdr[1 - W.inb][W.q] = h;
    }
  }
}

}  // namespace sdh

template <int S>
static hipError_t launch_s(int k, const sdh::ChainLaunch* L, int n_blocks, size_t lds, hipStream_t s) {
  switch (k) {
    case 1: hipLaunchKernelGGL((sdh::nfa_chain_kernel<S, 1>), dim3(n_blocks), dim3(256), lds, s, *L); break;
    case 2: hipLaunchKernelGGL((sdh::nfa_chain_kernel<S, 2>), dim3(n_blocks), dim3(256), lds, s, *L); break;
    case 4: hipLaunchKernelGGL((sdh::nfa_chain_kernel<S, 4>), dim3(n_blocks), dim3(256), lds, s, *L); break;
    case 8: hipLaunchKernelGGL((sdh::nfa_chain_kernel<S, 8>), dim3(n_blocks), dim3(256), lds, s, *L); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// host-side launchers (C linkage inside the library)
extern "C" hipError_t sdh_launch_chain(int n_states, int k, const sdh::ChainLaunch* L, int n_blocks,
                                       size_t lds, hipStream_t s) {
  if (n_blocks <= 0) return hipSuccess;
  switch (n_states) {
    case 1: return launch_s<1>(k, L, n_blocks, lds, s);
    case 2: return launch_s<2>(k, L, n_blocks, lds, s);
    case 3: return launch_s<3>(k, L, n_blocks, lds, s);
    case 4: return launch_s<4>(k, L, n_blocks, lds, s);
    default: return hipErrorInvalidValue;
  }
}
