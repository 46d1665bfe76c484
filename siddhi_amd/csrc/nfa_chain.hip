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
//
// Mapping to CDNA4: one 64-lane wave owns one (query instance, event chunk); each lane holds one
// partial match in registers (K register sets -> 64*K partials). The event stream is staged per
// wave in LDS tiles of 64 events (one coalesced load per attribute column, then wave-uniform
// broadcast reads); new partials take the first free lane (s_ff1 on the ballot of live lanes);
// matches are compacted with ballot + mbcnt into the wave's contiguous output segment. No MFMA:
// the step is compare/branch work.
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

template <class T>
__device__ __forceinline__ bool cmpv(int op, T a, T b) {
  switch (op) {
    case CMP_EQ: return a == b;
    case CMP_NE: return a != b;
    case CMP_GT: return a > b;
    case CMP_GE: return a >= b;
    case CMP_LT: return a < b;
    default: return a <= b;
  }
}

// Number.floatValue()/doubleValue()/longValue() of a raw attribute word
__device__ __forceinline__ float to_f32(uint64_t raw, int t) {
  switch (t) {
    case T_INT: return (float)(int32_t)(uint32_t)raw;
    case T_LONG: return (float)(int64_t)raw;
    case T_FLOAT: return __uint_as_float((uint32_t)raw);
    default: return (float)__longlong_as_double((long long)raw);
  }
}
__device__ __forceinline__ double to_f64(uint64_t raw, int t) {
  switch (t) {
    case T_INT: return (double)(int32_t)(uint32_t)raw;
    case T_LONG: return (double)(int64_t)raw;
    case T_FLOAT: return (double)__uint_as_float((uint32_t)raw);
    default: return __longlong_as_double((long long)raw);
  }
}
__device__ __forceinline__ int64_t to_i64(uint64_t raw, int t) {
  return t == T_INT ? (int64_t)(int32_t)(uint32_t)raw : (int64_t)raw;
}

// CompareConditionExpressionExecutor.execute:39-43 + the typed execute() of compare/**
__device__ __forceinline__ bool atom_cmp(const Atom& A, uint64_t l, uint64_t r) {
  switch (A.dom) {
    case D_F32: return cmpv(A.op, to_f32(l, A.lt), to_f32(r, A.rt));
    case D_F64: return cmpv(A.op, to_f64(l, A.lt), to_f64(r, A.rt));
    case D_I64: return cmpv(A.op, to_i64(l, A.lt), to_i64(r, A.rt));
    case D_I32: return cmpv(A.op, (int32_t)(uint32_t)l, (int32_t)(uint32_t)r);
    default: return cmpv(A.op, l, r);  // BOOL / STRING (dictionary id) equality
  }
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
  uint64_t cp[MAXCAP];     // captured raw attribute words read by later filters
  uint32_t cn;             // captured-null bits
};

__device__ __forceinline__ uint64_t cap_get(const PSet P, int idx) {
  uint64_t v = P.cp[0];
#pragma unroll
  for (int c = 1; c < MAXCAP; ++c) v = (idx == c) ? P.cp[c] : v;
  return v;
}

// operand fetch; `k` indexes the event inside the wave's LDS tile
__device__ __forceinline__ uint64_t fetch(int kind, int idx, int64_t c, const uint64_t* t_attr,
                                          const uint32_t* t_null, int k, const PSet P, bool& nul) {
  switch (kind) {
    case OPK_CUR:
      nul = (t_null[k] >> idx) & 1u;
      return t_attr[idx * WAVE + k];
    case OPK_CAP:
      nul = (P.cn >> idx) & 1u;
      return cap_get(P, idx);
    case OPK_CONST:
      nul = false;
      return (uint64_t)c;
    default:
      nul = true;
      return 0;
  }
}

// conjunction of the atoms of state s (FilterProcessor chain, null -> false)
__device__ __forceinline__ bool eval_state(const ChainQuery& Q, int s, const uint64_t* t_attr,
                                           const uint32_t* t_null, int k, const PSet P) {
  bool ok = true;
  const int a0 = Q.atom_begin[s], a1 = Q.atom_begin[s + 1];
  for (int a = a0; a < a1; ++a) {
    const Atom& A = Q.atoms[a];
    bool ln, rn;
    uint64_t l = fetch(A.lk, A.la, A.lc, t_attr, t_null, k, P, ln);
    uint64_t r = fetch(A.rk, A.ra, A.rc, t_attr, t_null, k, P, rn);
    ok = ok && !ln && !rn && atom_cmp(A, l, r);
  }
  return ok;
}

__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// first index i in [0, c0) with ts[i] >= target (64-ary search, all lanes cooperate)
__device__ int64_t lower_bound_ts(const int64_t* ts, int64_t c0, int64_t target, int lane) {
  int64_t lo = 0, hi = c0;  // answer in [lo, hi]
  while (hi - lo > 1) {
    int64_t span = hi - lo;
    int64_t p = lo + (span * lane) / WAVE;   // probe positions, p < hi
    bool below = ts[p] < target;
    uint64_t m = __ballot(below);
    int nb = __popcll(m);                    // ts is sorted: the first nb probes are below
    int64_t nlo = nb == 0 ? lo : lo + (span * (nb - 1)) / WAVE + 1;
    int64_t nhi = nb == WAVE ? hi : lo + (span * nb) / WAVE;
    lo = rfl64(nlo);
    hi = rfl64(nhi);
    if (nlo == nhi) break;
  }
  if (lo < c0 && ts[lo] < target) lo = lo + 1;
  return lo;
}

template <int S, int K>
__global__ __launch_bounds__(256) void nfa_chain_kernel(ChainLaunch L) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + wv;
  if (wid >= L.n_work) return;
  const WorkItem W = L.work[wid];
  const ChainQuery* __restrict__ Qp = L.queries + W.q;
  const ChainQuery& Q = *Qp;
  // wave-uniform program fields kept in SGPRs for the whole chunk
  const int64_t within = Q.within;
  const int every = Q.every, n_cap = Q.n_cap, qid = Q.qid;
  int sstream[S];
#pragma unroll
  for (int s = 0; s < S; ++s) sstream[s] = Q.state_stream[s];
  const int na = L.b.n_attr;
  uint64_t* t_attr = smem + (size_t)wv * WAVE * (na + 2);
  int64_t* t_ts = (int64_t*)(t_attr + WAVE * na);
  uint32_t* t_null = (uint32_t*)(t_attr + WAVE * (na + 1));
  const int stream = L.b.stream;
  const int pcap = L.pcap;

  // ---- start state: persisted table (chunk 0 / window reaching the batch start) or replay ----
  int64_t w0 = 0;
  if (W.chunk > 0) {
    int64_t target = L.b.ts[W.c0 - 1] - within;
    w0 = lower_bound_ts(L.b.ts, W.c0, target, lane);
  }
  PSet P[K];
  int seed_alive = 1;
  const int64_t* pin = L.part[W.inb] + (size_t)W.q * NF * pcap;
  if (w0 == 0) {
    seed_alive = L.hdr[W.inb][W.q].seed_alive;
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      const int li = kk * WAVE + lane;
      P[kk].st = (int)pin[F_STATE * pcap + li];
      P[kk].ts0 = pin[F_TS0 * pcap + li];
#pragma unroll
      for (int s = 0; s < MAXS - 1; ++s) P[kk].sq[s] = pin[(F_SEQ0 + s) * pcap + li];
#pragma unroll
      for (int c = 0; c < MAXCAP; ++c) P[kk].cp[c] = (uint64_t)pin[(F_CAP0 + c) * pcap + li];
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
    // ---- stage 64 events of the stream in this wave's LDS tile (coalesced column loads) ----
    const int64_t e = t + lane;
    const bool live = e < W.c1;
    int64_t ets = live ? L.b.ts[e] : INT64_MAX;
    uint32_t enull = 0;
    for (int a = 0; a < na; ++a) {
      uint64_t v = 0;
      if (live) {
        const int wdt = L.b.width[a];
        if (wdt == 8) v = ((const uint64_t*)L.b.col[a])[e];
        else if (wdt == 4) v = ((const uint32_t*)L.b.col[a])[e];
        else v = ((const uint8_t*)L.b.col[a])[e];
        if (L.b.nul[a] && ((const uint8_t*)L.b.nul[a])[e]) enull |= 1u << a;
      }
      t_attr[a * WAVE + lane] = v;
    }
    t_ts[lane] = ets;
    t_null[lane] = enull;
    // timestamps must be non-decreasing for chunk warm-up to be exact
    int64_t pred = __shfl_up(ets, 1, WAVE);
    if (lane == 0) pred = prev_tile_ts;
    if (live && ets < pred) unordered = true;
    prev_tile_ts = __shfl(ets, WAVE - 1, WAVE);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    const int cnt = (int)((W.c1 - t) < WAVE ? (W.c1 - t) : WAVE);
    for (int k = 0; k < cnt; ++k) {
      const int64_t j = t + k;
      const bool emit_ok = j >= W.c0;
      const int64_t cts = t_ts[k];
      const int64_t cseq = L.b.seq_base + j;

      // ---- non-start states, last to first (reverse registration order) ----
#pragma unroll
      for (int s = S - 1; s >= 1; --s) {
        if (sstream[s] != stream) continue;
        const bool last = (s == S - 1);
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          const bool in_s = P[kk].st == s;
          if (__ballot(in_s) == 0) continue;
          const bool exp = in_s && within >= 0 && expired(P[kk].ts0, cts, within);
          const bool pass = in_s && !exp && eval_state(Q, s, t_attr, t_null, k, P[kk]);
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
                for (int q2 = 0; q2 < MAXS - 1; ++q2)
                  if (q2 < S - 1) r[2 + q2] = P[kk].sq[q2];
                r[2 + S - 1] = cseq;
              }
              nmatch += __popcll(m);
            }
            if (pass || exp) P[kk].st = -1;
          } else {
            if (exp) P[kk].st = -1;
            if (pass) {
              P[kk].st = s + 1;
#pragma unroll
              for (int q2 = 1; q2 < MAXS - 1; ++q2)
                if (q2 == s) P[kk].sq[q2] = cseq;
              for (int c = 0; c < n_cap; ++c) {
                if (Q.cap_slot[c] != s) continue;
                const int at = Q.cap_attr[c];
                const uint64_t v = t_attr[at * WAVE + k];
                const uint32_t nb = (t_null[k] >> at) & 1u;
#pragma unroll
                for (int c2 = 0; c2 < MAXCAP; ++c2)
                  if (c2 == c) P[kk].cp[c2] = v;
                P[kk].cn = (P[kk].cn & ~(1u << c)) | (nb << c);
              }
            }
          }
        }
      }

      // ---- start state: the seed (every re-arms it, otherwise one match consumes it) ----
      if (seed_alive && sstream[0] == stream) {
        const bool p0 = eval_state(Q, 0, t_attr, t_null, k, P[0]);
        if (__ballot(p0) != 0) {  // uniform: the seed sees only the current event
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
            bool placed = false;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) {
              if (placed) continue;
              const uint64_t freem = ~__ballot(P[kk].st >= 0);
              if (freem == 0) continue;
              placed = true;
              const int fl = __builtin_ctzll(freem);
              if (lane == fl) {
                P[kk].st = 1;
                P[kk].ts0 = cts;
                P[kk].sq[0] = cseq;
                P[kk].cn = 0;
                for (int c = 0; c < n_cap; ++c) {
                  if (Q.cap_slot[c] != 0) continue;
                  const int at = Q.cap_attr[c];
                  const uint64_t v = t_attr[at * WAVE + k];
                  const uint32_t nb = (t_null[k] >> at) & 1u;
#pragma unroll
                  for (int c2 = 0; c2 < MAXCAP; ++c2)
                    if (c2 == c) P[kk].cp[c2] = v;
                  P[kk].cn |= nb << c;
                }
              }
            }
            if (!placed) overflow = true;
          }
          if (!every) seed_alive = 0;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
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
      for (int c = 0; c < MAXCAP; ++c) pout[(F_CAP0 + c) * pcap + li] = (int64_t)P[kk].cp[c];
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

// dense copy of the per-item output segments (for polling)
__global__ void compact_matches_kernel(const int64_t* __restrict__ src, const int64_t* __restrict__ seg_off,
                                       const int64_t* __restrict__ seg_count,
                                       const int64_t* __restrict__ dst_off, int rec_words, int n_items,
                                       int64_t* __restrict__ dst) {
  const int item = blockIdx.x;
  if (item >= n_items) return;
  const int64_t n = seg_count[item] * rec_words;
  const int64_t* s = src + seg_off[item] * rec_words;
  int64_t* d = dst + dst_off[item] * rec_words;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace sdh

// host-side launchers (C linkage inside the library)
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

extern "C" hipError_t sdh_launch_compact(const int64_t* src, const int64_t* seg_off, const int64_t* seg_count,
                                         const int64_t* dst_off, int rec_words, int n_items, int64_t* dst,
                                         hipStream_t s) {
  if (n_items == 0) return hipSuccess;
  hipLaunchKernelGGL(sdh::compact_matches_kernel, dim3(n_items), dim3(256), 0, s, src, seg_off, seg_count,
                     dst_off, rec_words, n_items, dst);
  return hipGetLastError();
}
