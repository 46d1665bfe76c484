// nfa_ratchet.hip -- K_ratchet: NFA step for the 2-state threshold-ratchet pattern family
//
//     every e1=S[f0] -> e2=S[cur.a OP e1.a] [within T]          OP in {<, <=, >, >=}
//
// (BASELINE.json configs[0..1]: `every e1=StockStream[price>T] -> e2=StockStream[price>e1.price]`.)
//
// Reference semantics (state/ = siddhi-core .../query/input/stream/state/):
//   * every pending partial of state 1 is visited on every event of S, in insertion order
//     (StreamPreStateProcessor.processAndReturn:292-337): expired -> removed (isExpired:102-113,
//     checked first); filter passes -> emitted and removed (StreamPostStateProcessor:53-72,
//     stateChanged); otherwise kept
//   * state 1 is visited before state 0 for the same event (reverse registration order,
//     PatternMultiProcessStreamReceiver.java:38-44), and a partial created by event j becomes
//     pending for j+1 (two-phase newAndEvery -> pending, :203-227,281-289)
//   * `every` re-arms the start state with a clone whose start slot is overwritten by the next
//     event (:218-227), so the start state is stateless: every event passing f0 opens a partial
//
// Why a deque is exact: the x-atom is `cur.a OP key` with key = e1.a in the same
// compare domain and no other atom on state 1. After event x is processed every surviving partial
// fails `x OP key` and the partial x opens (if any) has key x, so keys are monotone along the
// pending list: for `>` non-increasing from oldest to newest. The partials x matches are then a
// suffix (the newest) and -- with non-decreasing timestamps -- the expired ones a prefix (the
// oldest). Partials whose key is null or NaN can never match and expire silently: they are not
// observable and are not stored. Out-of-order timestamps switch the group to a full expiry scan.
//
// Mapping to CDNA4: one 64-lane wave = up to 64 same-shape patterns (lane = pattern instance) over
// one event chunk; events are wave-uniform (64-event tiles staged with coalesced loads, read per
// event with v_readlane). Each lane's deque is a ring in LDS ([slot][lane] 16-B entries,
// conflict-free ds_read/write_b128); the top key, bottom ts and bottom seq are cached in VGPRs so an
// event that pops nothing touches no LDS. Matches are compacted with ballot + mbcnt into
// per-wave output blocks (one atomic per 8K records). No MFMA: compare/branch work.
#include <hip/hip_runtime.h>

#include "nfa_types.h"

namespace sdh {

namespace {

__device__ __forceinline__ int wave_mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int64_t rfl64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int k) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, k);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), k);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

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
    default: return (int64_t)raw;
  }
}

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

__device__ __forceinline__ bool expired(int64_t t0, int64_t t, int64_t within) {
  int64_t d = (int64_t)((uint64_t)t0 - (uint64_t)t);
  int64_t a = d < 0 ? (int64_t)(0ull - (uint64_t)d) : d;
  return a > within;
}

__device__ int64_t lower_bound_ts(const int64_t* ts, int64_t c0, int64_t target, int lane) {
  int64_t lo = 0, hi = c0;
  while (hi - lo > 1) {
    const int64_t span = hi - lo;
    const int64_t p = lo + (span * lane) / WAVE;
    const uint64_t m = __ballot(ts[p] < target);
    const int nb = __popcll(m);
    const int64_t nlo = nb == 0 ? lo : lo + (span * (nb - 1)) / WAVE + 1;
    const int64_t nhi = nb == WAVE ? hi : lo + (span * nb) / WAVE;
    lo = rfl64(nlo);
    hi = rfl64(nhi);
    if (lo == hi) break;
  }
  if (lo < c0 && ts[lo] < target) lo = lo + 1;
  return lo;
}

// key of the x-atom operand in the compare domain. 32-bit kinds: binary32 bits / int32;
// 64-bit kinds: binary64 bits / int64. `ok` = usable key (not null, not NaN).
template <int KK>
__device__ __forceinline__ uint64_t stage_key(uint64_t raw, int conv, bool isnull, bool& ok) {
  if (KK == KK_F32) {
    float f;
    switch (conv) {
      case CV_F32_INT: f = (float)(int32_t)(uint32_t)raw; break;
      case CV_F32_LONG: f = (float)(int64_t)raw; break;
      default: f = __uint_as_float((uint32_t)raw);
    }
    ok = !isnull && !(f != f);
    return __float_as_uint(f);
  } else if (KK == KK_I32) {
    ok = !isnull;
    return (uint32_t)raw;
  } else {
    const int64_t k = to_key(raw, conv);
    ok = !isnull && !(KK == KK_F64 && __longlong_as_double(k) != __longlong_as_double(k));
    return (uint64_t)k;
  }
}

// `cur OP key` on stored keys (both valid: no NaN)
template <int KK>
__device__ __forceinline__ bool xcmp(int mask, uint64_t cur, uint64_t key) {
  bool lt, gt;
  if (KK == KK_F32) {
    const float a = __uint_as_float((uint32_t)cur), b = __uint_as_float((uint32_t)key);
    lt = a < b; gt = b < a;
  } else if (KK == KK_I32) {
    const int32_t a = (int32_t)(uint32_t)cur, b = (int32_t)(uint32_t)key;
    lt = a < b; gt = b < a;
  } else if (KK == KK_F64) {
    const double a = __longlong_as_double((int64_t)cur), b = __longlong_as_double((int64_t)key);
    lt = a < b; gt = b < a;
  } else {
    const int64_t a = (int64_t)cur, b = (int64_t)key;
    lt = a < b; gt = b < a;
  }
  const bool eq = !lt && !gt;
  return (lt && (mask & CM_LT)) || (gt && (mask & CM_GT)) || (eq && (mask & CM_EQ));
}

// pick element idx (wave-uniform) of a by-value kernel-argument array without indexing it
// dynamically (which would copy the argument into scratch)
template <class T, int N>
__device__ __forceinline__ T pick(const T (&arr)[N], int idx) {
  T v = arr[0];
#pragma unroll
  for (int c = 1; c < N; ++c) v = (idx == c) ? arr[c] : v;
  return v;
}

__device__ __forceinline__ uint64_t load_raw(const void* p, int width, int64_t e) {
  return width == 8 ? ((const uint64_t*)p)[e] : width == 4 ? ((const uint32_t*)p)[e] : ((const uint8_t*)p)[e];
}

}  // namespace

// LDS ring per lane, entry (slot e, lane l) at index e*64 + l:
//   A: uint4 {ts0.lo, ts0.hi, key.lo, key.hi}       B: uint32 seq (low 32 bits of e1's sequence)
template <int KK, bool FULL>
__global__ __launch_bounds__(64) void nfa_ratchet_kernel(RatchetLaunch L, int M) {
  extern __shared__ uint4 lds[];
  uint4* __restrict__ A = lds;
  uint32_t* __restrict__ B = reinterpret_cast<uint32_t*>(lds + (size_t)M * WAVE);
  const int lane = threadIdx.x;
  const int wid = blockIdx.x;
  if (wid >= L.n_items) return;
  const RatchetItem W = L.items[wid];
  const RatchetGroup* __restrict__ G = L.groups + W.g;
  const int mask = M - 1;
  const bool active = lane < G->n_lanes;
  const int64_t qid = G->qid[lane & 63];
  const int64_t within = G->within[lane & 63];
  const int64_t wmax = G->wmax;
  const bool has_within = wmax >= 0;
  const int n_f0 = G->n_f0;
  const int xmask = G->xmask, kconv = G->key_conv, kattr = G->key_attr;
  // f0 atoms: per-lane constants; operand columns resolved once (wave-uniform)
  int64_t f0c[RMAXF0];
  int f_left[RMAXF0], f_mask[RMAXF0], f_f64[RMAXF0], f_cur2[RMAXF0], f_conv[RMAXF0], f_conv2[RMAXF0];
  int f_w[RMAXF0], f_w2[RMAXF0];
  const void* f_ptr[RMAXF0];
  const void* f_ptr2[RMAXF0];
  const uint8_t* f_nul[RMAXF0];
  const uint8_t* f_nul2[RMAXF0];
#pragma unroll
  for (int a = 0; a < RMAXF0; ++a) {
    f0c[a] = a < n_f0 ? G->f0c[a][lane & 63] : 0;
    const RatchetAtom A0 = G->f0[a];
    f_left[a] = A0.cur_left; f_mask[a] = A0.mask; f_f64[a] = A0.f64; f_cur2[a] = A0.cur2;
    f_conv[a] = A0.conv; f_conv2[a] = A0.conv2;
    f_ptr[a] = pick(L.b.col, A0.attr); f_w[a] = pick(L.b.width, A0.attr); f_nul[a] = pick(L.b.nul, A0.attr);
    f_ptr2[a] = pick(L.b.col, A0.attr2); f_w2[a] = pick(L.b.width, A0.attr2); f_nul2[a] = pick(L.b.nul, A0.attr2);
  }
  const void* k_ptr = pick(L.b.col, kattr);
  const uint8_t* k_nul = pick(L.b.nul, kattr);
  const int k_w = pick(L.b.width, kattr);

  // ---- initial deque: persisted (window reaches the batch start) or empty (warm-up replay) ----
  int64_t w0 = 0;
  if (W.chunk > 0 && !FULL) w0 = lower_bound_ts(L.b.ts, W.c0, L.b.ts[W.c0 - 1] - wmax, lane);
  int n = 0, bot = 0;
  if (w0 == 0) {
    const size_t gb = (size_t)W.g * RSMAX * WAVE;
    n = pick(L.st, W.inb)[W.g].n[lane];
    const int64_t* __restrict__ i_ts = pick(L.ent_ts, W.inb);
    const int64_t* __restrict__ i_sq = pick(L.ent_seq, W.inb);
    const int64_t* __restrict__ i_ky = pick(L.ent_key, W.inb);
    for (int i = 0; i < n; ++i) {
      const size_t o = gb + (size_t)i * WAVE + lane;
      const int64_t t0 = i_ts[o];
      const int64_t sq = i_sq[o];
      const int64_t ky = i_ky[o];
      A[i * WAVE + lane] = make_uint4((uint32_t)t0, (uint32_t)((uint64_t)t0 >> 32), (uint32_t)ky,
                                      (uint32_t)((uint64_t)ky >> 32));
      B[i * WAVE + lane] = (uint32_t)sq;
    }
  }
  // VGPR caches of the deque ends
  uint64_t tkey = 0;
  uint32_t tseq = 0, bseq = 0;
  int64_t bts = 0;
  if (n > 0) {
    const uint4 t = A[((n - 1) & mask) * WAVE + lane];
    tkey = (uint64_t)t.z | ((uint64_t)t.w << 32);
    tseq = B[((n - 1) & mask) * WAVE + lane];
    const uint4 b = A[lane];
    bts = (int64_t)((uint64_t)b.x | ((uint64_t)b.y << 32));
    bseq = B[lane];
  }

  int blk = -1, fill = 0;
  bool overflow = false, unordered = false, mover = false, aged = false;
  int64_t prev_tile_ts = (w0 == 0) ? L.b.prev_ts : L.b.ts[w0 - 1];
  const int64_t seq_base = L.b.seq_base;
  const int RW = 4;

  for (int64_t t = w0; t < W.c1; t += WAVE) {
    // ---- stage 64 events (lane = event): ts, x-atom key, f0 column keys, validity bits ----
    const int64_t e = t + lane;
    const bool live = e < W.c1;
    const int64_t ets = live ? L.b.ts[e] : INT64_MAX;
    uint64_t xk = 0;
    bool xok = false;
    if (live) {
      const uint64_t raw = load_raw(k_ptr, k_w, e);
      const bool nl = k_nul && k_nul[e];
      xk = stage_key<KK>(raw, kconv, nl, xok);
    }
    // f0 operand keys, one per atom (lane = event)
    int64_t fk[RMAXF0], fk2[RMAXF0];
    uint32_t fnul = 0;
#pragma unroll
    for (int a = 0; a < RMAXF0; ++a) {
      fk[a] = 0;
      fk2[a] = 0;
      if (a < n_f0 && live) {
        fk[a] = to_key(load_raw(f_ptr[a], f_w[a], e), f_conv[a]);
        bool nl = f_nul[a] && f_nul[a][e];
        if (f_cur2[a]) {
          fk2[a] = to_key(load_raw(f_ptr2[a], f_w2[a], e), f_conv2[a]);
          nl = nl || (f_nul2[a] && f_nul2[a][e]);
        }
        if (nl) fnul |= 1u << a;
      }
    }
    const uint32_t vbits = (xok ? 1u : 0u) | (fnul << 1);
    int64_t pred = __shfl_up(ets, 1, WAVE);
    if (lane == 0) pred = prev_tile_ts;
    if (live && ets < pred) unordered = true;
    prev_tile_ts = __shfl(ets, WAVE - 1, WAVE);

    const int cnt = (int)((W.c1 - t) < WAVE ? (W.c1 - t) : WAVE);
#pragma unroll 1
    for (int k = 0; k < cnt; ++k) {
      const int64_t j = t + k;
      const bool emit_ok = j >= W.c0;
      const int64_t tt = readlane64(ets, k);
      const int64_t s = seq_base + j;
      const uint32_t slo = (uint32_t)s;
      const uint32_t vb = __builtin_amdgcn_readlane(vbits, k);
      const uint64_t x = (KK == KK_F32 || KK == KK_I32) ? (uint64_t)__builtin_amdgcn_readlane((uint32_t)xk, k)
                                                         : (uint64_t)readlane64((int64_t)xk, k);
      const bool x_ok = vb & 1u;

      // ---- 1. lazy `within` expiry (oldest first) ----
      if (has_within) {
        if (!FULL) {
          while (true) {
            const bool ex = n > 0 && expired(bts, tt, within);
            if (__ballot(ex) == 0) break;
            if (ex) {
              bot = (bot + 1) & mask;
              --n;
              if (n > 0) {
                const uint4 b = A[bot * WAVE + lane];
                bts = (int64_t)((uint64_t)b.x | ((uint64_t)b.y << 32));
                bseq = B[bot * WAVE + lane];
              }
            }
          }
        } else {
          // timestamps out of order: the expired partials are no longer a prefix
          int w = 0;
          for (int i = 0; i < n; ++i) {
            const int si = (bot + i) & mask;
            const uint4 a = A[si * WAVE + lane];
            const int64_t t0 = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
            if (!expired(t0, tt, within)) {
              const int di = (bot + w) & mask;
              if (di != si) {
                A[di * WAVE + lane] = a;
                B[di * WAVE + lane] = B[si * WAVE + lane];
              }
              ++w;
            }
          }
          n = w;
          if (n > 0) {
            const uint4 b = A[bot * WAVE + lane];
            bts = (int64_t)((uint64_t)b.x | ((uint64_t)b.y << 32));
            bseq = B[bot * WAVE + lane];
            const int ti = (bot + n - 1) & mask;
            const uint4 tp = A[ti * WAVE + lane];
            tkey = (uint64_t)tp.z | ((uint64_t)tp.w << 32);
            tseq = B[ti * WAVE + lane];
          }
        }
      }
      // sequence numbers are kept as their low 32 bits: a live partial must be < 2^31 events old
      if (n > 0 && (slo - bseq) >= 0x80000000u) aged = true;

      // ---- 2. matches: the newest partials whose key satisfies `cur OP key` ----
      while (true) {
        const bool mt = x_ok && n > 0 && xcmp<KK>(xmask, x, tkey);
        const uint64_t m = __ballot(mt);
        if (m == 0) break;
        if (emit_ok && !mover) {
          const int c = __popcll(m);
          if (fill + c > L.blk_recs) {
            if (blk >= 0 && lane == 0) L.blk_count[blk] = fill;
            blk = -1;
          }
          if (blk < 0) {
            int nb = 0;
            if (lane == 0) nb = atomicAdd(L.blk_next, 1);
            nb = __builtin_amdgcn_readfirstlane(nb);
            if (nb >= L.n_blocks) {
              mover = true;
            } else {
              blk = nb;
              fill = 0;
            }
          }
          if (!mover) {
            if (mt) {
              const int64_t s1 = s - (int64_t)(uint32_t)(slo - tseq);
              int64_t* r = L.match + ((size_t)blk * L.blk_recs + fill + wave_mbcnt(m)) * RW;
              reinterpret_cast<longlong2*>(r)[0] = make_longlong2(qid, tt);
              reinterpret_cast<longlong2*>(r)[1] = make_longlong2(s1, s);
            }
            fill += c;
          }
        }
        if (mt) {
          --n;
          if (n > 0) {
            const int ti = (bot + n - 1) & mask;
            const uint4 tp = A[ti * WAVE + lane];
            tkey = (uint64_t)tp.z | ((uint64_t)tp.w << 32);
            tseq = B[ti * WAVE + lane];
          }
        }
      }

      // ---- 3. start state: every event passing f0 opens a partial (pending from j+1) ----
      bool f0ok = active && x_ok;
#pragma unroll
      for (int a = 0; a < RMAXF0; ++a) {
        if (a < n_f0) {
          const int64_t cv = readlane64(fk[a], k);
          const bool cn = (vb >> (1 + a)) & 1u;
          bool ok;
          if (f_cur2[a]) {
            ok = !cn && cmp_keys(f_mask[a], f_f64[a], cv, readlane64(fk2[a], k));
          } else {
            ok = !cn && (f_left[a] ? cmp_keys(f_mask[a], f_f64[a], cv, f0c[a])
                                   : cmp_keys(f_mask[a], f_f64[a], f0c[a], cv));
          }
          f0ok = f0ok && ok;
        }
      }
      if (f0ok) {
        if (n == M) {
          overflow = true;
        } else {
          const int ti = (bot + n) & mask;
          A[ti * WAVE + lane] = make_uint4((uint32_t)tt, (uint32_t)((uint64_t)tt >> 32), (uint32_t)x,
                                           (uint32_t)(x >> 32));
          B[ti * WAVE + lane] = slo;
          if (n == 0) {
            bts = tt;
            bseq = slo;
          }
          ++n;
          tkey = x;
          tseq = slo;
        }
      }
    }
  }

  // ---- outputs ----
  if (blk >= 0 && lane == 0) L.blk_count[blk] = fill;
  const uint64_t any_over = __ballot(overflow), any_unord = __ballot(unordered), any_aged = __ballot(aged);
  if (lane == 0) {
    if (any_over) atomicOr(&L.err[0], 1);
    if (any_unord) atomicOr(&L.err[1], 1);
    if (mover) atomicOr(&L.err[2], 1);
    if (any_aged) atomicOr(&L.err[3], 1);
  }
  if (W.chunk == W.n_chunks - 1) {  // the last chunk owns the group's final deques
    const int ob = 1 - W.inb;
    const size_t gb = (size_t)W.g * RSMAX * WAVE;
    const int64_t slast = seq_base + W.c1 - 1;
    const uint32_t llo = (uint32_t)slast;
    int64_t* __restrict__ o_ts = pick(L.ent_ts, ob);
    int64_t* __restrict__ o_sq = pick(L.ent_seq, ob);
    int64_t* __restrict__ o_ky = pick(L.ent_key, ob);
    for (int i = 0; i < n; ++i) {
      const int si = (bot + i) & mask;
      const uint4 a = A[si * WAVE + lane];
      const size_t o = gb + (size_t)i * WAVE + lane;
      o_ts[o] = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
      o_ky[o] = (int64_t)((uint64_t)a.z | ((uint64_t)a.w << 32));
      o_sq[o] = slast - (int64_t)(uint32_t)(llo - B[si * WAVE + lane]);
    }
    pick(L.st, ob)[W.g].n[lane] = n;
  }
}

}  // namespace sdh

template <int KK>
static hipError_t launch_kk(bool full, const sdh::RatchetLaunch* L, int M, hipStream_t s) {
  const size_t lds = (size_t)M * 64 * (sizeof(uint4) + sizeof(uint32_t));
  if (full)
    hipLaunchKernelGGL((sdh::nfa_ratchet_kernel<KK, true>), dim3(L->n_items), dim3(64), lds, s, *L, M);
  else
    hipLaunchKernelGGL((sdh::nfa_ratchet_kernel<KK, false>), dim3(L->n_items), dim3(64), lds, s, *L, M);
  return hipGetLastError();
}

extern "C" hipError_t sdh_launch_ratchet(int key_kind, int full, int M, const sdh::RatchetLaunch* L,
                                         hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  if (M < 1 || (M & (M - 1)) || M > sdh::RSMAX) return hipErrorInvalidValue;
  switch (key_kind) {
    case sdh::KK_F32: return launch_kk<sdh::KK_F32>(full, L, M, s);
    case sdh::KK_I32: return launch_kk<sdh::KK_I32>(full, L, M, s);
    case sdh::KK_F64: return launch_kk<sdh::KK_F64>(full, L, M, s);
    case sdh::KK_I64: return launch_kk<sdh::KK_I64>(full, L, M, s);
    default: return hipErrorInvalidValue;
  }
}
