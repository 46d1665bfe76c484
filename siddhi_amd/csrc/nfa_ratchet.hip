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
#include "ratchet_common.h"

#ifndef SDH_RATCHET_UNROLL
#define SDH_RATCHET_UNROLL 1
#endif
#ifndef SDH_RATCHET_NOSTORE
#define SDH_RATCHET_NOSTORE 0
#endif
#define SDH_PRAGMA(x) _Pragma(#x)
#define SDH_UNROLL(n) SDH_PRAGMA(unroll n)

namespace sdh {

extern __shared__ uint4 ratchet_lds[];

// Spill / persisted entries: 32-bit keys A = uint4 {ts0.lo, ts0.hi, key, seq};
// 64-bit keys A = uint4 {ts0.lo, ts0.hi, key.lo, key.hi}, B = uint32 seq.
// (seq = low 32 bits of e1's global sequence number; a live partial is < 2^31 events old)
template <int KK>
__device__ __forceinline__ uint4 pack_entry(int64_t ts, typename KT<KK>::U key, uint32_t seq) {
  if constexpr (KT<KK>::W64)
    return make_uint4((uint32_t)ts, (uint32_t)((uint64_t)ts >> 32), (uint32_t)key, (uint32_t)(key >> 32));
  else
    return make_uint4((uint32_t)ts, (uint32_t)((uint64_t)ts >> 32), key, seq);
}

template <int KK>
__device__ __forceinline__ void unpack_entry(uint4 a, uint32_t b, int64_t& ts, typename KT<KK>::U& key, uint32_t& seq) {
  ts = (int64_t)((uint64_t)a.x | ((uint64_t)a.y << 32));
  if constexpr (KT<KK>::W64) {
    key = (uint64_t)a.z | ((uint64_t)a.w << 32);
    seq = b;
  } else {
    key = a.z;
    seq = a.w;
  }
}

// Two-level per-lane deque: the newest ML entries in an LDS ring (ratchet_lds, [slot][lane]),
// older ones in a global spill ring of SC entries (oldest first: spill, then LDS). Pops happen at
// the newest end (LDS), expiry at the oldest end; the spill is touched only while a lane holds
// more than ML pending partials. LDS ring entries hold only what the pops read -- {key, seq},
// 8 B for 32-bit keys -- and their ts0 lives in a per-lane HBM side ring (LT) that is read only
// when an entry becomes the oldest (expiry deadline) or leaves LDS; half-size entries double the
// waves an LDS-limited CU holds.
template <int KK>
struct Deque {
  using U = typename KT<KK>::U;
  uint4* SA;
  uint32_t* SB;
  int64_t* LT;
  int lane, lmask, smask, ML, SC;
  size_t sbase;   // (item * SC) * 64
  size_t ltbase;  // (item * ML) * 64
  int lbot = 0, ln = 0, sbot = 0, sn = 0;
  __device__ __forceinline__ int li(int slot) const { return (slot & lmask) * WAVE + lane; }
  __device__ __forceinline__ size_t si(int slot) const { return sbase + (size_t)(slot & smask) * WAVE + lane; }
  // ts0 of an LDS entry: events of the current batch read it back from the batch's ts column,
  // older (carried) partials from the side ring LT, written when they enter the LDS ring
  const int64_t* bts;  // batch timestamps
  int64_t seq_base;    // global seq of batch event 0
  int64_t sref;        // a seq >= every held entry's, within 2^31 (the item's last event)
  __device__ __forceinline__ int64_t full_seq(uint32_t seq_lo) const {
    return sref - (int64_t)(uint32_t)((uint32_t)sref - seq_lo);
  }
  __device__ __forceinline__ void lput_ks(int i, U key, uint32_t seq) const {
    if constexpr (KT<KK>::W64) ratchet_lds[i] = make_uint4((uint32_t)key, (uint32_t)(key >> 32), seq, 0u);
    else reinterpret_cast<uint2*>(ratchet_lds)[i] = make_uint2(key, seq);
  }
  __device__ __forceinline__ void lput(int i, int64_t ts, U key, uint32_t seq) const {
    lput_ks(i, key, seq);
    if (full_seq(seq) < seq_base) LT[ltbase + i] = ts;
  }
  __device__ __forceinline__ void lget_ks(int i, U& key, uint32_t& seq) const {
    if constexpr (KT<KK>::W64) {
      const uint4 a = ratchet_lds[i];
      key = (uint64_t)a.x | ((uint64_t)a.y << 32);
      seq = a.z;
    } else {
      const uint2 a = reinterpret_cast<const uint2*>(ratchet_lds)[i];
      key = a.x;
      seq = a.y;
    }
  }
  __device__ __forceinline__ void lget(int i, int64_t& ts, U& key, uint32_t& seq) const {
    lget_ks(i, key, seq);
    const int64_t k = full_seq(seq) - seq_base;
    ts = k >= 0 ? bts[k] : LT[ltbase + i];
  }
  __device__ __forceinline__ void sput(size_t i, int64_t ts, U key, uint32_t seq) const {
    SA[i] = pack_entry<KK>(ts, key, seq);
    if constexpr (KT<KK>::W64) SB[i] = seq;
  }
  __device__ __forceinline__ void sget(size_t i, int64_t& ts, U& key, uint32_t& seq) const {
    uint32_t b = 0;
    if constexpr (KT<KK>::W64) b = SB[i];
    unpack_entry<KK>(SA[i], b, ts, key, seq);
  }
  __device__ __forceinline__ int n() const { return ln + sn; }
  // i-th entry counted from the oldest
  __device__ __forceinline__ void at(int i, int64_t& ts, U& key, uint32_t& seq) const {
    if (i < sn) sget(si(sbot + i), ts, key, seq);
    else lget(li(lbot + i - sn), ts, key, seq);
  }
  __device__ __forceinline__ void top(int64_t& ts, U& key, uint32_t& seq) const { at(n() - 1, ts, key, seq); }
  __device__ __forceinline__ void bottom(int64_t& ts, U& key, uint32_t& seq) const { at(0, ts, key, seq); }
  // low seq bits of the oldest entry (n() > 0), without its ts0
  __device__ __forceinline__ uint32_t bottom_seq() const {
    if (sn > 0) {
      if constexpr (KT<KK>::W64) return SB[si(sbot)];
      else return SA[si(sbot)].w;
    }
    U k;
    uint32_t q;
    lget_ks(li(lbot), k, q);
    return q;
  }
  // append the newest entry; returns false on overflow
  __device__ __forceinline__ bool push_back(int64_t ts, U key, uint32_t seq) {
    if (ln == ML) {
      if (sn == SC) return false;
      int64_t t0; U k0; uint32_t q0;
      lget(li(lbot), t0, k0, q0);
      sput(si(sbot + sn), t0, k0, q0);
      ++sn;
      lbot = (lbot + 1) & lmask;
      --ln;
    }
    lput(li(lbot + ln), ts, key, seq);
    ++ln;
    return true;
  }
  // prepend an entry older than all held ones (reverse-scan warm-up); false on overflow
  __device__ __forceinline__ bool push_front(int64_t ts, U key, uint32_t seq) {
    if (sn == 0 && ln < ML) {
      lbot = (lbot - 1) & lmask;
      lput(li(lbot), ts, key, seq);
      ++ln;
      return true;
    }
    if (sn == SC) return false;
    sbot = (sbot - 1) & smask;
    sput(si(sbot), ts, key, seq);
    ++sn;
    return true;
  }
  __device__ __forceinline__ void pop_back(int p) {  // p <= ln, or p == 1
    if (ln > 0) ln -= p;
    else sn -= p;
  }
  __device__ __forceinline__ void pop_front() {
    if (sn > 0) { sbot = (sbot + 1) & smask; --sn; }
    else { lbot = (lbot + 1) & lmask; --ln; }
  }
  // timestamps out of order: drop every expired entry, keeping the order of the rest
  __device__ void compact_expired(int64_t tt, int64_t within) {
    int w = 0;
    for (int i = 0; i < sn; ++i) {
      int64_t t0; U k; uint32_t q;
      sget(si(sbot + i), t0, k, q);
      if (!expired(t0, tt, within)) {
        if (w != i) sput(si(sbot + w), t0, k, q);
        ++w;
      }
    }
    sn = w;
    w = 0;
    for (int i = 0; i < ln; ++i) {
      int64_t t0; U k; uint32_t q;
      lget(li(lbot + i), t0, k, q);
      if (!expired(t0, tt, within)) {
        if (w != i) lput(li(lbot + w), t0, k, q);
        ++w;
      }
    }
    ln = w;
  }
};

// SIM (the C2 family's form): 32-bit float keys, one start atom on the key's own float column with a
// plain interval (no negation), no null masks. The start filter is then two float compares of the
// event key against per-lane float bounds, and NaN keys fail every compare by themselves, so the
// per-event validity bits are not read; an empty deque's top key is NaN, so the match test needs no
// length check; a non-pushing lane writes its LDS entry to a dummy row instead of branching.
// PM (normal-mode pushes that qualify for the direct R18 placement; RatchetLaunch): 0 / 3 = 8-B /
// 16-B match records in per-wave blocks; 1 = COUNT, each (event, group) match total only (one coalesced store
// per 64-event tile); 2 = WRITE, the same step again writing every match as its compact row at its
// final R18 row. A lane's rows at an event are consecutive and the group's lanes hold consecutive
// ranks, so a row is base(event, group) + the matches of the lower lanes + the lane's count - 1 -
// the pop level; the count is known before the first pop: the first round's four compares give it
// unless a lane popped all four or ran through its LDS entries, and then a walk down the deque
// counts the rest (keys are monotone along it). The lower lanes' matches are mbcnt over the first
// round's ballots, a wave scan in the rare walk case.
template <int KK, int XM, bool FULL, int NF, bool SIM = false, int PM = 0, int MLC = 0>
// occupancy: the general forms at 7 waves per SIMD (72 VGPRs), the SIM form at 8 (64 VGPRs, a few
// spills; the LDS rings allow 8 at ML = 8). SIM at 10K C2 patterns: 7 waves 167.9 ms, 8 waves 156.1
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SIM ? 8 : 7))) void nfa_ratchet_kernel(RatchetLaunch L, int ML_, int SC) {
  // MLC > 0: the LDS ring depth as a compile-time constant (the SIM launches at the default 8): the
  // ring masks and the full-ring test then take no scalar registers, whose spills were reloaded at
  // every event
  const int ML = MLC > 0 ? MLC : ML_;
  using U = typename KT<KK>::U;
  constexpr bool W64 = KT<KK>::W64;
  const int lane = threadIdx.x;
  const int wid = blockIdx.x;
  if (wid >= L.n_items) return;
  const RatchetItem W = L.items[wid];
  const RatchetGroup* __restrict__ G = L.groups + W.g;
  Deque<KK> D;
  D.SA = L.spillA;
  D.SB = L.spillB;
  D.LT = L.lds_ts;
  D.ltbase = ((size_t)wid * ML) * WAVE;
  D.bts = L.b.ts;
  D.seq_base = L.b.seq_base;
  D.sref = L.b.seq_base + W.c1 - 1;
  D.lane = lane;
  D.ML = ML;
  D.SC = SC;
  D.lmask = ML - 1;
  D.smask = SC - 1;
  D.sbase = ((size_t)wid * SC) * WAVE;
  const bool active = lane < G->n_lanes;
  const int64_t within = G->within[lane & 63];
  const int32_t w32 = within >= INT32_MAX ? INT32_MAX : (int32_t)within;  // (within >= 0)
  const int64_t T0 = L.b.ts[W.c0];  // the 32-bit deadline domain's origin (rel_deadline)
  const int64_t wmax = G->wmax;
  const bool has_within = wmax >= 0;
  const int n_f0 = G->n_f0;
  const int xmask = G->xmask, kconv = G->key_conv, kattr = G->key_attr;
  const bool is_max = (xmask & CM_GT) != 0;
  // one-atom launches carry only constant-interval atoms (the host routes groups with a two-column
  // atom to the general variant), so their per-event start filter has no operand-kind branch
  constexpr bool IV = (NF == 1);
  // f0 atoms: constant atoms become per-lane intervals of sortable keys; two-column atoms stay
  // generic compares. Operand columns are resolved once (wave-uniform).
  int64_t f_lo[NF], f_hi[NF];
  bool f_neg[NF];
  int f_mask[NF], f_f64[NF], f_cur2[NF], f_conv[NF], f_conv2[NF];
  int f_w[NF], f_w2[NF];
  const void* f_ptr[NF];
  const void* f_ptr2[NF];
  const uint8_t* f_nul[NF];
  const uint8_t* f_nul2[NF];
#pragma unroll
  for (int a = 0; a < NF; ++a) {
    const RatchetAtom A0 = G->f0[a];
    const int64_t c = a < n_f0 ? G->f0c[a][lane & 63] : 0;
    int m = A0.mask;
    if (!A0.cur_left && !A0.cur2) {  // `c OP cur` -> `cur OP' c`
      const int lt = m & CM_LT, gt = m & CM_GT;
      m = (m & (CM_EQ | CM_NOT)) | (lt ? CM_GT : 0) | (gt ? CM_LT : 0);
    }
    f_mask[a] = m;
    f_f64[a] = A0.f64;
    f_cur2[a] = A0.cur2;
    f_conv[a] = A0.conv;
    f_conv2[a] = A0.conv2;
    f0_interval(m, A0.f64 != 0, c, f_lo[a], f_hi[a], f_neg[a]);
    f_ptr[a] = pick(L.b.col, A0.attr); f_w[a] = pick(L.b.width, A0.attr); f_nul[a] = pick(L.b.nul, A0.attr);
    f_ptr2[a] = pick(L.b.col, A0.attr2); f_w2[a] = pick(L.b.width, A0.attr2); f_nul2[a] = pick(L.b.nul, A0.attr2);
  }
  // SIM: the start atom's interval of sortable binary64 keys as binary32 bounds (x in [flo, fhi] iff
  // the widened key is in the interval; idle lanes get an empty one)
  float flo = 0.f, fhi = 0.f;
  if constexpr (SIM) {
    auto unsort = [](int64_t v) { return __longlong_as_double(v >= 0 ? v : (v ^ INT64_MAX)); };
    if (!active || f_lo[0] > f_hi[0]) {
      flo = __int_as_float(0x7f800000);   // +inf
      fhi = __int_as_float((int)0xff800000u);  // -inf
    } else {
      const double lo = f_lo[0] <= INT64_MIN + 1 ? -__longlong_as_double(0x7ff0000000000000ll) : unsort(f_lo[0]);
      const double hi = f_hi[0] == INT64_MAX ? __longlong_as_double(0x7ff0000000000000ll) : unsort(f_hi[0]);
      // the least float >= lo and the greatest float <= hi (one ulp step from the nearest; from +-0
      // the step is the least denormal of the right sign)
      flo = (float)lo;
      if (flo == 0.f && lo > 0.0) flo = __int_as_float(1);
      else if ((double)flo < lo) flo = __int_as_float(__float_as_int(flo) + (flo > 0.f ? 1 : -1));
      fhi = (float)hi;
      if (fhi == 0.f && hi < 0.0) fhi = __int_as_float((int)0x80000001u);
      else if ((double)fhi > hi) fhi = __int_as_float(__float_as_int(fhi) + (fhi > 0.f ? -1 : 1));
    }
  }
  const U TSENT = SIM ? (U)0x7fc00000u : (U)0;  // SIM: the top key of an empty deque (NaN)
  const void* k_ptr = pick(L.b.col, kattr);
  const uint8_t* k_nul = pick(L.b.nul, kattr);
  const int k_w = pick(L.b.width, kattr);
  const int64_t seq_base = L.b.seq_base;

  // stage one event per lane in two halves so that the next tile's loads are in flight while
  // the current tile is processed: load() issues the global loads, convert() builds ts, the
  // x-atom key, the f0 operand keys (sortable) and the validity bits
  struct Raw {
    int64_t ts;
    uint64_t k;
    uint64_t f[NF], f2[NF];
    uint32_t nul;  // bit 0: key null, 1+a: f0 atom a null
    bool live;
  };
  int64_t fk[NF], fk2[NF];
  auto load = [&](int64_t e, bool live, Raw& r) {
    r.live = live;
    r.ts = live ? L.b.ts[e] : INT64_MAX;
    r.k = live ? load_raw(k_ptr, k_w, e) : 0;
    uint32_t nl = (live && k_nul && k_nul[e]) ? 1u : 0u;
#pragma unroll
    for (int a = 0; a < NF; ++a) {
      r.f[a] = 0;
      r.f2[a] = 0;
      if (a < n_f0 && live) {
        r.f[a] = load_raw(f_ptr[a], f_w[a], e);
        bool n1 = f_nul[a] && f_nul[a][e];
        if (!IV && f_cur2[a]) {
          r.f2[a] = load_raw(f_ptr2[a], f_w2[a], e);
          n1 = n1 || (f_nul2[a] && f_nul2[a][e]);
        }
        if (n1) nl |= 2u << a;
      }
    }
    r.nul = nl;
  };
  auto convert = [&](const Raw& r, int64_t& ets, U& xk, uint32_t& vbits) {
    ets = r.ts;
    bool xok = false;
    xk = r.live ? (U)stage_key<KK>(r.k, kconv, (r.nul & 1u) != 0, xok) : (U)0;
#pragma unroll
    for (int a = 0; a < NF; ++a) {
      fk[a] = 0;
      fk2[a] = 0;
      if (a < n_f0 && r.live) {
        const int64_t k1 = to_key(r.f[a], f_conv[a]);
        if (!IV && f_cur2[a]) {
          fk[a] = k1;
          fk2[a] = to_key(r.f2[a], f_conv2[a]);
        } else {
          fk[a] = f_f64[a] ? sortable_f64(k1) : k1;
        }
      }
    }
    vbits = (xok ? 1u : 0u) | (r.nul & ~1u);
  };
  auto stage = [&](int64_t e, bool live, int64_t& ets, U& xk, uint32_t& vbits) {
    Raw r;
    load(e, live, r);
    convert(r, ets, xk, vbits);
  };
  // f0 of this lane's pattern on staged event k
  auto f0_pass = [&](int k, uint32_t vb) {
    bool ok = active && (vb & 1u);
#pragma unroll
    for (int a = 0; a < NF; ++a) {
      if (a < n_f0) {
        const int64_t v = readlane64(fk[a], k);
        const bool cn = (vb >> (1 + a)) & 1u;
        bool r;
        if (!IV && f_cur2[a]) r = cmp_keys(f_mask[a], f_f64[a], v, readlane64(fk2[a], k));
        else r = ((v >= f_lo[a]) && (v <= f_hi[a])) != f_neg[a];
        ok = ok && !cn && r;
      }
    }
    return ok;
  };

  // error flags as ints (a bool carried through the loops becomes a lane-mask phi: three SALU ops at
  // every merge point of the event loop)
  int overflow = 0, unordered = 0, mover = 0, aged = 0;
  // persisted deques of the group (pending partials at the start of the batch), oldest first
  const size_t gb = (size_t)W.g * L.rsmax * WAVE;
  const int n_in = pick(L.st, W.inb)[W.g].n[lane];
  const int64_t* __restrict__ i_ts = pick(L.ent_ts, W.inb);
  const int64_t* __restrict__ i_sq = pick(L.ent_seq, W.inb);
  const int64_t* __restrict__ i_ky = pick(L.ent_key, W.inb);

  if (W.c0 == 0) {
    // ---- first chunk: start from the persisted deques ----
    for (int i = 0; i < n_in; ++i) {
      const size_t o = gb + (size_t)i * WAVE + lane;
      if (!D.push_back(i_ts[o], (U)i_ky[o], (uint32_t)i_sq[o])) overflow = 1;
    }
  } else {
    // ---- later chunk: rebuild the pending partials at c0 by a REVERSE scan (exact, O(1) per
    // event): partial i (f0 passed, valid key k_i) is still pending before event c0 iff it is
    // not expired at c0-1 and no valid x_j, i < j < c0, satisfies `x_j OP k_i` -- i.e. iff the
    // max (for >, >=) / min (for <, <=) of those x_j does not. Partials older than
    // w0 = lower_bound(ts, ts[c0-1] - wmax) are expired by c0-1 (timestamps non-decreasing:
    // verified on every event the item reads; the host re-runs exactly otherwise).
    const int64_t t_last = L.b.ts[W.c0 - 1];
    const int64_t w0 = has_within ? lower_bound_ts(L.b.ts, W.c0, t_last - wmax, lane) : 0;
    bool r_has = false;  // reduction (max for >,>= / min for <,<=) of the valid x after the scan point
    U r_val = 0;
    auto better = [&](U a, U b) { return xcmp<KK>(is_max ? CM_GT : CM_LT, a, b); };
    // events [lo, hi) of one tile in detail (events < w0 masked off)
    auto detail_tile = [&](int64_t lo, int64_t hi) {
      const int64_t e = lo + lane;
      const bool live = e >= w0 && e < hi;
      int64_t ets;
      U xk;
      uint32_t vb;
      stage(e, live, ets, xk, vb);
      // inclusive suffix reduction over the tile's lanes (events)
      bool vh = (vb & 1u) != 0;
      U vv = xk;
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) {
        const U ov = shdown(vv, d);
        const bool oh = __shfl_down((int)vh, d, WAVE) != 0 && lane + d < WAVE;
        const bool take = oh && (!vh || better(ov, vv));
        vv = take ? ov : vv;
        vh = vh || oh;
      }
      U sv = shdown(vv, 1);
      bool sh = __shfl_down((int)vh, 1, WAVE) != 0 && lane + 1 < WAVE;
      if (r_has && (!sh || better(r_val, sv))) sv = r_val;
      sh = sh || r_has;
      const bool cand = live && (vb & 1u) && !(sh && xop<KK, XM>(xmask, sv, xk));
      uint64_t cm = wballot(cand);
      while (cm) {  // newest candidate first: prepend
        const int k = 63 - __builtin_clzll(cm);
        cm &= ~(1ull << k);
        const uint32_t vbk = __builtin_amdgcn_readlane(vb, k);
        const int64_t tk = readlane64(ets, k);
        const U xkk = rlane(xk, k);
        if (f0_pass(k, vbk) && !expired(tk, t_last, within))
          if (!D.push_front(tk, xkk, (uint32_t)(seq_base + lo + k))) overflow = 1;
      }
      const U tv = rlane(vv, 0);
      const bool th = __builtin_amdgcn_readlane((uint32_t)vh, 0) != 0;
      if (th && (!r_has || better(tv, r_val))) r_val = tv;
      r_has = r_has || th;
    };
    // the partial tile up to c0, then aligned tiles 64 at a time: a tile can hold a survivor only
    // if its best x is not dominated by the reduction of everything after it (x_i must satisfy
    // !(R OP x_i)); dominated tiles leave the reduction unchanged and are skipped on their summary
    int64_t hi = W.c0;
    const int64_t al = W.c0 & ~(int64_t)63;
    if (al < hi) {
      detail_tile(al, hi);
      hi = al;
    }
    const int slot = G->sum_slot;
    while (hi > w0) {
      const int64_t jhi = hi >> 6;
      const int64_t j = jhi - WAVE + lane;
      const bool tl = j >= 0 && (j + 1) * 64 > w0;
      U smx = 0;
      bool shs = false;
      if (tl) {
        const size_t o = (size_t)slot * L.n_tiles + j;
        shs = L.tsum_has[o] != 0;
        smx = (U)(is_max ? L.tsum_max[o] : L.tsum_min[o]);
      }
      // reduction after each tile: the later tiles of this group, then everything scanned before
      bool vh = shs;
      U vv = smx;
#pragma unroll
      for (int d = 1; d < WAVE; d <<= 1) {
        const U ov = shdown(vv, d);
        const bool oh = __shfl_down((int)vh, d, WAVE) != 0 && lane + d < WAVE;
        const bool take = oh && (!vh || better(ov, vv));
        vv = take ? ov : vv;
        vh = vh || oh;
      }
      U rv = shdown(vv, 1);
      bool rh = __shfl_down((int)vh, 1, WAVE) != 0 && lane + 1 < WAVE;
      if (r_has && (!rh || better(r_val, rv))) rv = r_val;
      rh = rh || r_has;
      const bool need = tl && shs && !(rh && xop<KK, XM>(xmask, rv, smx));
      uint64_t nm = wballot(need);
      while (nm) {  // newest tile first
        const int b = 63 - __builtin_clzll(nm);
        nm &= ~(1ull << b);
        const int64_t jt = jhi - WAVE + b;
        detail_tile(jt * 64, jt * 64 + 64);
      }
      // skipped tiles are dominated, so the reduction only moved on the detailed ones
      hi = (jhi - WAVE) * 64;
    }
    if (w0 == 0) {
      // the window reaches the batch start: carried partials survive unless expired or matched
      if (L.b.prev_ts > L.b.ts[0]) unordered = 1;
      for (int i = n_in - 1; i >= 0; --i) {
        const size_t o = gb + (size_t)i * WAVE + lane;
        const int64_t t0 = i_ts[o];
        const U ky = (U)i_ky[o];
        if (!expired(t0, t_last, within) && !(r_has && xop<KK, XM>(xmask, r_val, ky)))
          if (!D.push_front(t0, ky, (uint32_t)i_sq[o])) overflow = 1;
      }
    }
  }

  // Keep the top of every non-empty deque in LDS (ln >= 1): move the newest spilled entry up.
  auto refill = [&]() {
    if (D.ln == 0 && D.sn > 0) {
      // (an opaque copy of lbot: the slot address math stays on this rare path instead of being
      // hoisted into every matching event by loop-invariant code motion)
      asm volatile("" : "+v"(D.lbot));
      int64_t t0; U k0; uint32_t q0;
      D.sget(D.si(D.sbot + D.sn - 1), t0, k0, q0);
      --D.sn;
      D.lput(D.li(D.lbot), t0, k0, q0);
      D.ln = 1;
    }
  };
  refill();

  // VGPR caches of the deque ends: top key/seq, bottom deadline (rel_deadline; INT32_MAX while the
  // deque is empty, so a push lowers it to the new entry's deadline by a min: with ordered
  // timestamps every held entry's deadline is <= a newer one's)
  U tkey = 0;
  uint32_t tseq = 0;
  int32_t bdead = INT32_MAX;
  auto refresh_top = [&]() {
    if (D.ln > 0) D.lget_ks(D.li(D.lbot + D.ln - 1), tkey, tseq);
    else if (SIM) tkey = TSENT;
  };
  auto refresh_bottom = [&]() {
    bdead = INT32_MAX;
    if (D.n() > 0) {
      U k0;
      int64_t bts;
      uint32_t q0;
      D.bottom(bts, k0, q0);
      bdead = rel_deadline(sat_add(bts, within), T0);
    }
  };
  refresh_top();
  refresh_bottom();

  // output block state: fill >= FULL_FILL forces the block check, which also catches a full output
  constexpr int FULL_FILL = 1 << 30;
  int blk = -1, fill = FULL_FILL;
  unsigned long long n_emit = 0;  // records of this wave's closed blocks
  unsigned long long n_bytes = 0;  // bytes of this wave's closed blocks' records (+ PM 4 side entries)
  // the wave's current output block as a buffer resource: a record's address is a 32-bit lane offset
  // from the block base (no 64-bit address arithmetic per record), and the range check covers it
  __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(L.match, 0, 0, 0x00020000);
  int64_t prev_tile_ts = (W.c0 == 0) ? L.b.prev_ts : L.b.ts[W.c0 - 1];

  // one record per lane with `mt` (ballot m): per-wave output blocks (one atomic per block), ranks
  // by mbcnt. e2 =
  // batch event `off`; e1 = the partial with low seq bits q1. The common case costs one
  // compare-and-branch of bookkeeping (the record index is block base + fill + rank).
  const int32_t my_q = active ? G->qid[lane] : 0;
  const int cell = G->cell;
  int ev_tot = 0;     // COUNT: the wave's matches at the current event
  int32_t cntv = 0;   // COUNT: lane k = the matches at tile event k
  int32_t basev = 0;  // WRITE: lane k = the group's first row at tile event k
  int64_t pos = 0;    // WRITE: the lane's last row at the current event
  uint32_t lv = 0;    // WRITE: the lane's rows at the current event so far (the next one's level)
  auto put_row = [&](int64_t row, uint32_t off, uint32_t q1) {
    const int64_t s = seq_base + (int64_t)off;
    int32_t* o = L.crow + row * L.cw;
    const int32_t rel = (int32_t)(s - L.seq_ref), d0 = (int32_t)((uint32_t)s - q1);
    if (L.cw == 4) {
      *reinterpret_cast<int4*>(o) = make_int4(my_q, rel, d0, 0);
    } else {
      o[0] = my_q;
      o[1] = rel;
      o[2] = d0;
      o[3] = 0;
      for (int j = 4; j < L.cw; ++j) o[j] = INT32_MIN;
    }
  };
  // record width: compile-time in the chunked forms (PM 3 = 16-B records), read at run time in FULL.
  // PM 4 (device records, nfa_types.h rec4): 4-B entries {e1 distance | lane << 26} from the block's
  // start and one side entry {first entry, e2 offset} per matching event from its end downwards
  const bool wide = FULL ? L.wide != 0 : PM == 3;
  int sfill = 0;                              // PM 4: side entries in the current block
  bool new_blk = false;                       // PM 4: a block was taken since the last side entry
  const uint32_t sb32 = (uint32_t)seq_base;   // PM 4: e2 seq low bits = sb32 + off
  int d4over = 0;                             // PM 4: a distance reached 2^26 (err[4])
  // the next output block, taken when a pop round could overrun the current one (every round pops
  // at most 4 x 64 records: one check per round instead of one per ballot). Out of blocks, the wave
  // writes on into the spare block past the last (never read: the host doubles the blocks and re-runs)
  auto roll = [&]() {
    if (blk >= 0) {
      if (lane == 0) {
        L.blk_count[blk] = fill;
        L.blk_side[blk] = PM == 4 ? sfill : -1;
      }
      n_emit += (unsigned long long)fill;
      n_bytes += PM == 4 ? (unsigned long long)fill * 4 + (unsigned long long)sfill * 8
                         : (unsigned long long)fill * (wide ? 16 : 8);
    }
    sfill = 0;
    new_blk = true;  // (an event whose matches continue in this block needs a side entry here too)
    int nb = 0;
    if (lane == 0) nb = atomicAdd(L.blk_next, 1);
    nb = __builtin_amdgcn_readfirstlane(nb);
    if (nb >= L.n_blocks) {
      mover = 1;
      blk = -1;
      nb = L.n_blocks;
    } else {
      if (lane == 0) L.blk_group[nb] = W.g;
      blk = nb;
    }
    fill = 0;
    const int rb = wide ? 16 : 8;
    const uint64_t base = (uint64_t)(reinterpret_cast<char*>(L.match) + (size_t)nb * L.blk_recs * rb);
    const uint32_t blo = __builtin_amdgcn_readfirstlane((uint32_t)base), bhi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    wrs = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)bhi << 32) | blo), 0,
                                            __builtin_amdgcn_readfirstlane(L.blk_recs * rb), 0x00020000);
  };
  auto emit_room = [&]() {
    if constexpr (PM == 0 || PM == 3)
      if (fill > L.blk_recs - 4 * WAVE) roll();
    if constexpr (PM == 4)  // room for a round's 4 x 64 entries and one side entry between the two ends
      if (fill > ((L.blk_recs * 8 - 4 * WAVE * 4 - 8 - sfill * 8) >> 2)) roll();  // (fill starts at FULL_FILL)
  };
  auto emit = [&](bool mt, uint64_t m, uint32_t off, uint32_t q1) {
    if constexpr (PM == 1) {
      ev_tot += __popcll(m);
      return;
    }
    if constexpr (PM == 2) {
      if (mt) put_row(pos - (int64_t)lv, off, q1);
      lv += mt ? 1u : 0u;
      return;
    }
    if constexpr (PM == 4) {
      if (mt && !SDH_RATCHET_NOSTORE)
        __builtin_amdgcn_raw_buffer_store_b32(((sb32 + off) - q1) | ((uint32_t)lane << 26), wrs,
                                              (fill + wave_mbcnt(m)) * 4, 0, 0);
      fill += __popcll(m);
      return;
    }
    if (mt && !SDH_RATCHET_NOSTORE) {  // (NOSTORE: a measurement build without the record stores)
      const int r = fill + wave_mbcnt(m);
      if (!wide) {
        const u32x2 v = {off | ((uint32_t)lane << 26), q1};
        __builtin_amdgcn_raw_buffer_store_b64(v, wrs, r * 8, 0, 0);
      } else {
        const u32x4 v = {off, (uint32_t)lane, q1, 0u};
        __builtin_amdgcn_raw_buffer_store_b128(v, wrs, r * 16, 0, 0);
      }
    }
    fill += __popcll(m);
  };

  // ---- forward NFA step over the events this item emits for. Fast path: straight-line per
  // event (expiry check, up to four pops from one LDS round trip, push); rare cases (expiry,
  // spill refill / eviction, a fifth pop) branch to slow paths on a wave-uniform ballot ----
  // The tile is loaded at its start, not prefetched during the previous tile: a load still in flight
  // inside the event loop made the compiler wait for the vector-memory counter to drain (the match
  // records' stores included) at every event that writes its destination registers (C2 10K SIM:
  // prefetch 176.2 ms, load at tile start 167.8; the other resident waves cover the load)
  for (int64_t t = W.c0; t < W.c1; t += WAVE) {
    Raw cur;
    load(t + lane, t + lane < W.c1, cur);
    int64_t ets;
    U xk;
    uint32_t vbits;
    convert(cur, ets, xk, vbits);
    const bool live = cur.live;
    int64_t pred = __shfl_up(ets, 1, WAVE);
    if (lane == 0) pred = prev_tile_ts;
    if (live && ets < pred) unordered = 1;
    prev_tile_ts = __shfl(ets, WAVE - 1, WAVE);
    // the lazy forms compare in the 32-bit deadline domain (rel_deadline)
    int32_t ets32 = 0;
    if constexpr (!FULL)
      ets32 = ets >= T0 + (INT32_MAX - 1) ? INT32_MAX - 1 : ets <= T0 + INT32_MIN ? INT32_MIN : (int32_t)(ets - T0);
    const int cnt = (int)((W.c1 - t) < WAVE ? (W.c1 - t) : WAVE);
    // sequence numbers are kept as their low 32 bits: a live partial must stay < 2^31 events old
    // (checked once per tile against the tile's last event; the bottom only gets younger)
    // (PM 4: every distance a rec4 entry holds is below the bottom's, checked likewise against 2^26)
    if (D.n() > 0) {
      const uint32_t dist = (uint32_t)(seq_base + t + cnt - 1) - D.bottom_seq();
      if (dist >= 0x80000000u) aged = 1;
      if (PM == 4 && dist >= (1u << 26)) d4over = 1;
    }
    if constexpr (PM == 1) cntv = 0;
    if constexpr (PM == 2) basev = lane < cnt ? L.pbase[(int64_t)(t + lane) * L.n_cells + cell] : 0;

    SDH_UNROLL(SDH_RATCHET_UNROLL)
    for (int k = 0; k < cnt; ++k) {
      const int64_t tt = FULL ? readlane64(ets, k) : 0;
      const int32_t tt32 = FULL ? 0 : (int32_t)__builtin_amdgcn_readlane((uint32_t)ets32, k);
      const int64_t s = seq_base + t + k;
      const uint32_t slo = (uint32_t)s;
      const uint32_t vb = SIM ? 1u : __builtin_amdgcn_readlane(vbits, k);
      const U x = rlane(xk, k);
      const bool x_ok = SIM || (vb & 1u);

      // ---- 1. lazy `within` expiry (oldest first) ----
      if (!FULL || has_within) {
        if constexpr (!FULL) {
          // timestamps non-decreasing: expired(bts, tt) <=> tt > bts + within. Lanes without
          // `within` hold within = INT64_MAX, so their deadline saturates and never passes: the
          // check needs no group-level flag (one compare and branch per event)
          if (wballot(tt32 > bdead) != 0) {
            while (true) {
              const bool ex = D.n() > 0 && tt32 > bdead;
              if (wballot(ex) == 0) break;
              if (ex) {
                D.pop_front();
                refill();
                refresh_bottom();
                if (SIM && D.ln == 0) tkey = TSENT;
              }
            }
          }
        } else {
          const int n0 = D.n();
          D.compact_expired(tt, within);
          if (wballot(D.n() != n0) != 0) {
            refill();
            refresh_top();
            refresh_bottom();
          }
        }
      }

      // ---- 2. matches: the newest partials whose key satisfies `cur OP key` ----
      bool mt = SIM ? xop<KK, XM>(xmask, x, tkey) : (x_ok && D.ln > 0 && xop<KK, XM>(xmask, x, tkey));
      uint64_t m = wballot(mt);
      if constexpr (PM == 1) ev_tot = 0;
      if constexpr (PM == 2) lv = 0;
      bool round1 = true;
      while (m) {
        emit_room();
        if constexpr (PM == 4) {  // the event's side entry: its first entry's index and e2 offset
          if (round1 || new_blk) {  // (again at the head of a block the event's matches spill into)
            round1 = false;
            new_blk = false;
            if (lane == 0) {
              const u32x2 se = {(uint32_t)fill, (uint32_t)(t + k)};
              __builtin_amdgcn_raw_buffer_store_b64(se, wrs, L.blk_recs * 8 - (sfill + 1) * 8, 0, 0);
            }
            ++sfill;
          }
        }
        // the three LDS entries under the top, read unconditionally (in-bounds ring slots)
        const int topl = D.lbot + D.ln - 1;
        U k1, k2, k3;
        uint32_t q1, q2, q3;
        D.lget_ks(D.li(topl - 1), k1, q1);
        D.lget_ks(D.li(topl - 2), k2, q2);
        D.lget_ks(D.li(topl - 3), k3, q3);
        const bool c1 = mt && D.ln > 1 && xop<KK, XM>(xmask, x, k1);
        const bool c2 = c1 && D.ln > 2 && xop<KK, XM>(xmask, x, k2);
        const bool c3 = c2 && D.ln > 3 && xop<KK, XM>(xmask, x, k3);
        const uint32_t off = (uint32_t)(t + k);
        if constexpr (PM == 2) {
          if (round1) {  // the lane's count at this event, then its last row
            round1 = false;
            const int p1 = (int)mt + (int)c1 + (int)c2 + (int)c3;
            const bool more = mt && ((p1 == 4 && D.ln > 4) || (p1 == D.ln && D.sn > 0));
            const int64_t base = L.row0 + (int64_t)__builtin_amdgcn_readlane(basev, k);
            if (wballot(more) == 0) {
              const int below = wave_mbcnt(m) + wave_mbcnt(wballot(c1)) + wave_mbcnt(wballot(c2)) +
                                wave_mbcnt(wballot(c3));
              pos = base + below + p1 - 1;
            } else {
              int cl = p1;
              if (more) {  // walk on below the first four / into the spill ring
                for (int d = p1;; ++d) {
                  U kd;
                  uint32_t qd;
                  if (d < D.ln) {
                    D.lget_ks(D.li(D.lbot + D.ln - 1 - d), kd, qd);
                  } else if (d - D.ln < D.sn) {
                    int64_t td;
                    D.sget(D.si(D.sbot + D.sn - 1 - (d - D.ln)), td, kd, qd);
                  } else {
                    break;
                  }
                  if (!xop<KK, XM>(xmask, x, kd)) break;
                  ++cl;
                }
              }
              int incl = cl;  // inclusive scan over the lanes (rank order)
#pragma unroll
              for (int dd = 1; dd < WAVE; dd <<= 1) {
                const int o = __shfl_up(incl, dd, WAVE);
                incl += lane >= dd ? o : 0;
              }
              pos = base + incl - 1;
            }
          }
        }
        emit(mt, m, off, tseq);
        const uint64_t m1 = wballot(c1);
        if (m1) {
          emit(c1, m1, off, q1);
          const uint64_t m2 = wballot(c2);
          if (m2) {
            emit(c2, m2, off, q2);
            const uint64_t m3 = wballot(c3);
            if (m3) emit(c3, m3, off, q3);
          }
        }
        const int p = (int)mt + (int)c1 + (int)c2 + (int)c3;
        D.ln -= p;
        // new top: prefetched unless four popped (then read it) or the LDS part ran dry. The pop
        // masks nest (c3 -> c2 -> c1 -> mt), so three selects place the entry under the last pop
        tkey = mt ? k1 : tkey;
        tkey = c1 ? k2 : tkey;
        tkey = c2 ? k3 : tkey;
        tseq = mt ? q1 : tseq;
        tseq = c1 ? q2 : tseq;
        tseq = c2 ? q3 : tseq;
        const bool fix = (c3 && D.ln > 0) || (mt && D.ln == 0);
        // (a plain divergent `if`: its exec-mask skip branch is the wave-uniform test; an outer
        // ballot would re-materialise the mask through a VGPR)
        if (fix) {
          refill();
          refresh_top();
        }
        bdead = (p > 0 && D.n() == 0) ? INT32_MAX : bdead;
        // more matches are possible only where four were popped or the top was refilled
        mt = SIM ? (fix && xop<KK, XM>(xmask, x, tkey)) : (fix && x_ok && D.ln > 0 && xop<KK, XM>(xmask, x, tkey));
        m = wballot(mt);
      }
      if constexpr (PM == 1) cntv = lane == k ? ev_tot : cntv;

      // ---- 3. start state: every event passing f0 opens a partial (pending from j+1) ----
      bool f;
      if constexpr (SIM) {
        const float xf = __uint_as_float((uint32_t)x);
        f = xf >= flo && xf <= fhi;
      } else {
        f = f0_pass(k, vb);
      }
      if (f && D.ln == ML) {
        // LDS ring full: move its oldest entry to the spill ring (rare)
        if (D.sn == SC) {
          overflow = 1;
        } else {
          int64_t t0; U k0; uint32_t q0;
          D.lget(D.li(D.lbot), t0, k0, q0);
          D.sput(D.si(D.sbot + D.sn), t0, k0, q0);
          ++D.sn;
          D.lbot = (D.lbot + 1) & D.lmask;
          --D.ln;
        }
      }
      const bool push = f && D.ln < ML;
      if constexpr (SIM) D.lput_ks(push ? D.li(D.lbot + D.ln) : ML * WAVE + lane, x, slo);  // (dummy row)
      else if (push) D.lput_ks(D.li(D.lbot + D.ln), x, slo);  // ts0 = ts of this batch event
      if constexpr (!FULL) {  // a push into an empty deque sets its deadline (see bdead)
        const int32_t dl = __builtin_elementwise_add_sat(tt32, w32);
        bdead = push ? min(bdead, dl) : bdead;
      }
      D.ln += push ? 1 : 0;
      tkey = push ? x : tkey;
      tseq = push ? slo : tseq;
    }
    if constexpr (PM == 1)
      if (lane < cnt) L.pcnt[(int64_t)(t + lane) * L.n_cells + cell] = cntv;
  }

  // ---- outputs ----
  if (blk >= 0 && (PM == 0 || PM == 3 || PM == 4)) {
    if (lane == 0) {
      L.blk_count[blk] = fill;
      L.blk_side[blk] = PM == 4 ? sfill : -1;
    }
    n_emit += (unsigned long long)fill;
    n_bytes += PM == 4 ? (unsigned long long)fill * 4 + (unsigned long long)sfill * 8
                       : (unsigned long long)fill * (wide ? 16 : 8);
  }
  const uint64_t any_over = wballot(overflow != 0), any_unord = wballot(unordered != 0), any_aged = wballot(aged != 0);
  const uint64_t d4 = wballot(d4over != 0);
  if (lane == 0) {
    if (L.dev_records && n_emit) atomicAdd(L.rec_total, n_emit);
    if (L.dev_records && n_bytes) atomicAdd(L.rec_total + 2, n_bytes);
    if (any_over) atomicOr(&L.err[0], 1);
    if (any_unord) atomicOr(&L.err[1], 1);
    if (mover) atomicOr(&L.err[2], 1);
    if (any_aged) atomicOr(&L.err[3], 1);
    if (d4) atomicOr(&L.err[4], 1);
  }
  if (W.chunk == W.n_chunks - 1) {  // the last chunk owns the group's final deques
    const int ob = 1 - W.inb;
    const int64_t slast = seq_base + W.c1 - 1;
    const uint32_t llo = (uint32_t)slast;
    int64_t* __restrict__ o_ts = pick(L.ent_ts, ob);
    int64_t* __restrict__ o_sq = pick(L.ent_seq, ob);
    int64_t* __restrict__ o_ky = pick(L.ent_key, ob);
    const int n = D.n();
    for (int i = 0; i < n; ++i) {
      int64_t t0;
      U ky;
      uint32_t sq;
      D.at(i, t0, ky, sq);
      const size_t o = gb + (size_t)i * WAVE + lane;
      o_ts[o] = t0;
      o_ky[o] = (int64_t)(uint64_t)ky;
      o_sq[o] = slast - (int64_t)(uint32_t)(llo - sq);
    }
    pick(L.st, ob)[W.g].n[lane] = n;
  }
  (void)W64;
}

// per aligned 64-event tile: max and min x-atom key over the valid events (one wave per tile)
template <int KK>
__global__ __launch_bounds__(256) void ratchet_tile_summary(StreamBatch b, int attr, int conv, int64_t n_tiles,
                                                            uint64_t* tmax, uint64_t* tmin, uint8_t* thas) {
  using U = typename KT<KK>::U;
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile >= n_tiles) return;
  const int64_t e = tile * 64 + lane;
  bool ok = false;
  U k = 0;
  if (e < b.n) {
    const uint8_t* nl = pick(b.nul, attr);
    k = (U)stage_key<KK>(load_raw(pick(b.col, attr), pick(b.width, attr), e), conv, nl && nl[e], ok);
  }
  U mx = k, mn = k;
  bool h = ok;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    U omx, omn;
    if constexpr (sizeof(U) == 8) {
      omx = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mx >> 32), d, WAVE) << 32) |
            (uint32_t)__shfl_xor((int)(uint32_t)mx, d, WAVE);
      omn = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mn >> 32), d, WAVE) << 32) |
            (uint32_t)__shfl_xor((int)(uint32_t)mn, d, WAVE);
    } else {
      omx = (U)__shfl_xor((int)mx, d, WAVE);
      omn = (U)__shfl_xor((int)mn, d, WAVE);
    }
    const bool oh = __shfl_xor((int)h, d, WAVE) != 0;
    if (oh && (!h || xcmp<KK>(CM_GT, omx, mx))) mx = omx;
    if (oh && (!h || xcmp<KK>(CM_LT, omn, mn))) mn = omn;
    h = h || oh;
  }
  if (lane == 0) {
    tmax[tile] = (uint64_t)mx;
    tmin[tile] = (uint64_t)mn;
    thas[tile] = h ? 1 : 0;
  }
}

}  // namespace sdh

extern "C" hipError_t sdh_launch_ratchet_summary(int key_kind, const sdh::StreamBatch* B, int attr, int conv,
                                                 int64_t n_tiles, uint64_t* tmax, uint64_t* tmin, uint8_t* thas,
                                                 hipStream_t s) {
  if (n_tiles <= 0) return hipSuccess;
  const dim3 grid((unsigned)((n_tiles + 3) / 4)), block(256);
  switch (key_kind) {
    case sdh::KK_F32: hipLaunchKernelGGL(sdh::ratchet_tile_summary<sdh::KK_F32>, grid, block, 0, s, *B, attr, conv, n_tiles, tmax, tmin, thas); break;
    case sdh::KK_I32: hipLaunchKernelGGL(sdh::ratchet_tile_summary<sdh::KK_I32>, grid, block, 0, s, *B, attr, conv, n_tiles, tmax, tmin, thas); break;
    case sdh::KK_F64: hipLaunchKernelGGL(sdh::ratchet_tile_summary<sdh::KK_F64>, grid, block, 0, s, *B, attr, conv, n_tiles, tmax, tmin, thas); break;
    default: hipLaunchKernelGGL(sdh::ratchet_tile_summary<sdh::KK_I64>, grid, block, 0, s, *B, attr, conv, n_tiles, tmax, tmin, thas); break;
  }
  return hipGetLastError();
}

template <int KK, int XM, bool FULL, int NF, bool SIM = false>
static void launch_one(const sdh::RatchetLaunch* L, int ML, int SC, hipStream_t s) {
  const bool w64 = (KK == sdh::KK_F64 || KK == sdh::KK_I64);
  const size_t lds = (size_t)(ML + (SIM ? 1 : 0)) * 64 * (w64 ? 16 : 8);  // (SIM: + the dummy row)
  auto go = [&](auto pm, auto mlc) {
    hipLaunchKernelGGL((sdh::nfa_ratchet_kernel<KK, XM, FULL, NF, SIM, decltype(pm)::value, decltype(mlc)::value>),
                       dim3(L->n_items), dim3(64), lds, s, *L, ML, SC);
  };
  auto pick_pm = [&](auto mlc) {
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I0 = std::integral_constant<int, 0>;
    if constexpr (!FULL) {
      if (L->pcnt) return go(I1{}, mlc);
      if (L->crow) return go(I2{}, mlc);
      if (L->wide) return go(I3{}, mlc);
      if constexpr (SIM)
        if (L->rec4) return go(std::integral_constant<int, 4>{}, mlc);
    }
    go(I0{}, mlc);
  };
  // the SIM form at the default ring depth takes it as a compile-time constant (MLC)
  if constexpr (SIM) {
    if (ML == 8) return pick_pm(std::integral_constant<int, 8>{});
  }
  pick_pm(std::integral_constant<int, 0>{});
}

template <int KK, int XM, bool FULL, int NF, bool SIM = false>
static int occupancy_one(int ML) {
  const bool w64 = (KK == sdh::KK_F64 || KK == sdh::KK_I64);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, sdh::nfa_ratchet_kernel<KK, XM, FULL, NF, SIM>, 64,
                                                   (size_t)(ML + (SIM ? 1 : 0)) * 64 * (w64 ? 16 : 8)) != hipSuccess)
    return 0;
  return nb;
}

template <int KK>
static int occupancy_kk(bool full, int nf, int ML, bool sim) {
  // the four orientations share one register allocation; XM = 0 stands for all
  if (full) return occupancy_one<KK, -1, true, sdh::RMAXF0>(ML);
  if constexpr (KK == sdh::KK_F32)
    if (sim && nf <= 1) return occupancy_one<KK, 0, false, 1, true>(ML);
  return nf <= 1 ? occupancy_one<KK, 0, false, 1>(ML) : occupancy_one<KK, 0, false, sdh::RMAXF0>(ML);
}

// nf: max f0 atoms over the launched groups (one-atom start filters get a leaner register set)
template <int KK>
static hipError_t launch_kk(int xm, bool full, int nf, bool sim, const sdh::RatchetLaunch* L, int ML, int SC,
                            hipStream_t s) {
  if (full) {
    launch_one<KK, -1, true, sdh::RMAXF0>(L, ML, SC, s);
  } else if (KK == sdh::KK_F32 && sim && nf <= 1) {
    if constexpr (KK == sdh::KK_F32) {
      switch (xm) {
        case 0: launch_one<KK, 0, false, 1, true>(L, ML, SC, s); break;
        case 1: launch_one<KK, 1, false, 1, true>(L, ML, SC, s); break;
        case 2: launch_one<KK, 2, false, 1, true>(L, ML, SC, s); break;
        default: launch_one<KK, 3, false, 1, true>(L, ML, SC, s); break;
      }
    }
  } else if (nf <= 1) {
    switch (xm) {
      case 0: launch_one<KK, 0, false, 1>(L, ML, SC, s); break;
      case 1: launch_one<KK, 1, false, 1>(L, ML, SC, s); break;
      case 2: launch_one<KK, 2, false, 1>(L, ML, SC, s); break;
      default: launch_one<KK, 3, false, 1>(L, ML, SC, s); break;
    }
  } else {
    switch (xm) {
      case 0: launch_one<KK, 0, false, sdh::RMAXF0>(L, ML, SC, s); break;
      case 1: launch_one<KK, 1, false, sdh::RMAXF0>(L, ML, SC, s); break;
      case 2: launch_one<KK, 2, false, sdh::RMAXF0>(L, ML, SC, s); break;
      default: launch_one<KK, 3, false, sdh::RMAXF0>(L, ML, SC, s); break;
    }
  }
  return hipGetLastError();
}

// resident waves per CU of the K_ratchet instantiation (chunk planning fills the chip in one round)
extern "C" int sdh_ratchet_occupancy(int key_kind, int full, int nf, int ML, int sim) {
  switch (key_kind) {
    case sdh::KK_F32: return occupancy_kk<sdh::KK_F32>(full, nf, ML, sim != 0);
    case sdh::KK_I32: return occupancy_kk<sdh::KK_I32>(full, nf, ML, false);
    case sdh::KK_F64: return occupancy_kk<sdh::KK_F64>(full, nf, ML, false);
    default: return occupancy_kk<sdh::KK_I64>(full, nf, ML, false);
  }
}

// xmask: normalized `cur OP key` CmpMask of the launched groups (all equal); nf: max f0 atoms;
// ML, SC powers of two
extern "C" hipError_t sdh_launch_ratchet(int key_kind, int xmask, int full, int nf, int sim, int ML, int SC,
                                         const sdh::RatchetLaunch* L, hipStream_t s) {
  if (L->n_items <= 0) return hipSuccess;
  if (ML < 4 || (ML & (ML - 1)) || SC < 1 || (SC & (SC - 1)) || nf > sdh::RMAXF0) return hipErrorInvalidValue;
  const int xm = xmask == sdh::CM_GT ? 0 : xmask == (sdh::CM_GT | sdh::CM_EQ) ? 1 : xmask == sdh::CM_LT ? 2 : 3;
  switch (key_kind) {
    case sdh::KK_F32: return launch_kk<sdh::KK_F32>(xm, full, nf, sim != 0, L, ML, SC, s);
    case sdh::KK_I32: return launch_kk<sdh::KK_I32>(xm, full, nf, false, L, ML, SC, s);
    case sdh::KK_F64: return launch_kk<sdh::KK_F64>(xm, full, nf, false, L, ML, SC, s);
    case sdh::KK_I64: return launch_kk<sdh::KK_I64>(xm, full, nf, false, L, ML, SC, s);
    default: return hipErrorInvalidValue;
  }
}
