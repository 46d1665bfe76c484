// ratchet_common.h -- device helpers shared by the K_ratchet (nfa_ratchet.hip) and gated K_gate
// (nfa_gate.hip) kernels: ballots and lane reads, the x-atom key domains and compares, start-filter
// intervals, the 32-bit deadline domain.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "nfa_types.h"

namespace sdh {

namespace {

// ballot of a bool (HIP's __ballot takes an int: the bool -> int -> bool round trip costs a v_cndmask
// and a v_cmp per ballot in the event loop)
__device__ __forceinline__ uint64_t wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

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
    const uint64_t m = wballot(ts[p] < target);
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

// ---- key traits: 32-bit keys (binary32 / int32) or 64-bit keys (binary64 / int64) ----
template <int KK>
struct KT {
  static constexpr bool W64 = (KK == KK_F64 || KK == KK_I64);
  using U = typename std::conditional<W64, uint64_t, uint32_t>::type;
};

template <class U>
__device__ __forceinline__ U rlane(U v, int k) {
  if constexpr (sizeof(U) == 8) return (U)readlane64((int64_t)v, k);
  else return (U)__builtin_amdgcn_readlane((uint32_t)v, k);
}

template <class U>
__device__ __forceinline__ U shdown(U v, int d) {
  if constexpr (sizeof(U) == 8) {
    const uint32_t lo = (uint32_t)__shfl_down((int)(uint32_t)v, d, WAVE);
    const uint32_t hi = (uint32_t)__shfl_down((int)(uint32_t)(v >> 32), d, WAVE);
    return ((uint64_t)hi << 32) | lo;
  } else {
    return (U)__shfl_down((int)v, d, WAVE);
  }
}

// x-atom compare `cur OP key` with the normalized operator known at compile time (XM >= 0) or at
// run time (XM < 0: FULL-expiry kernels). Keys are valid (no NaN).
template <int KK, int XM>
__device__ __forceinline__ bool xop(int xmask, uint64_t cur, uint64_t key) {
  if constexpr (XM < 0) {
    return xcmp<KK>(xmask, cur, key);
  } else {
    constexpr int m = XM == 0 ? CM_GT : XM == 1 ? (CM_GT | CM_EQ) : XM == 2 ? CM_LT : (CM_LT | CM_EQ);
    if constexpr (KK == KK_F32) {
      const float a = __uint_as_float((uint32_t)cur), b = __uint_as_float((uint32_t)key);
      return m == CM_GT ? a > b : m == (CM_GT | CM_EQ) ? a >= b : m == CM_LT ? a < b : a <= b;
    } else if constexpr (KK == KK_I32) {
      const int32_t a = (int32_t)(uint32_t)cur, b = (int32_t)(uint32_t)key;
      return m == CM_GT ? a > b : m == (CM_GT | CM_EQ) ? a >= b : m == CM_LT ? a < b : a <= b;
    } else if constexpr (KK == KK_F64) {
      const double a = __longlong_as_double((int64_t)cur), b = __longlong_as_double((int64_t)key);
      return m == CM_GT ? a > b : m == (CM_GT | CM_EQ) ? a >= b : m == CM_LT ? a < b : a <= b;
    } else {
      const int64_t a = (int64_t)cur, b = (int64_t)key;
      return m == CM_GT ? a > b : m == (CM_GT | CM_EQ) ? a >= b : m == CM_LT ? a < b : a <= b;
    }
  }
}

// order-preserving int64 image of a binary64 key: -0.0 and +0.0 map together, NaN to INT64_MIN
__device__ __forceinline__ int64_t sortable_f64(int64_t b) {
  const double d = __longlong_as_double(b);
  if (d != d) return INT64_MIN;
  if (d == 0.0) return 0;
  return b >= 0 ? b : (b ^ INT64_MAX);
}

// f0 atom `cur OP c` (mask over the current-event operand; CM_NOT allowed with EQ only) as an
// interval [lo, hi] of sortable keys, optionally complemented: pass = (lo <= v <= hi) ^ neg.
// NaN operands (INT64_MIN) fall outside every non-complemented interval.
__device__ __forceinline__ void f0_interval(int mask, bool f64, int64_t c, int64_t& lo, int64_t& hi, bool& neg) {
  neg = (mask & CM_NOT) != 0;
  const int m = mask & (CM_LT | CM_GT | CM_EQ);
  const int64_t vmin = f64 ? INT64_MIN + 1 : INT64_MIN;
  if (f64) {
    const double d = __longlong_as_double(c);
    if (d != d) {  // compares with NaN are false (!= true)
      lo = 1;
      hi = 0;
      return;
    }
    c = sortable_f64(c);
  }
  lo = vmin;
  hi = INT64_MAX;
  const bool empty_lo = (m & CM_GT) && !(m & CM_EQ) && c == INT64_MAX;
  const bool empty_hi = (m & CM_LT) && !(m & CM_EQ) && c == vmin;
  if (m == CM_EQ) { lo = c; hi = c; }
  else if (m == CM_GT) { lo = c + (c == INT64_MAX ? 0 : 1); }
  else if (m == (CM_GT | CM_EQ)) { lo = c; }
  else if (m == CM_LT) { hi = c - (c == vmin ? 0 : 1); }
  else if (m == (CM_LT | CM_EQ)) { hi = c; }
  if (empty_lo || empty_hi) { lo = 1; hi = 0; }
}

__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {  // b >= 0
  return a > INT64_MAX - b ? INT64_MAX : a + b;
}

// Expiry deadlines of the lazy (ordered-timestamp) forms live in a 32-bit domain relative to the
// item's first timestamp T0: the host routes batches whose ts span is 2^31 - 2 or more (or whose
// timestamps are beyond +-2^61) to the FULL form, so every event's ts - T0 of an ordered batch is in
// [0, 2^31 - 2]. A deadline (ts0 + within, saturated) maps to ts - T0 clamped to [INT32_MIN,
// INT32_MAX]: INT32_MAX (never) and INT32_MIN (already passed) keep `tt > deadline` exact. Out-of-order
// batches produce garbage here but are flagged from the 64-bit timestamps and re-run in FULL form.
__device__ __forceinline__ int32_t rel_deadline(int64_t d, int64_t T0) {  // |T0| <= 2^61
  if (d >= T0 + INT32_MAX) return INT32_MAX;
  if (d <= T0 + INT32_MIN) return INT32_MIN;
  return (int32_t)(d - T0);
}

}  // namespace sdh
