// String.valueOf of a float / double partition key (ValuePartitionExecutor.java:34-40): Java 8's
// Float.toString / Double.toString (sun.misc.FloatingDecimal, a JDK dependency outside the reference
// tree), restated from its published algorithm for the fan-out order of partitions keyed by float or
// double values (chm_order.h hashes "streamId" + this text). Host code.
//
// dtoa: an integer value that fits a long prints its digits (trailing zeros dropped, digits past the
// float's precision rounded away); anything else runs Steele & White digit generation from the
// estimated decimal exponent with the JDK's stopping test -- low: B < M, high: B + M > 10S (>= in the
// arbitrary-precision path) -- in 32-bit, 64-bit or arbitrary-precision arithmetic, whichever the
// operands fit, the fixed-width paths wrapping like Java ints / longs; E-form values generate at
// least two digits; the last digit is rounded by the stopping condition (the digit count is kept).
// tests/java_fmt.py restates it again for the tests; the oracle has its own.
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace sdh {
namespace jfmt {

// unsigned arbitrary-precision integer, 32-bit limbs, least significant first
struct Big {
  std::vector<uint32_t> w;
  static Big of(uint64_t v) {
    Big b;
    while (v) {
      b.w.push_back((uint32_t)v);
      v >>= 32;
    }
    return b;
  }
  void trim() {
    while (!w.empty() && w.back() == 0) w.pop_back();
  }
  void mul_small(uint32_t m) {
    uint64_t c = 0;
    for (auto& x : w) {
      c += (uint64_t)x * m;
      x = (uint32_t)c;
      c >>= 32;
    }
    if (c) w.push_back((uint32_t)c);
  }
  void mul_pow5(int k) {
    for (; k >= 13; k -= 13) mul_small(1220703125u);  // 5^13
    uint32_t m = 1;
    for (; k > 0; --k) m *= 5;
    mul_small(m);
  }
  void shl(int k) {
    if (w.empty() || k <= 0) return;
    const int limbs = k / 32, bits = k % 32;
    std::vector<uint32_t> r((size_t)limbs, 0);
    uint32_t carry = 0;
    for (uint32_t x : w) {
      r.push_back(bits ? (x << bits) | carry : x);
      carry = bits ? x >> (32 - bits) : 0;
    }
    if (carry) r.push_back(carry);
    w.swap(r);
  }
  static int cmp(const Big& a, const Big& b) {
    if (a.w.size() != b.w.size()) return a.w.size() < b.w.size() ? -1 : 1;
    for (size_t i = a.w.size(); i-- > 0;)
      if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
    return 0;
  }
  static Big add(const Big& a, const Big& b) {
    Big r;
    uint64_t c = 0;
    for (size_t i = 0; i < std::max(a.w.size(), b.w.size()); ++i) {
      c += (i < a.w.size() ? a.w[i] : 0u) + (uint64_t)(i < b.w.size() ? b.w[i] : 0u);
      r.w.push_back((uint32_t)c);
      c >>= 32;
    }
    if (c) r.w.push_back((uint32_t)c);
    return r;
  }
  void sub(const Big& b) {  // *this >= b
    int64_t c = 0;
    for (size_t i = 0; i < w.size(); ++i) {
      c += (int64_t)w[i] - (i < b.w.size() ? b.w[i] : 0u);
      w[i] = (uint32_t)c;
      c = c < 0 ? -1 : 0;
    }
    trim();
  }
};

inline Big pow52(int p5, int p2, uint64_t m = 1) {
  Big b = Big::of(m);
  b.mul_pow5(p5);
  b.shl(p2);
  return b;
}

constexpr int kN5Bits[27] = {0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};

// floor(log10(2^p)) for 1 < p < 64 (the digits of 2^p past the first)
inline int insignificant_digits_pow2(int p) {
  if (p <= 1 || p >= 64) return 0;
  return (int)std::floor((double)p * 0.30102999566398119521);
}

struct Digits {
  std::vector<int> d;
  int dec_exp = 0;  // value = 0.d1 d2 ... x 10^dec_exp
};

inline void roundup(Digits& r) {
  size_t i = r.d.size() - 1;
  int q = r.d[i];
  if (q == 9) {
    while (q == 9 && i > 0) {
      r.d[i] = 0;
      q = r.d[--i];
    }
    if (q == 9) {  // carry out: a leading 1, the rest zeros, one more decimal place
      r.dec_exp += 1;
      r.d[0] = 1;
      return;
    }
  }
  r.d[i] = q + 1;
}

inline int estimate_dec_exp(uint64_t fract, int bin_exp) {
  const uint64_t b = 0x3FF0000000000000ull | (fract & 0xFFFFFFFFFFFFFull);
  double d2;
  std::memcpy(&d2, &b, 8);
  const double d = (d2 - 1.5) * 0.289529654 + 0.176091259 + (double)bin_exp * 0.301029995663981;
  return (int)std::floor(d);
}

struct Stop {
  bool low = false, high = false;
  int64_t low_diff = 0;  // sign of 2B - 10S at the stop (ties: 0)
};

// the fixed-width digit loop (T = int32_t or int64_t: Java int / long arithmetic, wrapping)
template <class T, class U>
Stop fixed_digits(uint64_t fract, int B5, int B2, int S5, int S2, int M5, int M2, int& dec_exp, Digits& r) {
  auto p5 = [](int k) {
    U v = 1;
    for (int i = 0; i < k; ++i) v *= 5;
    return v;
  };
  T b = (T)((U)(T)((U)fract * p5(B5)) << B2);
  const T s = (T)(p5(S5) << S2);
  T m = (T)(p5(M5) << M2);
  const T tens = (T)((U)s * 10);
  T q = b / s;
  b = (T)((U)(b % s) * 10);
  m = (T)((U)m * 10);
  Stop st;
  st.low = b < m;
  st.high = (T)((U)b + (U)m) > tens;
  if (q == 0 && !st.high) --dec_exp;
  else r.d.push_back((int)q);
  if (dec_exp < -3 || dec_exp >= 8) st.high = st.low = false;  // E-form: at least two digits
  while (!st.low && !st.high) {
    q = b / s;
    b = (T)((U)(b % s) * 10);
    m = (T)((U)m * 10);
    if (m > 0) {
      st.low = b < m;
      st.high = (T)((U)b + (U)m) > tens;
    } else {  // m overflowed: the JDK stops here
      st.low = st.high = true;
    }
    r.d.push_back((int)q);
  }
  st.low_diff = (int64_t)(T)((U)(T)((U)b << 1) - (U)tens);
  return st;
}

inline Stop big_digits(uint64_t fract, int B5, int B2, int S5, int S2, int M5, int M2, int& dec_exp, Digits& r) {
  const Big S = pow52(S5, S2), tenS = pow52(S5 + 1, S2 + 1);
  Big B = pow52(B5, B2, fract), M = pow52(M5 + 1, M2 + 1);
  auto quo_rem = [&]() {  // q = B / S (< 10), B = (B % S) * 10
    int q = 0;
    while (Big::cmp(B, S) >= 0) {
      B.sub(S);
      ++q;
    }
    B.mul_small(10);
    B.trim();
    return q;
  };
  Stop st;
  int q = quo_rem();
  st.low = Big::cmp(B, M) < 0;
  st.high = Big::cmp(Big::add(B, M), tenS) >= 0;
  if (q == 0 && !st.high) --dec_exp;
  else r.d.push_back(q);
  if (dec_exp < -3 || dec_exp >= 8) st.high = st.low = false;
  while (!st.low && !st.high) {
    q = quo_rem();
    M.mul_small(10);
    st.low = Big::cmp(B, M) < 0;
    st.high = Big::cmp(Big::add(B, M), tenS) >= 0;
    r.d.push_back(q);
  }
  if (st.high && st.low) {
    Big b2 = B;
    b2.shl(1);
    st.low_diff = Big::cmp(b2, tenS);
  }
  return st;
}

// FloatingDecimal.BinaryToASCIIBuffer.dtoa (isCompatibleFormat = true): the value is
// fract * 2^(bin_exp - 52), fract with its high bit at 52 and n_sig significant bits
inline Digits dtoa(int bin_exp, uint64_t fract, int n_sig) {
  Digits r;
  const int tail = __builtin_ctzll(fract);
  const int n_fract_bits = 53 - tail;
  const int n_tiny = std::max(0, n_fract_bits - bin_exp - 1);
  if (bin_exp <= 62 && bin_exp >= -21 && n_tiny == 0 && n_fract_bits < 64) {
    // easy case: an integer that fits a long (developLongDigits)
    const int insig = bin_exp > n_sig ? insignificant_digits_pow2(bin_exp - n_sig - 1) : 0;
    uint64_t lv = bin_exp >= 52 ? fract << (bin_exp - 52) : fract >> (52 - bin_exp);
    int de = 0;
    if (insig) {
      uint64_t p10 = 1;
      for (int i = 0; i < insig; ++i) p10 *= 10;
      const uint64_t residue = lv % p10;
      lv /= p10;
      de += insig;
      if (residue >= (p10 >> 1)) ++lv;
    }
    const std::string s = std::to_string((unsigned long long)lv);
    size_t keep = s.size();
    while (keep > 1 && s[keep - 1] == '0') --keep;
    de += (int)(s.size() - keep);
    for (size_t i = 0; i < keep; ++i) r.d.push_back(s[i] - '0');
    r.dec_exp = de + (int)keep;
    return r;
  }
  int dec_exp = estimate_dec_exp(fract, bin_exp);
  const int B5 = std::max(0, -dec_exp), S5 = std::max(0, dec_exp), M5 = B5;
  int B2 = B5 + n_tiny + bin_exp, S2 = S5 + n_tiny, M2 = B2 - n_sig;
  fract >>= tail;
  B2 -= n_fract_bits - 1;
  const int c2 = std::min(B2, S2);
  B2 -= c2;
  S2 -= c2;
  M2 -= c2;
  if (n_fract_bits == 1) M2 -= 1;  // a power of two: the lower neighbour is half as far
  if (M2 < 0) {
    B2 -= M2;
    S2 -= M2;
    M2 = 0;
  }
  const int b_bits = n_fract_bits + B2 + (B5 < 27 ? kN5Bits[B5] : B5 * 3);
  const int ten_s_bits = S2 + 1 + (S5 + 1 < 27 ? kN5Bits[S5 + 1] : (S5 + 1) * 3);
  Stop st;
  if (b_bits < 32 && ten_s_bits < 32)
    st = fixed_digits<int32_t, uint32_t>(fract, B5, B2, S5, S2, M5, M2, dec_exp, r);
  else if (b_bits < 64 && ten_s_bits < 64)
    st = fixed_digits<int64_t, uint64_t>(fract, B5, B2, S5, S2, M5, M2, dec_exp, r);
  else
    st = big_digits(fract, B5, B2, S5, S2, M5, M2, dec_exp, r);
  r.dec_exp = dec_exp + 1;
  if (st.high) {
    if (!st.low) roundup(r);
    else if (st.low_diff > 0 || (st.low_diff == 0 && (r.d.back() & 1))) roundup(r);
  }
  return r;
}

// FloatingDecimal.BinaryToASCIIBuffer.getChars
inline std::string format(bool neg, const Digits& r) {
  std::string d;
  for (int x : r.d) d.push_back((char)('0' + x));
  std::string out = neg ? "-" : "";
  const int n = (int)d.size(), e = r.dec_exp;
  if (e > 0 && e < 8) {
    const int c = std::min(n, e);
    out += d.substr(0, (size_t)c);
    if (c < e) out += std::string((size_t)(e - c), '0') + ".0";
    else out += "." + (c < n ? d.substr((size_t)c) : std::string("0"));
  } else if (e <= 0 && e > -3) {
    out += "0." + std::string((size_t)-e, '0') + d;
  } else {
    out += d.substr(0, 1) + "." + (n > 1 ? d.substr(1) : std::string("0")) + "E";
    out += e <= 0 ? "-" + std::to_string(-e + 1) : std::to_string(e - 1);
  }
  return out;
}

// Double.toString of the double with raw bits `bits`
inline std::string double_to_string(uint64_t bits) {
  const bool neg = (bits >> 63) != 0;
  uint64_t fract = bits & ((1ull << 52) - 1);
  int be = (int)((bits >> 52) & 0x7FF);
  if (be == 0x7FF) return fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
  int n_sig;
  if (be == 0) {
    if (!fract) return neg ? "-0.0" : "0.0";
    const int lz = __builtin_clzll(fract), shift = lz - 11;
    fract <<= shift;
    be = 1 - shift;
    n_sig = 64 - lz;
  } else {
    fract |= 1ull << 52;
    n_sig = 53;
  }
  return format(neg, dtoa(be - 1023, fract, n_sig));
}

// Float.toString of the float with raw bits `bits`
inline std::string float_to_string(uint32_t bits) {
  const bool neg = (bits >> 31) != 0;
  uint32_t fract = bits & ((1u << 23) - 1);
  int be = (int)((bits >> 23) & 0xFF);
  if (be == 0xFF) return fract ? "NaN" : (neg ? "-Infinity" : "Infinity");
  int n_sig;
  if (be == 0) {
    if (!fract) return neg ? "-0.0" : "0.0";
    const int lz = __builtin_clz(fract), shift = lz - 8;
    fract <<= shift;
    be = 1 - shift;
    n_sig = 32 - lz;
  } else {
    fract |= 1u << 23;
    n_sig = 24;
  }
  return format(neg, dtoa(be - 127, (uint64_t)fract << 29, n_sig));
}

}  // namespace jfmt
}  // namespace sdh
