// oracle.cpp -- CPU restatement of the reference pattern/sequence engine.
//
// TEST INFRASTRUCTURE ONLY (the parity checker for libsiddhi_hip.so): only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline may load this library.
//
// Pinned by the reference's own known-answer tests, transcribed into tests/golden/*.json by
// tests/golden/extract_reference_tests.py (EveryPatternTestCase, WithinPatternTestCase,
// CountPatternTestCase, LogicalPatternTestCase, ComplexPatternTestCase, SequenceTestCase,
// PatternPartitionTestCase, SequencePartitionTestCase). The Java engine itself cannot run in this
// image (no JDK), so no outputs of the reference were generated here.
//
// Abbreviation: state/ = modules/siddhi-core/src/main/java/org/wso2/siddhi/core/query/input/stream/state/
//
// The object model is restated literally: StateEvent objects shared between pending lists,
// shallow every-clones (state/../event/state/StateEventCloner.java:46-58), StreamEvent chains for
// count slots (event/state/StateEvent.java:208-236), two-phase newAndEvery -> pending promotion.
// Garbage is reclaimed by a mark/sweep over all pending lists (the JVM's job in the reference).
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

using i64 = int64_t;

// ------------------------------------------------------------------------------------------
// IR (siddhi_amd/ir.py)
// ------------------------------------------------------------------------------------------
enum { T_INT, T_LONG, T_FLOAT, T_DOUBLE, T_BOOL, T_STRING };
enum { OP_CONST = 1, OP_ATTR, OP_IS_NULL, OP_STREAM_IS_NULL, OP_CMP, OP_AND, OP_OR, OP_NOT, OP_ARITH };
enum { CMP_EQ, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE };
enum { AR_ADD, AR_SUB, AR_MUL, AR_DIV, AR_MOD };
enum { K_STREAM, K_COUNT, K_LOGICAL, K_ABSENT };
enum { L_AND, L_OR };
enum { Q_PATTERN, Q_SEQUENCE };
enum { R_SINGLE, R_MULTI };
enum { N_STREAM, N_NEXT, N_EVERY, N_LOGICAL, N_COUNT };

struct Insn {
  int op, lt, rt, res;
  i64 a, b, imm;
};
using Code = std::vector<Insn>;

struct StateDef {
  int kind, stream, is_start, min, max, ltype, partner, next_pre, next_every, within_every,
      callback, this_last, has_selector;
  i64 waiting;  // K_ABSENT: the 'for' time (ms)
  std::vector<Code> filters;
};
struct RecvDef {
  int stream, kind;
  std::vector<int> procs;
};
struct NodeDef {
  int type, a, b, pre;
};
struct QueryDef {
  int type;
  i64 within;
  int partition;
  std::vector<StateDef> states;
  std::vector<int> start_ids;
  std::vector<RecvDef> recvs;
  std::vector<NodeDef> nodes;
};
struct PartKey {
  int stream;
  Code code;
};
struct FanOut {  // a stream the partition's queries read but no key covers
  int stream;
  int32_t id_hash;  // String.hashCode of the stream id
  int id_len;
};
struct PartDef {
  std::vector<PartKey> keys;
  std::vector<int> queries;
  std::vector<FanOut> fanout;
};
struct Program {
  std::vector<std::vector<int>> stream_types;
  std::vector<QueryDef> queries;
  std::vector<PartDef> parts;
};

struct Reader {
  const i64* w;
  size_t n, i = 0;
  i64 next() {
    if (i >= n) throw std::runtime_error("IR blob truncated");
    return w[i++];
  }
};

Code read_code(Reader& r) {
  Code c(r.next());
  for (auto& ins : c) {
    i64 w0 = r.next();
    ins.op = w0 & 0xff;
    ins.lt = (w0 >> 8) & 0xff;
    ins.rt = (w0 >> 16) & 0xff;
    ins.res = (w0 >> 24) & 0xff;
    ins.a = r.next();
    ins.b = r.next();
    ins.imm = r.next();
  }
  return c;
}

Program parse_ir(const void* blob, size_t len) {
  if (len < 16 || std::memcmp(blob, "SDHIR001", 8) != 0) throw std::runtime_error("bad IR magic");
  Reader r{reinterpret_cast<const i64*>(static_cast<const char*>(blob) + 8), (len - 8) / 8};
  Program p;
  if (r.next() != 2) throw std::runtime_error("unsupported IR version");
  p.stream_types.resize(r.next());
  for (auto& st : p.stream_types) {
    st.resize(r.next());
    for (auto& t : st) t = (int)r.next();
  }
  i64 nstr = r.next();
  for (i64 k = 0; k < nstr; ++k) {
    i64 nb = r.next();
    for (i64 j = 0; j < (nb + 7) / 8; ++j) r.next();
  }
  p.queries.resize(r.next());
  for (auto& q : p.queries) {
    q.type = (int)r.next();
    q.within = r.next();
    q.states.resize(r.next());
    q.partition = (int)r.next();
    r.next();  // selector present
    for (auto& s : q.states) {
      s.kind = (int)r.next(); s.stream = (int)r.next(); s.is_start = (int)r.next();
      s.min = (int)r.next(); s.max = (int)r.next(); s.ltype = (int)r.next();
      s.partner = (int)r.next(); s.next_pre = (int)r.next(); s.next_every = (int)r.next();
      s.within_every = (int)r.next(); s.callback = (int)r.next(); s.this_last = (int)r.next();
      s.has_selector = (int)r.next();
      s.waiting = r.next();
      s.filters.resize(r.next());
      for (auto& f : s.filters) f = read_code(r);
    }
    q.start_ids.resize(r.next());
    for (auto& x : q.start_ids) x = (int)r.next();
    q.recvs.resize(r.next());
    for (auto& rv : q.recvs) {
      rv.stream = (int)r.next(); rv.kind = (int)r.next();
      rv.procs.resize(r.next());
      for (auto& x : rv.procs) x = (int)r.next();
    }
    q.nodes.resize(r.next());
    for (auto& n : q.nodes) {
      n.type = (int)r.next(); n.a = (int)r.next(); n.b = (int)r.next(); n.pre = (int)r.next();
    }
    i64 nout = r.next();
    for (i64 k = 0; k < nout; ++k) read_code(r);
  }
  p.parts.resize(r.next());
  for (auto& pd : p.parts) {
    pd.keys.resize(r.next());
    for (auto& k : pd.keys) {
      k.stream = (int)r.next();
      k.code = read_code(r);
    }
    pd.queries.resize(r.next());
    for (auto& x : pd.queries) x = (int)r.next();
  }
  if (r.i < r.n)  // trailer: the partitions' fan-out streams
    for (auto& pd : p.parts) {
      pd.fanout.resize(r.next());
      for (auto& f : pd.fanout) {
        f.stream = (int)r.next();
        f.id_hash = (int32_t)r.next();
        f.id_len = (int)r.next();
      }
    }
  return p;
}

// ------------------------------------------------------------------------------------------
// java.util.concurrent.ConcurrentHashMap (JDK 8, the reference's runtime; not in /root/reference --
// restated from its published algorithm): the iteration order of a map filled by put() in a given
// order, single-threaded. PartitionStreamReceiver.send(ComplexEvent):277-281 walks its
// cachedStreamJunctionMap.values() in this order. Parity of multi-key orders is unpinned (the
// reference KAT, PatternPartitionTestCase query 30, has one key).
// ------------------------------------------------------------------------------------------
struct JavaCHM {
  struct Node {
    int32_t hash;  // spread(h)
    int id;
  };
  struct Bin {
    std::vector<Node> nodes;  // list order (a TreeBin: its `first` list order)
    bool tree = false;
  };
  std::vector<Bin> tab;
  int64_t size_ctl = 0, count = 0;
  static int32_t spread(int32_t h) { return (int32_t)(((uint32_t)h ^ ((uint32_t)h >> 16)) & 0x7fffffffu); }
  // transfer:2330-2470 to a table twice as large: a list bin splits at its lastRun -- the nodes
  // before it are prepended to their half (reversed), the run keeps its order; a TreeBin splits in
  // order and untreeifies at <= 6 nodes (UNTREEIFY_THRESHOLD)
  void transfer() {
    const size_t n = tab.size();
    std::vector<Bin> nt(2 * n);
    for (size_t i = 0; i < n; ++i) {
      Bin& b = tab[i];
      if (b.nodes.empty()) continue;
      std::vector<Node> lo, hi;
      if (!b.tree) {
        size_t last = 0;
        int run = b.nodes[0].hash & (int)n;
        for (size_t k = 1; k < b.nodes.size(); ++k)
          if ((b.nodes[k].hash & (int)n) != run) {
            run = b.nodes[k].hash & (int)n;
            last = k;
          }
        std::vector<Node>& tail = run == 0 ? lo : hi;
        tail.assign(b.nodes.begin() + (long)last, b.nodes.end());
        for (size_t k = 0; k < last; ++k) {
          std::vector<Node>& dst = (b.nodes[k].hash & (int)n) == 0 ? lo : hi;
          dst.insert(dst.begin(), b.nodes[k]);
        }
        nt[i].nodes = lo;
        nt[i + n].nodes = hi;
      } else {
        for (const Node& x : b.nodes) ((x.hash & (int)n) == 0 ? lo : hi).push_back(x);
        nt[i].nodes = lo;
        nt[i].tree = lo.size() > 6;
        nt[i + n].nodes = hi;
        nt[i + n].tree = hi.size() > 6;
      }
    }
    tab.swap(nt);
    size_ctl = (int64_t)(2 * n) - (int64_t)(n >> 1);
  }
  static int64_t table_size_for(int64_t c) {
    int64_t n = 1;
    while (n < c) n <<= 1;
    return n;
  }
  // tryPresize:2262-2300 (treeifyBin on a table shorter than MIN_TREEIFY_CAPACITY)
  void try_presize(int64_t size) {
    const int64_t c = table_size_for(size + (size >> 1) + 1);
    while (c > size_ctl) transfer();
  }
  // putVal:1010-1060 + addCount:2230-2260
  void put(int32_t h, int id) {
    if (tab.empty()) {
      tab.resize(16);  // DEFAULT_CAPACITY
      size_ctl = 12;
    }
    const int32_t hs = spread(h);
    const size_t i = (size_t)hs & (tab.size() - 1);
    Bin& b = tab[i];
    int64_t bin_count = 0;
    if (b.nodes.empty()) {
      b.nodes.push_back({hs, id});
    } else if (b.tree) {
      bin_count = 2;
      b.nodes.insert(b.nodes.begin(), Node{hs, id});  // putTreeVal: the new node becomes `first`
    } else {
      bin_count = (int64_t)b.nodes.size();
      b.nodes.push_back({hs, id});
      if (bin_count >= 8) {  // TREEIFY_THRESHOLD -> treeifyBin
        if (tab.size() < 64) try_presize((int64_t)tab.size() << 1);
        else tab[i].tree = true;
      }
    }
    ++count;
    if (bin_count >= 0)
      while (count >= size_ctl) transfer();
  }
  std::vector<int> order() const {
    std::vector<int> o;
    for (const Bin& b : tab)
      for (const Node& x : b.nodes) o.push_back(x.id);
    return o;
  }
};

// String.hashCode of `prefix + s` from the prefix's hash and the UTF-16 (here ASCII) units of s
// Java 8 Float.toString / Double.toString (sun.misc.FloatingDecimal; the JDK is outside the
// reference tree): String.valueOf of a float / double partition key. The oracle's own restatement
// (the engine has csrc/java_fmt.h, the tests tests/java_fmt.py; test_java_fmt.py compares the three).
// Magnitudes: base-2^32 little-endian limbs.
using Mag = std::vector<uint32_t>;
Mag mag_of(uint64_t v, int p5, int p2) {
  Mag m;
  for (; v; v >>= 32) m.push_back((uint32_t)v);
  for (int k = 0; k < p5; ++k) {
    uint64_t c = 0;
    for (auto& x : m) { c += (uint64_t)x * 5; x = (uint32_t)c; c >>= 32; }
    if (c) m.push_back((uint32_t)c);
  }
  for (int k = 0; k < p2; ++k) {
    uint32_t c = 0;
    for (auto& x : m) { uint32_t nc = x >> 31; x = (x << 1) | c; c = nc; }
    if (c) m.push_back(c);
  }
  return m;
}
int mag_cmp(Mag a, Mag b) {
  while (!a.empty() && !a.back()) a.pop_back();
  while (!b.empty() && !b.back()) b.pop_back();
  if (a.size() != b.size()) return a.size() < b.size() ? -1 : 1;
  for (size_t i = a.size(); i-- > 0;) if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
  return 0;
}
Mag mag_add(const Mag& a, const Mag& b) {
  Mag r(std::max(a.size(), b.size()) + 1, 0);
  uint64_t c = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    c += (uint64_t)(i < a.size() ? a[i] : 0) + (i < b.size() ? b[i] : 0);
    r[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}
void mag_sub(Mag& a, const Mag& b) {
  int64_t br = 0;
  for (size_t i = 0; i < a.size(); ++i) {
    int64_t d = (int64_t)a[i] - (i < b.size() ? b[i] : 0) - br;
    br = d < 0;
    a[i] = (uint32_t)(d + (br << 32));
  }
}
Mag mag_mul10(const Mag& a) {
  Mag r = mag_add(a, a), r4 = mag_add(r, r);
  return mag_add(mag_add(r4, r4), r);  // 8a + 2a
}

std::string java_fp_string(uint64_t raw, bool dbl) {
  const int MB = dbl ? 52 : 23, EB = dbl ? 11 : 8, bias = dbl ? 1023 : 127;
  const bool neg = (raw >> (MB + EB)) & 1;
  uint64_t f = raw & ((1ull << MB) - 1);
  int be = (int)((raw >> MB) & ((1u << EB) - 1));
  if (be == (1 << EB) - 1) return f ? "NaN" : neg ? "-Infinity" : "Infinity";
  int nsig;
  if (be == 0) {
    if (!f) return neg ? "-0.0" : "0.0";
    int width = 0;
    for (uint64_t t = f; t; t >>= 1) ++width;
    const int shift = MB + 1 - width;  // normalise the denormal
    f <<= shift;
    be = 1 - shift;
    nsig = width;
  } else {
    f |= 1ull << MB;
    nsig = MB + 1;
  }
  be -= bias;
  f <<= 52 - MB;
  std::vector<int> dg;
  int decexp;  // value = 0.dg x 10^decexp
  int tz = 0;
  while (!((f >> tz) & 1)) ++tz;
  const int nfb = 53 - tz, tiny = std::max(0, nfb - be - 1);
  static const int n5[27] = {0, 3, 5, 7, 10, 12, 14, 17, 19, 21, 24, 26, 28, 31, 33, 35, 38, 40, 42, 45, 47, 49, 52, 54, 56, 59, 61};
  if (be >= -21 && be <= 62 && tiny == 0) {
    // an integer in a long: its digits, the digits past the float's precision rounded away
    uint64_t v = be >= 52 ? f << (be - 52) : f >> (52 - be);
    int drop = 0;
    if (be > nsig) {
      const int p = be - nsig - 1;
      if (p > 1 && p < 64) drop = (int)std::floor(p * 0.30102999566398119521);  // digits of 2^p - 1
    }
    decexp = drop;
    if (drop) {
      uint64_t t = 1;
      for (int i = 0; i < drop; ++i) t *= 10;
      const uint64_t rem = v % t;
      v = v / t + (rem >= t / 2 ? 1 : 0);
    }
    std::string s = std::to_string((unsigned long long)v);
    while (s.size() > 1 && s.back() == '0') { s.pop_back(); ++decexp; }
    for (char c : s) dg.push_back(c - '0');
    decexp += (int)dg.size();
  } else {
    double d2;
    const uint64_t b2 = 0x3FF0000000000000ull | (f & 0xFFFFFFFFFFFFFull);
    std::memcpy(&d2, &b2, 8);
    int de = (int)std::floor((d2 - 1.5) * 0.289529654 + 0.176091259 + (double)be * 0.301029995663981);
    const int B5 = std::max(0, -de), S5 = std::max(0, de);
    int B2 = B5 + tiny + be, S2 = S5 + tiny, M2 = B2 - nsig;
    const uint64_t fr = f >> tz;
    B2 -= nfb - 1;
    const int common = std::min(B2, S2);
    B2 -= common; S2 -= common; M2 -= common;
    if (nfb == 1) --M2;
    if (M2 < 0) { B2 -= M2; S2 -= M2; M2 = 0; }
    const int bbits = nfb + B2 + (B5 < 27 ? n5[B5] : B5 * 3);
    const int tbits = S2 + 1 + (S5 + 1 < 27 ? n5[S5 + 1] : (S5 + 1) * 3);
    bool low, high;
    int ldiff;  // sign of 2B - 10S where it decides the last digit
    if (bbits < 64 && tbits < 64) {
      const int W = bbits < 32 && tbits < 32 ? 32 : 64;  // Java int / long arithmetic, wrapping
      auto wr = [W](unsigned __int128 x) -> int64_t {
        return W == 32 ? (int64_t)(int32_t)(uint32_t)x : (int64_t)(uint64_t)x;
      };
      unsigned __int128 p5b = 1, p5s = 1;
      for (int i = 0; i < B5; ++i) p5b *= 5;
      for (int i = 0; i < S5; ++i) p5s *= 5;
      int64_t b = wr((unsigned __int128)(uint64_t)wr((unsigned __int128)fr * p5b) << B2);
      const int64_t sv = wr(p5s << S2);
      int64_t m = wr(p5b << M2);  // (M5 = B5)
      const int64_t tens = wr((unsigned __int128)(uint64_t)sv * 10);
      int64_t q = b / sv;
      b = wr((unsigned __int128)(uint64_t)(b % sv) * 10);
      m = wr((unsigned __int128)(uint64_t)m * 10);
      low = b < m;
      high = wr((unsigned __int128)(uint64_t)b + (uint64_t)m) > tens;
      if (q == 0 && !high) --de;
      else dg.push_back((int)q);
      if (de < -3 || de >= 8) low = high = false;
      while (!low && !high) {
        q = b / sv;
        b = wr((unsigned __int128)(uint64_t)(b % sv) * 10);
        m = wr((unsigned __int128)(uint64_t)m * 10);
        if (m > 0) {
          low = b < m;
          high = wr((unsigned __int128)(uint64_t)b + (uint64_t)m) > tens;
        } else {
          low = high = true;
        }
        dg.push_back((int)q);
      }
      const int64_t diff = wr((unsigned __int128)(uint64_t)wr((unsigned __int128)(uint64_t)b << 1) - (uint64_t)tens);
      ldiff = diff > 0 ? 1 : diff < 0 ? -1 : 0;
    } else {
      const Mag S = mag_of(1, S5, S2), T = mag_of(1, S5 + 1, S2 + 1);
      Mag B = mag_of(fr, B5, B2), M = mag_of(1, B5 + 1, M2 + 1);
      auto step = [&]() {
        int q = 0;
        while (mag_cmp(B, S) >= 0) { mag_sub(B, S); ++q; }
        B = mag_mul10(B);
        return q;
      };
      int q = step();
      low = mag_cmp(B, M) < 0;
      high = mag_cmp(mag_add(B, M), T) >= 0;
      if (q == 0 && !high) --de;
      else dg.push_back(q);
      if (de < -3 || de >= 8) low = high = false;
      while (!low && !high) {
        q = step();
        M = mag_mul10(M);
        low = mag_cmp(B, M) < 0;
        high = mag_cmp(mag_add(B, M), T) >= 0;
        dg.push_back(q);
      }
      ldiff = high && low ? mag_cmp(mag_add(B, B), T) : 0;
    }
    decexp = de + 1;
    const bool up = high && (!low || ldiff > 0 || (ldiff == 0 && (dg.back() & 1)));
    if (up) {  // roundup: the digit count stays
      size_t i = dg.size() - 1;
      while (dg[i] == 9 && i > 0) dg[i--] = 0;
      if (dg[i] == 9) { dg[0] = 1; ++decexp; }
      else ++dg[i];
    }
  }
  std::string ds;
  for (int x : dg) ds.push_back((char)('0' + x));
  std::string out = neg ? "-" : "";
  const int n = (int)ds.size();
  if (decexp > 0 && decexp < 8) {
    const int c = std::min(n, decexp);
    out += ds.substr(0, c);
    if (c < decexp) out += std::string(decexp - c, '0') + ".0";
    else out += "." + (c < n ? ds.substr(c) : std::string("0"));
  } else if (decexp <= 0 && decexp > -3) {
    out += "0." + std::string(-decexp, '0') + ds;
  } else {
    out += ds.substr(0, 1) + "." + (n > 1 ? ds.substr(1) : std::string("0")) + "E" +
           (decexp <= 0 ? "-" + std::to_string(1 - decexp) : std::to_string(decexp - 1));
  }
  return out;
}

int32_t java_hash_append(int32_t h, const std::string& s) {
  uint32_t u = (uint32_t)h;
  for (unsigned char c : s) u = 31u * u + c;
  return (int32_t)u;
}

// ------------------------------------------------------------------------------------------
// Event model (event/stream/StreamEvent.java, event/state/StateEvent.java)
// ------------------------------------------------------------------------------------------
struct InEvent {     // an input event (values live here; StreamEvents are per-use copies)
  int stream;
  i64 ts;
  std::vector<i64> vals;
  std::vector<uint8_t> nulls;
};

struct StreamEvent {  // copyStreamEvent result: same values, own `next` link
  i64 seq;
  i64 ts;
  StreamEvent* next = nullptr;
  bool mark = false;
};

struct StateEvent {
  std::vector<StreamEvent*> slots;
  i64 ts = -1;
  bool mark = false;
};

struct Heap {
  std::vector<StreamEvent*> sev;
  std::vector<StateEvent*> stev;
  size_t last_live = 0;
  ~Heap() {
    for (auto* p : sev) delete p;
    for (auto* p : stev) delete p;
  }
  StreamEvent* copy(i64 seq, i64 ts) {
    auto* e = new StreamEvent{seq, ts};
    sev.push_back(e);
    return e;
  }
  StateEvent* state(size_t n) {
    auto* s = new StateEvent;
    s->slots.assign(n, nullptr);
    stev.push_back(s);
    return s;
  }
};

// Java semantics helpers ----------------------------------------------------------------------
struct Value {
  int type = T_INT;
  bool null = true;
  i64 i = 0;     // int/long/bool/string-id
  float f = 0;
  double d = 0;
};

Value mk_null() { return Value(); }

float as_f(const Value& v) {  // Number.floatValue() / binary numeric promotion to float
  switch (v.type) {
    case T_INT: return (float)(int32_t)v.i;
    case T_LONG: return (float)v.i;
    case T_FLOAT: return v.f;
    default: return (float)v.d;
  }
}
double as_d(const Value& v) {
  switch (v.type) {
    case T_INT: return (double)(int32_t)v.i;
    case T_LONG: return (double)v.i;
    case T_FLOAT: return (double)v.f;
    default: return v.d;
  }
}
i64 as_l(const Value& v) { return v.i; }  // only int/long reach here

template <class T>
bool cmp_op(int op, T a, T b) {
  switch (op) {
    case CMP_EQ: return a == b;
    case CMP_NE: return a != b;
    case CMP_GT: return a > b;
    case CMP_GE: return a >= b;
    case CMP_LT: return a < b;
    default: return a <= b;
  }
}

// The typed compare table of executor/condition/compare/** (execute() bodies at lines 33-38):
// ordering compares use Java binary numeric promotion; ==/!= follow each executor's explicit
// conversion, which differs only for Long x Float / Float x Long (both sides .doubleValue()).
bool typed_compare(int op, const Value& l, const Value& r) {
  int lt = l.type, rt = r.type;
  if (lt == T_STRING || lt == T_BOOL) {
    bool eq = l.i == r.i;  // String.equals on dictionary ids / boolean ==
    return op == CMP_EQ ? eq : !eq;
  }
  bool is_eq = (op == CMP_EQ || op == CMP_NE);
  if (lt == T_DOUBLE || rt == T_DOUBLE) return cmp_op(op, as_d(l), as_d(r));
  if (lt == T_FLOAT || rt == T_FLOAT) {
    if (is_eq && (lt == T_LONG || rt == T_LONG))  // EqualCompare...LongFloat.java:36 / FloatLong.java:37
      return cmp_op(op, as_d(l), as_d(r));
    return cmp_op(op, as_f(l), as_f(r));
  }
  if (lt == T_LONG || rt == T_LONG) return cmp_op(op, as_l(l), as_l(r));
  return cmp_op(op, (int32_t)l.i, (int32_t)r.i);
}

// executor/math/{add,subtract,multiply,divide,mod}/*.java: null in -> null; /0 and %0 -> null
// for every type (incl. 0.0f / -0.0); integer ops wrap like the JVM.
Value arith(int op, int res, const Value& l, const Value& r) {
  Value v;
  v.type = res;
  if (l.null || r.null) return mk_null();
  v.null = false;
  if (res == T_INT) {
    int32_t a = (int32_t)l.i, b = (int32_t)r.i;
    uint32_t ua = (uint32_t)a, ub = (uint32_t)b;
    switch (op) {
      case AR_ADD: v.i = (int32_t)(ua + ub); break;
      case AR_SUB: v.i = (int32_t)(ua - ub); break;
      case AR_MUL: v.i = (int32_t)(ua * ub); break;
      case AR_DIV:
        if (b == 0) return mk_null();
        v.i = (a == INT32_MIN && b == -1) ? INT32_MIN : a / b;
        break;
      default:
        if (b == 0) return mk_null();
        v.i = (b == -1) ? 0 : a % b;
    }
  } else if (res == T_LONG) {
    i64 a = l.i, b = r.i;
    uint64_t ua = (uint64_t)a, ub = (uint64_t)b;
    switch (op) {
      case AR_ADD: v.i = (i64)(ua + ub); break;
      case AR_SUB: v.i = (i64)(ua - ub); break;
      case AR_MUL: v.i = (i64)(ua * ub); break;
      case AR_DIV:
        if (b == 0) return mk_null();
        v.i = (a == INT64_MIN && b == -1) ? INT64_MIN : a / b;
        break;
      default:
        if (b == 0) return mk_null();
        v.i = (b == -1) ? 0 : a % b;
    }
  } else if (res == T_FLOAT) {
    volatile float a = as_f(l), b = as_f(r);
    switch (op) {
      case AR_ADD: v.f = a + b; break;
      case AR_SUB: v.f = a - b; break;
      case AR_MUL: v.f = a * b; break;
      case AR_DIV: if (b == 0.0f) return mk_null(); v.f = a / b; break;
      default: if (b == 0.0f) return mk_null(); v.f = std::fmod((float)a, (float)b);
    }
  } else {
    volatile double a = as_d(l), b = as_d(r);
    switch (op) {
      case AR_ADD: v.d = a + b; break;
      case AR_SUB: v.d = a - b; break;
      case AR_MUL: v.d = a * b; break;
      case AR_DIV: if (b == 0.0) return mk_null(); v.d = a / b; break;
      default: if (b == 0.0) return mk_null(); v.d = std::fmod((double)a, (double)b);
    }
  }
  return v;
}

// StateEvent.getStreamEvent(int[] position), StateEvent.java:138-182
StreamEvent* chain_at(StreamEvent* head, i64 idx) {
  if (!head) return nullptr;
  if (idx >= 0) {
    StreamEvent* e = head;
    for (i64 k = 1; k <= idx; ++k) {
      e = e->next;
      if (!e) return nullptr;
    }
    return e;
  }
  if (idx == -1) {  // CURRENT
    StreamEvent* e = head;
    while (e->next) e = e->next;
    return e;
  }
  if (idx == -2) {  // LAST
    if (!head->next) return nullptr;
    StreamEvent* e = head;
    while (e->next->next) e = e->next;
    return e;
  }
  std::vector<StreamEvent*> v;
  for (StreamEvent* e = head; e; e = e->next) v.push_back(e);
  i64 k = (i64)v.size() + idx;
  if (k < 0) return nullptr;
  return v[k];
}

struct Engine;

struct EvalCtx {
  const std::vector<InEvent>* log;
  const std::vector<std::vector<int>>* stream_types;
};

Value load_attr(const EvalCtx& cx, StreamEvent* ev, int attr, int type) {
  if (!ev) return mk_null();
  const InEvent& in = (*cx.log)[ev->seq];
  if (in.nulls[attr]) return mk_null();
  Value v;
  v.type = type;
  v.null = false;
  i64 raw = in.vals[attr];
  switch (type) {
    case T_INT: v.i = (int32_t)raw; break;
    case T_FLOAT: { uint32_t b = (uint32_t)raw; std::memcpy(&v.f, &b, 4); break; }
    case T_DOUBLE: std::memcpy(&v.d, &raw, 8); break;
    default: v.i = raw;
  }
  return v;
}

Value run_code(const EvalCtx& cx, const Code& code, const std::vector<StreamEvent*>& slots) {
  std::vector<Value> st;
  st.reserve(16);
  for (const Insn& in : code) {
    switch (in.op) {
      case OP_CONST: {
        Value v;
        v.type = in.res;
        v.null = false;
        if (in.res == T_FLOAT) { uint32_t b = (uint32_t)in.imm; std::memcpy(&v.f, &b, 4); }
        else if (in.res == T_DOUBLE) std::memcpy(&v.d, &in.imm, 8);
        else if (in.res == T_INT) v.i = (int32_t)in.imm;
        else v.i = in.imm;
        st.push_back(v);
        break;
      }
      case OP_ATTR:
        st.push_back(load_attr(cx, chain_at(slots[in.a], in.b), (int)in.imm, in.res));
        break;
      case OP_STREAM_IS_NULL: {  // IsNullStreamConditionExpressionExecutor
        Value v; v.type = T_BOOL; v.null = false;
        v.i = chain_at(slots[in.a], in.b) == nullptr;
        st.push_back(v);
        break;
      }
      case OP_IS_NULL: {
        Value x = st.back(); st.pop_back();
        Value v; v.type = T_BOOL; v.null = false; v.i = x.null;
        st.push_back(v);
        break;
      }
      case OP_NOT: {  // NotConditionExpressionExecutor: only TRUE -> FALSE
        Value x = st.back(); st.pop_back();
        Value v; v.type = T_BOOL; v.null = false;
        v.i = !(!x.null && x.i);
        st.push_back(v);
        break;
      }
      case OP_AND:
      case OP_OR: {  // And/OrConditionExpressionExecutor: null is false
        Value r = st.back(); st.pop_back();
        Value l = st.back(); st.pop_back();
        bool lb = !l.null && l.i, rb = !r.null && r.i;
        Value v; v.type = T_BOOL; v.null = false;
        v.i = in.op == OP_AND ? (lb && rb) : (lb || rb);
        st.push_back(v);
        break;
      }
      case OP_CMP: {  // CompareConditionExpressionExecutor.java:39-43
        Value r = st.back(); st.pop_back();
        Value l = st.back(); st.pop_back();
        Value v; v.type = T_BOOL; v.null = false;
        v.i = (!l.null && !r.null) && typed_compare((int)in.imm, l, r);
        st.push_back(v);
        break;
      }
      case OP_ARITH: {
        Value r = st.back(); st.pop_back();
        Value l = st.back(); st.pop_back();
        st.push_back(arith((int)in.imm, in.res, l, r));
        break;
      }
      default: throw std::runtime_error("bad opcode");
    }
  }
  if (st.size() != 1) throw std::runtime_error("malformed bytecode");
  return st.back();
}

// ------------------------------------------------------------------------------------------
// One query runtime (one StateStreamRuntime, or one per-key clone of it)
// ------------------------------------------------------------------------------------------
struct Match {
  int query;
  i64 key;
  i64 ts;
  std::vector<std::vector<i64>> slots;
  // merge metadata (multi-rank tests): the sequence number of the event whose processing produced
  // the match (timers: the event they fire before, or the next sequence number on an advance), and
  // for an absent state's timer match the instance's running max of fired times, else INT64_MIN
  i64 seq = -1;
  i64 tb = INT64_MIN;
};

struct Runtime;

struct Pre {
  // StreamPreStateProcessor / CountPreStateProcessor / LogicalPreStateProcessor state
  std::list<StateEvent*> pending, newAndEvery;
  bool stateChanged = false, initialized = false;
  bool successCondition = false, startStateReset = false;  // CountPreStateProcessor
  bool iterating = false;
  // AbsentStreamPreStateProcessor (state/AbsentStreamPreStateProcessor.java:38-54) and its
  // Scheduler's toNotifyQueue (util/Scheduler.java:45: a FIFO of notification times)
  i64 lastScheduledTime = 0;
  bool active = true;
  std::list<i64> timers;
  i64 lastArrivalTime = 0;  // AbsentLogicalPreStateProcessor.java:42
};
struct Post {
  bool isEventReturned = false;
};

struct Runtime {
  Engine* eng;
  int qi;
  i64 key;
  const QueryDef* q;
  std::vector<Pre> pres;
  std::vector<Post> posts;

  Runtime(Engine* e, int qi_, i64 key_, const QueryDef* qd)
      : eng(e), qi(qi_), key(key_), q(qd), pres(qd->states.size()), posts(qd->states.size()) {}

  size_t nslots() const { return q->states.size(); }
  const StateDef& S(int i) const { return q->states[i]; }
  // an absent side of a logical state (AbsentLogicalPre/PostStateProcessor); IR waiting_ms -2 is
  // `and not B` without 'for' (the reference's waitingTime -1)
  bool absentL(int i) const { return S(i).kind == K_LOGICAL && S(i).waiting != -1; }
  i64 W(int i) const { return S(i).waiting == -2 ? -1 : S(i).waiting; }
  bool absentAny(int i) const { return S(i).kind == K_ABSENT || absentL(i); }

  // ---- pre processors -----------------------------------------------------------------------
  // StreamPreStateProcessor.init():157-166 (a SEQUENCE start whose next state is absent re-inits too)
  void init_pre(int i) {
    const StateDef& s = S(i);
    Pre& p = pres[i];
    const bool absent_next = q->type == Q_SEQUENCE && s.next_pre >= 0 && absentAny(s.next_pre);
    if (s.is_start && (!p.initialized || s.next_every >= 0 || absent_next)) {
      StateEvent* se = new_state();
      addState(i, se);
      p.initialized = true;
    }
  }
  StateEvent* new_state();

  // StreamPreStateProcessor.addState:203-216 / CountPreStateProcessor.addState:109-132 /
  // LogicalPreStateProcessor.addState:57-76
  void addState(int i, StateEvent* se) {
    const StateDef& s = S(i);
    Pre& p = pres[i];
    if (s.kind == K_LOGICAL) {
      if (absentL(i) && !p.active) return;  // AbsentLogicalPreStateProcessor.addState:64-86
      Pre& pp = pres[s.partner];
      if (s.is_start || q->type == Q_SEQUENCE) {
        if (p.newAndEvery.empty()) p.newAndEvery.push_back(se);
        if (pp.newAndEvery.empty()) pp.newAndEvery.push_back(se);
      } else {
        p.newAndEvery.push_back(se);
        pp.newAndEvery.push_back(se);
      }
      if (absentL(i) && !s.is_start && W(i) != -1) {
        p.timers.push_back(se->ts + W(i));
        if (absentL(s.partner)) pp.timers.push_back(se->ts + W(s.partner));
      }
      return;
    }
    if (s.kind == K_ABSENT) {  // AbsentStreamPreStateProcessor.addState:78-101
      if (!p.active) return;
      if (q->type == Q_SEQUENCE) p.newAndEvery.clear();
      p.newAndEvery.push_back(se);
      if (!s.is_start) {
        p.lastScheduledTime = se->ts + s.waiting;
        p.timers.push_back(p.lastScheduledTime);
      }
      return;
    }
    if (q->type == Q_SEQUENCE) {
      if (p.newAndEvery.empty()) p.newAndEvery.push_back(se);
    } else {
      p.newAndEvery.push_back(se);
    }
    if (s.kind == K_COUNT && s.min == 0 && se->slots[i] == nullptr) processMinCountReached(i, se);
  }

  // StreamPreStateProcessor.addEveryState:218-227 (slot NOT cleared) /
  // LogicalPreStateProcessor.addEveryState:78-92 (own and partner slots cleared)
  void addEveryState(int i, StateEvent* se) {
    const StateDef& s = S(i);
    StateEvent* c = clone(se);
    if (s.kind == K_LOGICAL) {
      // AbsentLogicalPreStateProcessor.addEveryState:89-100 keeps the time of its own last event
      if (absentL(i) && c->slots[i]) c->ts = c->slots[i]->ts;
      c->slots[i] = nullptr;
      pres[i].newAndEvery.push_back(c);
      c->slots[s.partner] = nullptr;
      pres[s.partner].newAndEvery.push_back(c);
      return;
    }
    pres[i].newAndEvery.push_back(c);
    if (s.kind == K_ABSENT) {  // AbsentStreamPreStateProcessor.addEveryState:103-115
      pres[i].lastScheduledTime = se->ts + s.waiting;
      pres[i].timers.push_back(pres[i].lastScheduledTime);
    }
  }

  StateEvent* clone(StateEvent* se);  // StateEventCloner.copyStateEvent:46-58 (shallow)

  void promote(int i) {
    Pre& p = pres[i];
    if (p.iterating && !p.newAndEvery.empty())  // Java LinkedList iterator -> CME on next()
      throw std::runtime_error("ConcurrentModificationException (reference engine would throw)");
    p.pending.splice(p.pending.end(), p.newAndEvery);
  }

  // updateState: StreamPre:281-289, CountPre:149-156, LogicalPre:118-130
  void updateState(int i) {
    const StateDef& s = S(i);
    if (s.kind == K_COUNT && pres[i].startStateReset) {
      pres[i].startStateReset = false;
      init_pre(i);
    }
    promote(i);
    if (s.kind == K_LOGICAL) promote(s.partner);
  }

  // resetState: StreamPre:262-278, LogicalPre:94-116
  void resetState(int i) {
    const StateDef& s = S(i);
    Pre& p = pres[i];
    if (s.kind == K_LOGICAL) {
      Pre& pp = pres[s.partner];
      if (s.ltype == L_OR || p.pending.size() == pp.pending.size()) {
        p.pending.clear();
        pp.pending.clear();
        if (s.is_start && p.newAndEvery.empty()) {
          if (q->type == Q_SEQUENCE && s.next_every < 0 && next_pending_nonempty(i)) return;
          init_pre(i);
        }
      }
      return;
    }
    p.pending.clear();
    // AbsentStreamPreStateProcessor.resetState:117-138 re-inits a start state whatever its
    // newAndEvery list holds
    if (s.is_start && (s.kind == K_ABSENT || p.newAndEvery.empty())) {
      if (q->type == Q_SEQUENCE && s.next_every < 0 && next_pending_nonempty(i)) return;
      init_pre(i);
    }
  }
  bool next_pending_nonempty(int i) {
    int n = S(i).next_pre;
    if (n < 0) throw std::runtime_error("NullPointerException in resetState (no next state)");
    return !pres[n].pending.empty();
  }

  // CountPreStateProcessor.startStateReset:142-147
  void startStateReset(int i) {
    if (S(i).kind != K_COUNT) throw std::runtime_error("callback target is not a count state");
    pres[i].startStateReset = true;
    if (S(i).callback >= 0) throw std::runtime_error("StackOverflowError in startStateReset (reference)");
  }

  bool isExpired(int i, StateEvent* se, i64 ts) {  // StreamPreStateProcessor.isExpired:102-113
    const StateDef& s = S(i);
    if (!s.is_start && q->within >= 0) {
      for (int sid : q->start_ids) {
        StreamEvent* ev = se->slots[sid];
        if (ev) {
          uint64_t d = (uint64_t)ev->ts - (uint64_t)ts;
          i64 sd = (i64)d;
          i64 a = sd < 0 ? (i64)(0 - (uint64_t)sd) : sd;  // Math.abs(long), MIN stays MIN
          if (a > q->within) return true;
        }
      }
    }
    return false;
  }

  // StreamPreStateProcessor.process(StateEvent):115-121 -> FilterProcessor chain -> post
  void process(int i, StateEvent* se);
  bool filters_pass(int i, StateEvent* se);

  // ---- post processors ------------------------------------------------------------------------
  // StreamPostStateProcessor.process:53-72
  void streamPost(int i, StateEvent* se) {
    const StateDef& s = S(i);
    pres[i].stateChanged = true;
    se->ts = se->slots[i]->ts;
    if (s.has_selector) posts[i].isEventReturned = true;
    if (s.next_pre >= 0) addState(s.next_pre, se);
    if (s.next_every >= 0) addEveryState(s.next_every, se);
    if (s.callback >= 0) startStateReset(s.callback);
  }
  // CountPostStateProcessor.processMinCountReached:73-85
  void processMinCountReached(int i, StateEvent* se) {
    const StateDef& s = S(i);
    if (s.has_selector) {
      pres[i].stateChanged = true;
      posts[i].isEventReturned = true;
    }
    if (s.next_pre >= 0) addState(s.next_pre, se);
    if (s.next_every >= 0) addEveryState(s.next_every, se);
  }
  // CountPostStateProcessor.process:45-71
  void countPost(int i, StateEvent* se) {
    const StateDef& s = S(i);
    StreamEvent* e = se->slots[i];
    i64 n = 1;
    while (e->next) { ++n; e = e->next; }
    pres[i].successCondition = true;
    se->ts = e->ts;
    if (n >= s.min) {
      if (q->type == Q_SEQUENCE) {
        if (s.next_pre >= 0) addState(s.next_pre, se);
        if (n != s.max) addState(i, se);
      } else if (n == s.min) {
        processMinCountReached(i, se);
      }
      if (n == s.max) pres[i].stateChanged = true;
    }
  }
  // LogicalPostStateProcessor.process:59-87
  void logicalPost(int i, StateEvent* se) {
    const StateDef& s = S(i);
    if (absentL(i)) {  // AbsentLogicalPostStateProcessor.process:37-49
      pres[i].stateChanged = true;
      posts[i].isEventReturned = true;
      pres[i].lastArrivalTime = se->slots[i]->ts;  // updateLastArrivalTime
      return;
    }
    if (s.ltype == L_AND) {
      const bool go = absentL(s.partner) ? partnerCanProceed(s.partner, se) : se->slots[s.partner] != nullptr;
      if (go) streamPost(i, se);
      else pres[i].stateChanged = true;
    } else {
      streamPost(i, se);
      // 'from A or B select' case: thisStatePreProcessor.thisLastProcessor == partner post
      if (S(s.partner).has_selector && s.this_last == s.partner) posts[s.partner].isEventReturned = true;
    }
  }

  // AbsentStreamPostStateProcessor.process:31-52: the absent event arrived -- the partial is
  // dropped (stateChanged) and the waiting restarts from this event
  void absentPost(int i, StateEvent* se) {
    const StateDef& s = S(i);
    Pre& p = pres[i];
    p.stateChanged = true;
    StreamEvent* ev = se->slots[i];
    se->ts = ev->ts;
    posts[i].isEventReturned = true;
    if (s.is_start && s.next_every == i) addEveryState(i, se);
    p.lastScheduledTime = ev->ts + s.waiting;  // AbsentStreamPreStateProcessor.updateLastArrivalTime:69-75
    p.timers.push_back(p.lastScheduledTime);
  }
  // AbsentStreamPreStateProcessor.sendEvent:212-228
  void absentSend(int i, StateEvent* se);
  // AbsentStreamPreStateProcessor.process:140-210: a timer event of this processor's scheduler
  void absentTimer(int i, i64 currentTime, i64 actualCurrentTime);

  // AbsentLogicalPreStateProcessor.partnerCanProceed:342-372 (asked by the partner's AND post)
  bool partnerCanProceed(int j, StateEvent* se) {
    const StateDef& a = S(j);
    Pre& pa = pres[j];
    if (q->type == Q_SEQUENCE && a.next_every < 0 && pa.lastArrivalTime > 0) return false;
    if (W(j) == -1) {
      if (a.next_every < 0) return se->slots[j] == nullptr;
      if (pa.lastArrivalTime > 0) {
        pa.lastArrivalTime = 0;
        init_pre(j);
        return false;
      }
      return true;
    }
    return se->slots[j] != nullptr;
  }
  // StateEvent.addEvent:212-222 with StreamEventPool.borrowEvent()'s empty event (no data, ts -1)
  void addDummyEvent(StateEvent* se, int i);
  void absentLogicalSend(int i, StateEvent* se);                        // :225-244
  void absentLogicalTimer(int i, i64 currentTime, i64 actualCurrentTime);  // :107-181
  std::vector<StateEvent*> absentLogicalProcessAndReturn(int i, i64 seq, i64 ts);  // :246-300

  // ---- processAndReturn -----------------------------------------------------------------------
  std::vector<StateEvent*> processAndReturn(int i, i64 seq, i64 ts);

  // ---- inner state runtime tree (state/runtime/*InnerStateRuntime.java) ---------------------
  void node_init(int n) {
    const NodeDef& d = q->nodes[n];
    switch (d.type) {
      case N_STREAM: case N_COUNT: init_pre(d.pre); break;
      case N_NEXT: node_init(d.a); node_init(d.b); break;
      case N_EVERY: node_init(d.a); break;
      case N_LOGICAL: node_init(d.b); node_init(d.a); break;
    }
  }
  void node_reset(int n) {
    const NodeDef& d = q->nodes[n];
    switch (d.type) {
      case N_STREAM: case N_COUNT: case N_EVERY: resetState(d.pre); break;
      case N_NEXT: node_reset(d.b); node_reset(d.a); break;
      case N_LOGICAL: node_reset(d.b); break;
    }
  }
  void node_update(int n) {
    const NodeDef& d = q->nodes[n];
    switch (d.type) {
      case N_STREAM: case N_COUNT: case N_EVERY: updateState(d.pre); break;
      case N_NEXT: node_update(d.a); node_update(d.b); break;
      case N_LOGICAL: node_update(d.b); break;
    }
  }

  void receive(int stream, i64 seq, i64 ts);
  void mark_roots();
};

struct Engine {
  Program prog;
  std::vector<InEvent> log;
  Heap heap;
  std::vector<std::unique_ptr<Runtime>> top;        // unpartitioned queries (index = query)
  // per partition: key -> instance runtimes (one per partition query)
  std::vector<std::map<i64, std::vector<std::unique_ptr<Runtime>>>> part_inst;
  std::vector<std::vector<i64>> key_order;          // creation order per partition
  std::vector<int> key_type;                        // per partition: the keys' value type
  std::vector<Match> matches;
  std::vector<std::pair<Runtime*, StateEvent*>> deferred;  // single-receiver chunk deferral
  std::vector<i64> deferred_seq;
  std::string err;
  i64 cur_seq = 0;             // the event being processed (Match::seq)
  std::map<i64, std::pair<int32_t, int64_t>> str_info;  // dictionary id -> (String.hashCode, length)
  bool in_timer = false;       // a timer is firing (Match::tb = timer_key)
  i64 timer_key = INT64_MIN;
  size_t gc_threshold = 1 << 20;
  // time (the runtime's TimestampGenerator): the last event's timestamp or an explicit advance;
  // absent processors' schedulers fire at their notification times as it passes them
  bool started = false;
  i64 now = 0;
  bool has_absent = false;
  bool playback = false;  // @app:playback (TimestampGeneratorImpl.currentTime = the last event time)

  // SiddhiAppRuntime.start -> AbsentStreamPreStateProcessor.start:276-286 (start states with a
  // 'for' time schedule their first check)
  void start(i64 t) {
    started = true;
    now = t;
    for (auto& r : top) {
      if (!r) continue;
      for (size_t i = 0; i < r->pres.size(); ++i) {
        const StateDef& s = r->q->states[i];
        Pre& p = r->pres[i];
        if (s.kind == K_ABSENT && s.is_start && s.waiting != -1 && p.active) {
          p.lastScheduledTime = t + s.waiting;
          p.timers.push_back(p.lastScheduledTime);
        }
        // AbsentLogicalPreStateProcessor.start:320-330
        if (r->absentL((int)i) && s.is_start && r->W((int)i) != -1 && p.active) p.timers.push_back(t + r->W((int)i));
      }
    }
  }
  // Scheduler.sendTimerEvents:186-214 for every scheduler, in time order, up to time t: the
  // scheduler whose queue head is earliest fires its head (ties: query, then state order); a timer
  // may schedule more (they fire too if due)
  void advance(i64 t) {
    if (!started) start(t);
    if (has_absent) {
      // per instance, the running max of the times fired in this call (the device's timer tiebreak,
      // kgen.h fire_timers)
      std::map<Runtime*, i64> runmax;
      for (;;) {
        // every scheduler in (query, key) order -- top-level runtimes and each partition's per-key
        // clones (PartitionRuntime.cloneIfNotExist gives every key its own schedulers; clones are
        // never start()ed) -- the earliest queue head fires first, ties in that order
        Runtime* best = nullptr;
        int bi = -1;
        i64 bt = 0;
        auto consider = [&](Runtime* r) {
          for (size_t i = 0; i < r->pres.size(); ++i) {
            const Pre& p = r->pres[i];
            if (p.timers.empty() || p.timers.front() > t) continue;
            if (!best || p.timers.front() < bt) {
              best = r;
              bi = (int)i;
              bt = p.timers.front();
            }
          }
        };
        for (size_t qi = 0; qi < prog.queries.size(); ++qi) {
          const int pi = prog.queries[qi].partition;
          if (pi < 0) {
            if (top[qi]) consider(top[qi].get());
            continue;
          }
          const auto& qs = prog.parts[pi].queries;
          const size_t slot = std::find(qs.begin(), qs.end(), (int)qi) - qs.begin();
          for (auto& kv : part_inst[pi]) consider(kv.second[slot].get());
        }
        if (!best) break;
        best->pres[bi].timers.pop_front();
        now = bt;
        i64& rm = runmax.emplace(best, INT64_MIN).first->second;
        rm = bt > rm ? bt : rm;
        in_timer = true;
        timer_key = rm;
        if (best->absentL(bi)) best->absentLogicalTimer(bi, bt, playback ? t : bt);
        else best->absentTimer(bi, bt, playback ? t : bt);
        in_timer = false;
      }
    }
    if (t > now) now = t;
  }

  void emit(Runtime* rt, StateEvent* se) {
    Match m;
    m.query = rt->qi;
    m.key = rt->key;
    m.ts = se->ts;
    m.slots.resize(se->slots.size());
    for (size_t k = 0; k < se->slots.size(); ++k)
      for (StreamEvent* e = se->slots[k]; e; e = e->next) m.slots[k].push_back(e->seq);
    m.seq = cur_seq;
    m.tb = in_timer ? timer_key : INT64_MIN;
    matches.push_back(std::move(m));
  }

  void gc() {
    size_t live_before = heap.sev.size() + heap.stev.size();
    if (live_before < gc_threshold) return;
    for (auto& r : top) if (r) r->mark_roots();
    for (auto& pr : deferred) {
      pr.second->mark = true;
      for (StreamEvent* ev : pr.second->slots)
        for (; ev && !ev->mark; ev = ev->next) ev->mark = true;
    }
    for (auto& pm : part_inst)
      for (auto& kv : pm)
        for (auto& r : kv.second) r->mark_roots();
    size_t w = 0;
    for (auto* s : heap.stev) {
      if (s->mark) { s->mark = false; heap.stev[w++] = s; } else delete s;
    }
    heap.stev.resize(w);
    w = 0;
    for (auto* e : heap.sev) {
      if (e->mark) { e->mark = false; heap.sev[w++] = e; } else delete e;
    }
    heap.sev.resize(w);
    size_t live = heap.sev.size() + heap.stev.size();
    gc_threshold = std::max<size_t>(1 << 20, live * 2);
  }
};

StateEvent* Runtime::new_state() { return eng->heap.state(nslots()); }

void Runtime::addDummyEvent(StateEvent* se, int i) {
  StreamEvent* ev = eng->heap.copy(-1, -1);
  if (!se->slots[i]) se->slots[i] = ev;
  else { StreamEvent* t = se->slots[i]; while (t->next) t = t->next; t->next = ev; }
}

StateEvent* Runtime::clone(StateEvent* se) {
  StateEvent* c = eng->heap.state(nslots());
  c->slots = se->slots;
  c->ts = se->ts;
  return c;
}

bool Runtime::filters_pass(int i, StateEvent* se) {
  EvalCtx cx{&eng->log, &eng->prog.stream_types};
  for (const Code& f : S(i).filters) {
    Value v = run_code(cx, f, se->slots);
    if (v.null || !v.i) return false;  // FilterProcessor.process:55-66
  }
  return true;
}

void Runtime::process(int i, StateEvent* se) {
  pres[i].stateChanged = false;
  if (!filters_pass(i, se)) return;
  switch (S(i).kind) {
    case K_STREAM: streamPost(i, se); break;
    case K_ABSENT: absentPost(i, se); break;
    case K_COUNT: countPost(i, se); break;
    default: logicalPost(i, se); break;
  }
}

std::vector<StateEvent*> Runtime::processAndReturn(int i, i64 seq, i64 ts) {
  std::vector<StateEvent*> ret;
  const StateDef& s = S(i);
  Pre& p = pres[i];
  if (s.kind == K_ABSENT && !p.active) return ret;  // AbsentStreamPreStateProcessor.processAndReturn:231-244
  if (absentL(i)) return absentLogicalProcessAndReturn(i, seq, ts);
  p.iterating = true;
  for (auto it = p.pending.begin(); it != p.pending.end();) {
    StateEvent* se = *it;
    if (s.kind == K_COUNT) {
      // CountPreStateProcessor.processAndReturn:53-93 (no within check, R9)
      if ((int)nslots() > i + 1 && se->slots[i + 1] != nullptr) { it = p.pending.erase(it); continue; }
      if ((int)nslots() > i + 2 && se->slots[i + 2] != nullptr) { it = p.pending.erase(it); continue; }
      StreamEvent* ev = eng->heap.copy(seq, ts);
      if (!se->slots[i]) se->slots[i] = ev;        // StateEvent.addEvent:212-222
      else { StreamEvent* t = se->slots[i]; while (t->next) t = t->next; t->next = ev; }
      p.successCondition = false;
      process(i, se);
      if (posts[s.this_last].isEventReturned) {
        posts[s.this_last].isEventReturned = false;
        ret.push_back(se);
      }
      bool removed = false;
      if (p.stateChanged) { it = p.pending.erase(it); removed = true; }
      if (!p.successCondition) {
        // StateEvent.removeLastEvent:224-236
        StreamEvent* a = se->slots[i];
        if (a) {
          bool done = false;
          while (a->next) {
            if (!a->next->next) { a->next = nullptr; done = true; break; }
            a = a->next;
          }
          if (!done) se->slots[i] = nullptr;
        }
        if (q->type == Q_SEQUENCE) {
          if (removed) throw std::runtime_error("IllegalStateException (double iterator.remove)");
          it = p.pending.erase(it);
          removed = true;
        }
      }
      if (!removed) ++it;
      continue;
    }
    // StreamPreStateProcessor.processAndReturn:292-337 / LogicalPreStateProcessor:133-178
    if (isExpired(i, se, ts)) {
      it = p.pending.erase(it);
      if (s.within_every >= 0) {
        addEveryState(s.within_every, se);
        updateState(s.within_every);
      }
      continue;
    }
    if (s.kind == K_LOGICAL && s.ltype == L_OR && se->slots[s.partner] != nullptr) {
      it = p.pending.erase(it);
      continue;
    }
    se->slots[i] = eng->heap.copy(seq, ts);
    process(i, se);
    if (posts[s.this_last].isEventReturned) {
      posts[s.this_last].isEventReturned = false;
      ret.push_back(se);
    }
    if (p.stateChanged) {
      it = p.pending.erase(it);
    } else {
      se->slots[i] = nullptr;
      if (q->type == Q_SEQUENCE) {
        // removeOnNoStateChange: true for StreamPre, false for AbsentStreamPre (:246-248)
        if (s.kind == K_ABSENT) ++it;
        else it = p.pending.erase(it);
        if ((s.kind == K_STREAM || s.kind == K_ABSENT) && s.callback >= 0) startStateReset(s.callback);
      } else {
        ++it;
      }
    }
  }
  p.iterating = false;
  if (s.kind == K_ABSENT) ret.clear();  // an absent processor always returns an empty chunk
  return ret;
}

void Runtime::absentSend(int i, StateEvent* se) {
  const StateDef& s = S(i);
  if (s.has_selector) eng->emit(this, se);   // thisStatePostProcessor.nextProcessor: the selector
  if (s.next_pre >= 0) addState(s.next_pre, se);
  if (s.next_every >= 0) addEveryState(s.next_every, se);
  else if (s.is_start) pres[i].active = false;
  if (s.callback >= 0) startStateReset(s.callback);
}

void Runtime::absentLogicalSend(int i, StateEvent* se) {
  const StateDef& s = S(i);
  if (s.has_selector) eng->emit(this, se);
  if (s.next_pre >= 0) addState(s.next_pre, se);
  if (s.next_every >= 0) {
    addEveryState(s.next_every, se);
  } else if (s.is_start) {
    pres[i].active = false;
    if (s.ltype == L_OR && absentL(s.partner)) pres[s.partner].active = false;
  }
  if (s.callback >= 0) startStateReset(s.callback);
}

void Runtime::absentLogicalTimer(int i, i64 currentTime, i64 actualCurrentTime) {
  const StateDef& s = S(i);
  Pre& p = pres[i];
  const i64 w = W(i);
  if (!p.active) return;
  bool notProcessed = true;
  if (currentTime >= p.lastArrivalTime + w) {
    std::vector<StateEvent*> ret;
    if (s.is_start && q->type == Q_SEQUENCE && p.newAndEvery.empty() && p.pending.empty()) {
      addState(i, new_state());
    } else if (q->type == Q_SEQUENCE && !p.newAndEvery.empty()) {
      resetState(i);
    }
    updateState(i);
    for (auto it = p.pending.begin(); it != p.pending.end();) {
      StateEvent* se = *it;
      if (isExpired(i, se, currentTime)) {
        it = p.pending.erase(it);
        if (s.within_every >= 0) {
          addEveryState(s.within_every, se);
          updateState(s.within_every);
        }
        continue;
      }
      // waitingTimePassed:184-192
      const bool passed = se->slots[i] == nullptr ? currentTime >= se->ts + w : currentTime >= se->slots[i]->ts + w;
      if (!passed) { ++it; continue; }
      it = p.pending.erase(it);
      const bool partner = se->slots[s.partner] != nullptr;
      if (s.ltype == L_OR && !partner) {
        addDummyEvent(se, i);
        ret.push_back(se);
      } else if (s.ltype == L_AND && partner) {
        ret.push_back(se);
      } else if (s.ltype == L_AND && !partner) {
        addDummyEvent(se, i);  // the partner may still proceed
      }
    }
    notProcessed = ret.empty();
    for (StateEvent* se : ret) absentLogicalSend(i, se);
    p.lastArrivalTime = 0;
  }
  if (s.next_every >= 0 || (notProcessed && s.is_start)) {
    const i64 nextBreak = p.lastArrivalTime == 0 ? actualCurrentTime + w : p.lastArrivalTime + w;
    p.timers.push_back(nextBreak);
  }
}

std::vector<StateEvent*> Runtime::absentLogicalProcessAndReturn(int i, i64 seq, i64 ts) {
  const StateDef& s = S(i);
  Pre& p = pres[i];
  if (!p.active) return {};
  p.iterating = true;
  for (auto it = p.pending.begin(); it != p.pending.end();) {
    StateEvent* se = *it;
    if (isExpired(i, se, ts)) {
      if (s.within_every >= 0) {
        addEveryState(s.within_every, se);
        updateState(s.within_every);
      }
      it = p.pending.erase(it);
      continue;
    }
    if (s.ltype == L_OR && se->slots[s.partner] != nullptr) {
      it = p.pending.erase(it);
      continue;
    }
    StreamEvent* cur = se->slots[i];
    se->slots[i] = eng->heap.copy(seq, ts);
    process(i, se);
    if (W(i) != -1 || (q->type == Q_SEQUENCE && s.ltype == L_AND && s.next_every >= 0)) se->slots[i] = cur;
    bool removed = false;
    if (posts[s.this_last].isEventReturned) {
      posts[s.this_last].isEventReturned = false;
      it = p.pending.erase(it);  // no longer an absent candidate
      removed = true;
      if (q->type == Q_SEQUENCE) {
        auto& pp = pres[s.partner].pending;
        for (auto jt = pp.begin(); jt != pp.end(); ++jt)
          if (*jt == se) { pp.erase(jt); break; }
      }
    }
    if (!p.stateChanged) {
      se->slots[i] = cur;
      if (q->type == Q_SEQUENCE) {
        if (removed) throw std::runtime_error("IllegalStateException (double iterator.remove)");
        it = p.pending.erase(it);
        removed = true;
      }
    }
    if (!removed) ++it;
  }
  p.iterating = false;
  return {};
}

void Runtime::absentTimer(int i, i64 currentTime, i64 actualCurrentTime) {
  const StateDef& s = S(i);
  Pre& p = pres[i];
  if (!p.active) return;
  std::vector<StateEvent*> ret;
  bool initialize = s.is_start && p.newAndEvery.empty() && p.pending.empty();
  if (initialize && q->type == Q_SEQUENCE && s.next_every < 0 && p.lastScheduledTime > 0) initialize = false;
  if (initialize) {
    addState(i, new_state());
  } else if (q->type == Q_SEQUENCE && !p.newAndEvery.empty()) {
    resetState(i);
  }
  updateState(i);
  for (auto it = p.pending.begin(); it != p.pending.end();) {
    StateEvent* se = *it;
    if (isExpired(i, se, currentTime)) {
      it = p.pending.erase(it);
      if (s.within_every >= 0 && s.next_every != i) {
        if (s.next_every < 0) throw std::runtime_error("NullPointerException in absent expiry (reference)");
        addEveryState(s.next_every, se);
      }
      continue;
    }
    if ((se->ts == -1 && currentTime >= p.lastScheduledTime) || (se->ts != -1 && currentTime >= se->ts + s.waiting)) {
      it = p.pending.erase(it);
      se->ts = currentTime;
      ret.push_back(se);
      continue;
    }
    ++it;
  }
  if (s.within_every >= 0) updateState(s.within_every);
  const bool notProcessed = ret.empty();
  for (StateEvent* se : ret) absentSend(i, se);
  // actualCurrentTime: the timestamp generator's time -- the timer's own in a live runtime, the
  // event time that let it fire in playback (:202-205)
  if (actualCurrentTime > s.waiting + currentTime) p.lastScheduledTime = actualCurrentTime + s.waiting;
  if (notProcessed && p.lastScheduledTime < currentTime) {
    p.lastScheduledTime = currentTime + s.waiting;
    p.timers.push_back(p.lastScheduledTime);
  }
}

void Runtime::receive(int stream, i64 seq, i64 ts) {
  eng->cur_seq = seq;
  const RecvDef* rv = nullptr;
  for (auto& r : q->recvs)
    if (r.stream == stream) rv = &r;
  if (!rv) return;
  if (rv->kind == R_SINGLE) {
    // SingleProcessStreamReceiver.processAndClear:57-80 (selector deferred to chunk end)
    if (q->type == Q_SEQUENCE) { node_reset(0); node_update(0); }   // StateStreamRuntime.resetAndUpdate
    else updateState(rv->procs[0]);                                  // PatternSingle.stabilizeStates
    for (StateEvent* se : processAndReturn(rv->procs[0], seq, ts)) {
      eng->deferred.push_back({this, se});
      eng->deferred_seq.push_back(seq);
    }
  } else {
    // MultiProcessStreamReceiver.receive:268-279 + StateMultiProcessStreamReceiver.processAndClear:53-74
    if (q->type == Q_SEQUENCE) { node_reset(0); node_update(0); }
    else for (int p : rv->procs) updateState(p);                     // PatternMulti.stabilizeStates
    for (int k = (int)rv->procs.size() - 1; k >= 0; --k)             // reverse registration order
      for (StateEvent* se : processAndReturn(rv->procs[k], seq, ts)) eng->emit(this, se);
  }
}

void Runtime::mark_roots() {
  auto mark_state = [](StateEvent* s) {
    s->mark = true;
    for (StreamEvent* e : s->slots)
      for (; e && !e->mark; e = e->next) e->mark = true;
  };
  for (Pre& p : pres) {
    for (StateEvent* s : p.pending) mark_state(s);
    for (StateEvent* s : p.newAndEvery) mark_state(s);
  }
}

i64 key_of(const Value& v) {
  // PartitionKey = String.valueOf(value) (ValuePartitionExecutor.java:34-40); the planner
  // restricts a partition's keys to one type class so raw-value identity equals string identity.
  switch (v.type) {
    case T_FLOAT: { float f = v.f; if (std::isnan(f)) return 0x7fc00000; uint32_t b; std::memcpy(&b, &f, 4); return b; }
    case T_DOUBLE: { double d = v.d; if (std::isnan(d)) return 0x7ff8000000000000LL; i64 b; std::memcpy(&b, &d, 8); return b; }
    default: return v.i;
  }
}

void deliver_deferred(Engine* e) {
  for (size_t i = 0; i < e->deferred.size(); ++i) {
    e->cur_seq = e->deferred_seq[i];
    e->emit(e->deferred[i].first, e->deferred[i].second);
  }
  e->deferred.clear();
  e->deferred_seq.clear();
}

// One receiver (a query, or a partition key's clone of it) processes its chunk event by event
// (ProcessStreamReceiver.receive(Event[]):137-151 / receive(ComplexEvent):105-119 build one
// ComplexEventChunk); a single-stream receiver hands its matches to the selector at the end of its
// chunk (SingleProcessStreamReceiver.processAndClear:57-80), a multi-stream one as they complete
// (StateMultiProcessStreamReceiver.processAndClear:53-74, Runtime::receive). A per-event send is a
// chunk of one event.
void run_chunk(Engine* e, Runtime* rt, int stream, const std::vector<i64>& seqs) {
  for (i64 seq : seqs) rt->receive(stream, seq, e->log[seq].ts);
  deliver_deferred(e);
}

// One junction subscriber (a top-level query, or a partition's PartitionStreamReceiver) receives
// the whole chunk before the next subscriber does (StreamJunction.sendEvent(Event[]):218-236 loops
// over its receivers in subscription order). Inside a partition the key's junction holds the clones
// in the partition's query order (PartitionRuntime.clonePartition:270 iterates metaQueryRuntimeMap,
// a ConcurrentHashMap of query names: the planner emits PartDef::queries in that order).
void deliver_to(Engine* e, int qi, int stream, const std::vector<i64>& seqs) {
  const Program& P = e->prog;
  const QueryDef& q = P.queries[qi];
  if (q.partition < 0) {
    run_chunk(e, e->top[qi].get(), stream, seqs);
    return;
  }
  const int pi = q.partition;
  const PartDef& pd = P.parts[pi];
  for (const FanOut& fo : pd.fanout) {
    if (fo.stream != stream) continue;
    // PartitionStreamReceiver.receive(Event[]):200-213 / receive(Event):166-175 with no executor
    // for this stream -> send(ComplexEvent):277-281: the whole chunk to every key's junction
    // "streamId + key" in its cachedStreamJunctionMap's order; keys joined it at clonePartition
    // (updatePartitionStreamReceivers:312-316), in creation order
    const auto& ko = e->key_order[pi];
    auto value_of = [&](i64 k) {  // String.valueOf (ValuePartitionExecutor.java:34-40)
      if (e->key_type[pi] == T_BOOL) return std::string(k ? "true" : "false");
      if (e->key_type[pi] == T_FLOAT) return java_fp_string((uint64_t)(uint32_t)k, false);
      if (e->key_type[pi] == T_DOUBLE) return java_fp_string((uint64_t)k, true);
      return std::to_string((long long)k);
    };
    // a string key's String.valueOf is its text: "streamId" + text hashes as id_hash * 31^len + hash
    auto key_hash = [&](i64 k) -> int32_t {
      if (e->key_type[pi] != T_STRING) return java_hash_append(fo.id_hash, value_of(k));
      auto it = e->str_info.find(k);
      if (it == e->str_info.end()) throw std::runtime_error("partition key string id without its text hash");
      uint32_t h = (uint32_t)fo.id_hash;
      for (int64_t c = 0; c < it->second.second; ++c) h *= 31u;
      return (int32_t)(h + (uint32_t)it->second.first);
    };
    JavaCHM m;
    for (size_t k = 0; k < ko.size(); ++k) m.put(key_hash(ko[k]), (int)k);
    for (int k : m.order())
      for (auto& rt : e->part_inst[pi].at(ko[(size_t)k])) run_chunk(e, rt.get(), stream, seqs);
    return;
  }
  const PartKey* pk = nullptr;  // (the planner allows one key per stream and partition)
  for (const PartKey& k : pd.keys)
    if (k.stream == stream) pk = &k;
  if (!pk) return;
  // PartitionStreamReceiver.receive(Event[]):214-239: the chunk splits into runs of consecutive
  // events with equal keys (an event whose key is null is skipped and does not end a run); each run
  // goes to its key's junction (send(String, ComplexEvent):270-275), the key's clones created on
  // its first run (PartitionRuntime.cloneIfNotExist:257-306, seeded at init)
  std::vector<i64> run;
  i64 run_key = 0;
  int run_type = T_INT;
  auto flush = [&]() {
    if (run.empty()) return;
    auto& inst = e->part_inst[pi];
    auto it = inst.find(run_key);
    if (it == inst.end()) {
      std::vector<std::unique_ptr<Runtime>> rts;
      for (int pq : pd.queries) {
        rts.emplace_back(new Runtime(e, pq, run_key, &P.queries[pq]));
        rts.back()->node_init(0);
      }
      it = inst.emplace(run_key, std::move(rts)).first;
      e->key_order[pi].push_back(run_key);
      e->key_type[pi] = run_type;
    }
    for (auto& rt : it->second) run_chunk(e, rt.get(), stream, run);
    run.clear();
  };
  for (i64 seq : seqs) {
    EvalCtx cx{&e->log, &P.stream_types};
    std::vector<StreamEvent*> slots(1);
    StreamEvent tmp{seq, e->log[seq].ts};
    slots[0] = &tmp;
    Value kv = run_code(cx, pk->code, slots);
    if (kv.null) continue;  // ValuePartitionExecutor.execute: a null value has no key
    const i64 key = key_of(kv);
    if (!run.empty() && key != run_key) flush();
    run_key = key;
    run_type = kv.type;
    run.push_back(seq);
  }
  flush();
}

void send_chunk(Engine* e, int stream, const std::vector<i64>& seqs) {
  const Program& P = e->prog;
  std::vector<char> part_done(P.parts.size(), 0);
  for (size_t qi = 0; qi < P.queries.size(); ++qi) {
    const QueryDef& q = P.queries[qi];
    if (q.partition >= 0) {
      if (part_done[q.partition]) continue;
      part_done[q.partition] = 1;
    }
    deliver_to(e, (int)qi, stream, seqs);
  }
}

}  // namespace

struct OracleEngine : Engine {};

extern "C" {

int oracle_create(const void* blob, size_t len, OracleEngine** out) {
  try {
    auto* e = new OracleEngine;
    e->prog = parse_ir(blob, len);
    e->top.resize(e->prog.queries.size());
    for (size_t qi = 0; qi < e->prog.queries.size(); ++qi) {
      if (e->prog.queries[qi].partition >= 0) continue;
      e->top[qi].reset(new Runtime(e, (int)qi, -1, &e->prog.queries[qi]));
      e->top[qi]->node_init(0);  // QueryRuntime.init -> StateStreamRuntime.setCommonProcessor
    }
    e->part_inst.resize(e->prog.parts.size());
    e->key_order.resize(e->prog.parts.size());
    e->key_type.resize(e->prog.parts.size(), T_INT);
    for (const auto& q : e->prog.queries)
      for (const auto& st : q.states) e->has_absent |= st.kind == K_ABSENT || (st.kind == K_LOGICAL && st.waiting != -1);
    *out = e;
    return 0;
  } catch (const std::exception& ex) {
    *out = nullptr;
    return -1;
  }
}

int oracle_send(OracleEngine* e, int32_t stream, int64_t n, const int64_t* ts, const int64_t* vals,
                const uint8_t* nulls, int as_chunk) {
  try {
    if (stream < 0 || stream >= (int)e->prog.stream_types.size()) throw std::runtime_error("bad stream");
    size_t na = e->prog.stream_types[stream].size();
    std::vector<i64> seqs;
    for (int64_t k = 0; k < n; ++k) {
      InEvent ev;
      ev.stream = stream;
      ev.ts = ts[k];
      ev.vals.assign(vals + k * na, vals + (k + 1) * na);
      if (nulls) ev.nulls.assign(nulls + k * na, nulls + (k + 1) * na);
      else ev.nulls.assign(na, 0);
      seqs.push_back((i64)e->log.size());
      e->log.push_back(std::move(ev));
      if (as_chunk) continue;
      // timers due up to this event fire before it (playback order: TimestampGenerator time
      // change -> Scheduler.sendTimerEvents before the event reaches the junction)
      e->cur_seq = seqs.back();
      e->advance(ts[k]);
      send_chunk(e, stream, seqs);
      seqs.clear();
      e->gc();
    }
    if (!seqs.empty()) {
      // InputHandler.send(Event[]):77-85: the generator's time moves once, to the chunk's last
      // timestamp, before the chunk reaches the junction -- the timers due by then fire first (with
      // the chunk's first seq), none fire inside the chunk. A runtime not started yet starts with
      // the chunk's first event, as with single events.
      e->cur_seq = seqs.front();
      if (!e->started) e->start(ts[0]);
      e->advance(ts[n - 1]);
      send_chunk(e, stream, seqs);
    }
    e->gc();
    return 0;
  } catch (const std::exception& ex) {
    e->err = ex.what();
    e->deferred.clear();
    e->deferred_seq.clear();
    return -1;
  }
}

int64_t oracle_num_matches(const OracleEngine* e) { return (int64_t)e->matches.size(); }

// the text of string dictionary ids as (String.hashCode, UTF-16 length): a string partition key's
// String.valueOf (the fan-out order hashes it)
void oracle_set_strings(OracleEngine* e, int64_t n, const int32_t* ids, const int32_t* hash, const int32_t* len) {
  for (int64_t i = 0; i < n; ++i) e->str_info[ids[i]] = {hash[i], (int64_t)len[i]};
}

// test hook: Java 8 Float / Double.toString of raw bits (java_fp_string)
int oracle_java_fmt(uint64_t bits, int is_double, char* out, int cap) {
  const std::string t = java_fp_string(bits, is_double != 0);
  if ((int)t.size() >= cap) return -1;
  std::memcpy(out, t.c_str(), t.size() + 1);
  return (int)t.size();
}

// test hook: the iteration position of each of n keys (String.hashCode values, inserted in order)
// in the restated ConcurrentHashMap
void oracle_chm_positions(const int32_t* hashes, int64_t n, int32_t* pos) {
  JavaCHM m;
  for (int64_t k = 0; k < n; ++k) m.put(hashes[k], (int)k);
  const std::vector<int> o = m.order();
  for (size_t r = 0; r < o.size(); ++r) pos[o[r]] = (int32_t)r;
}

int64_t oracle_match_words(const OracleEngine* e) {
  int64_t w = 0;
  for (auto& m : e->matches)
    for (auto& s : m.slots) w += 1 + (int64_t)s.size();
  return w;
}

int oracle_get_matches(const OracleEngine* e, int64_t* query, int64_t* key, int64_t* ts,
                       int64_t* off, int64_t* words) {
  int64_t w = 0;
  for (size_t i = 0; i < e->matches.size(); ++i) {
    const Match& m = e->matches[i];
    query[i] = m.query;
    key[i] = m.key;
    ts[i] = m.ts;
    off[i] = w;
    for (auto& s : m.slots) {
      words[w++] = (int64_t)s.size();
      for (i64 q : s) words[w++] = q;
    }
  }
  off[e->matches.size()] = w;
  return 0;
}

// per match: the producing event's sequence number and the timer tiebreak (Match::seq, Match::tb)
int oracle_get_match_meta(const OracleEngine* e, int64_t* seq, int64_t* tb) {
  for (size_t i = 0; i < e->matches.size(); ++i) {
    seq[i] = e->matches[i].seq;
    tb[i] = e->matches[i].tb;
  }
  return 0;
}

void oracle_clear_matches(OracleEngine* e) { e->matches.clear(); }

// the runtime starts at time t (SiddhiAppRuntime.start); without it the first event or advance starts it
int oracle_start(OracleEngine* e, int64_t t) {
  try {
    if (e->started) throw std::runtime_error("already started");
    e->start(t);
    return 0;
  } catch (const std::exception& ex) {
    e->err = ex.what();
    return -1;
  }
}

int oracle_set_playback(OracleEngine* e, int on) {
  e->playback = on != 0;
  return 0;
}

// time passes to t with no event (the scheduler thread of a live runtime; a playback heartbeat)
int oracle_advance_time(OracleEngine* e, int64_t t) {
  try {
    e->cur_seq = (i64)e->log.size();
    e->advance(t);
    e->gc();
    return 0;
  } catch (const std::exception& ex) {
    e->err = ex.what();
    return -1;
  }
}

int64_t oracle_live_partials(const OracleEngine* e) {  // entries of every pending list
  int64_t n = 0;
  auto count = [&](const Runtime& r) {
    for (const auto& p : r.pres) n += (int64_t)p.pending.size();
  };
  for (const auto& r : e->top)
    if (r) count(*r);
  for (const auto& pm : e->part_inst)
    for (const auto& kv : pm)
      for (const auto& r : kv.second) count(*r);
  return n;
}

const char* oracle_error(const OracleEngine* e) { return e->err.c_str(); }

void oracle_destroy(OracleEngine* e) { delete e; }

}  // extern "C"
