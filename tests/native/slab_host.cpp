// slab_host.cpp -- TEST INFRASTRUCTURE ONLY: the K_slab per-partial semantics (siddhi_amd/csrc/
// slab.h, the per-lane body of nfa_slab.hip) run on the host, one instance (query, key) at a time
// the way one lane of the device kernel runs it: entries stepped in storage order per event,
// arrivals in the next element ranked by their position in the list they leave, new partials
// appended, dead entries dropped when the push ends; matches ordered by the device table's key
// (trigger seq, receiver rank, emission index = list position). Lets the restatement be checked
// against the oracle without a GPU. Never part of the product path.
#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../siddhi_amd/csrc/slab_lower.h"

using namespace sdh;
using namespace sdh::slab;

namespace {

struct Rec {
  int64_t seq, rank, idx, query, key, ts;
  std::vector<std::vector<int64_t>> slots;
};

struct Host {
  kg::LProgram P;
  std::vector<kg::GQuery> gq;
  std::vector<Shape> shape;
  std::vector<int> rank;
  // per partition: key -> per partition query its entries (EW words each)
  std::vector<std::map<int64_t, std::vector<std::vector<uint32_t>>>> inst;
  std::vector<Rec> out;
  std::string err;
};

void step_instance(Host* h, int qi, int64_t key, std::vector<uint32_t>& ent, int stream, int64_t seq, int64_t ts,
                   const int64_t* vals, const uint8_t* nulls) {
  const kg::GQuery& q = h->gq[qi];
  const Shape& sh = h->shape[qi];
  const int st = sh.proc[stream];
  if (st < 0) return;
  const int EW = sh.EW;
  int64_t w[kg::GMAXNA];
  uint32_t nb = 0;
  for (int j = 0; j < q.n_cap[stream]; ++j) {
    const int a = q.cap_attr[stream][j];
    w[j] = vals[a];
    if (nulls && nulls[a]) nb |= 1u << j;
  }
  const Ev ev{ts, seq, w, 1, nb};
  const int n = (int)(ent.size() / EW);
  if (st == 0) {
    bool marker = false, any = false;
    uint32_t mx = 0;
    for (int k = 0; k < n; ++k) {
      const uint32_t* e = &ent[(size_t)k * EW];
      if (e[0] & EF_MARKER) marker = true;
      bool in1 = false;
      for (int x = 0; x < 2; ++x)
        if (sh.nxt[0][x] >= 0 && (e[0] & in_bit(sh.nxt[0][x]))) in1 = true;
      if (in1) {
        mx = (!any || pos_of(e, 1) > mx) ? pos_of(e, 1) : mx;
        any = true;
      }
    }
    if (!(sh.every || !marker)) return;
    if (!start_pass(sh, &q, kg::LaneConsts{&q, nullptr}, ev)) return;
    ent.resize(ent.size() + EW);
    open_partial(sh, &ent[(size_t)n * EW], 0, any ? mx + 1 : 0, ev);
    if (!sh.every) {
      ent.resize(ent.size() + EW, 0);
      ent[(size_t)(n + 1) * EW] = EF_MARKER;
    }
    return;
  }
  bool moved = false;
  for (int k = 0; k < n; ++k) {
    uint32_t* e = &ent[(size_t)k * EW];
    const int r = step(sh, &q, kg::LaneConsts{&q, nullptr}, st, e, ev, q.within);
    if (r & R_EMIT) {
      const int words = record_words(sh, e, st);
      std::vector<int64_t> rr(words);
      write_record(sh, e, st, words, qi, key, (int64_t)pos_of(e, sh.elem[st]), stream, ev, rr.data());
      Rec rc;
      rc.seq = seq;
      rc.rank = h->rank[(size_t)qi * h->P.stream_types.size() + stream];
      rc.idx = rr[5];
      rc.query = qi;
      rc.key = key;
      rc.ts = rr[3];
      int p = 7;
      for (int j = 0; j < sh.S; ++j) {
        const int c = (int)rr[p++];
        rc.slots.emplace_back(rr.begin() + p, rr.begin() + p + c);
        p += c;
      }
      h->out.push_back(rc);
    }
    if (r & R_MOVE) {
      e[0] |= EF_MOVED;
      moved = true;
    }
  }
  if (moved) {
    const int ne = sh.elem[st] + 1, es = sh.elem[st];
    const int n0 = sh.nxt[st][0], n1 = sh.nxt[st][1];
    uint32_t mx = 0;
    bool any = false;
    for (int k = 0; k < n; ++k) {
      const uint32_t* e = &ent[(size_t)k * EW];
      if ((e[0] & EF_MOVED) || !((e[0] & in_bit(n0)) || (n1 >= 0 && (e[0] & in_bit(n1))))) continue;
      mx = (!any || pos_of(e, ne) > mx) ? pos_of(e, ne) : mx;
      any = true;
    }
    const uint32_t base = any ? mx + 1 : 0;
    for (int k = 0; k < n; ++k) {
      uint32_t* e = &ent[(size_t)k * EW];
      if (!(e[0] & EF_MOVED)) continue;
      uint32_t rank = 0;
      for (int k2 = 0; k2 < n; ++k2) {
        const uint32_t* e2 = &ent[(size_t)k2 * EW];
        if ((e2[0] & EF_MOVED) && pos_of(e2, es) < pos_of(e, es)) ++rank;
      }
      set_pos(e, ne, base + rank);
      e[0] |= in_bit(n0) | (n1 >= 0 ? in_bit(n1) : 0u);
    }
    for (int k = 0; k < n; ++k) ent[(size_t)k * EW] &= ~EF_MOVED;
  }
}

// the push is over: entries in no list (and not markers) are dropped (the kernel's write-back)
void compact(const Shape& sh, std::vector<uint32_t>& ent) {
  const int EW = sh.EW, n = (int)(ent.size() / EW);
  int w = 0;
  for (int k = 0; k < n; ++k) {
    const uint32_t f = ent[(size_t)k * EW];
    if (!((f & EF_INLIST) || (f & EF_MARKER))) continue;
    if (w != k) std::copy(ent.begin() + (size_t)k * EW, ent.begin() + (size_t)(k + 1) * EW, ent.begin() + (size_t)w * EW);
    ++w;
  }
  ent.resize((size_t)w * EW);
}

}  // namespace

extern "C" {

// every query must be a K_slab shape; otherwise null with the reason in *why (cap bytes)
void* slh_create(const void* blob, size_t len, char* why, size_t cap) {
  try {
    auto* h = new Host;
    h->P = kg::read_program(blob, len);
    kg::Sizing sz;
    for (int qi = 0; qi < (int)h->P.q.size(); ++qi) {
      h->gq.push_back(kg::lower_gen(h->P, qi, sz));
      Shape s;
      std::string w;
      if (!shape_of_query(h->P, qi, h->gq.back(), &s, &w)) {
        snprintf(why, cap, "query %d: %s", qi, w.c_str());
        delete h;
        return nullptr;
      }
      h->shape.push_back(s);
    }
    h->rank = kg::output_ranks(h->P);
    h->inst.resize(h->P.parts.size());
    return h;
  } catch (const std::exception& ex) {
    snprintf(why, cap, "%s", ex.what());
    return nullptr;
  }
}

int slh_send(void* hp, int stream, int64_t n, int64_t seq0, const int64_t* ts, const int64_t* vals,
             const uint8_t* nulls) {
  Host* h = (Host*)hp;
  try {
    const size_t na = h->P.stream_types[stream].size();
    for (size_t pi = 0; pi < h->P.parts.size(); ++pi) {
      const kg::LPart& pd = h->P.parts[pi];
      int attr = -1;
      for (const auto& key : pd.keys)
        if (key.stream == stream) attr = (int)key.code[0].imm;
      if (attr < 0) continue;
      std::map<int64_t, bool> touched;
      for (int64_t k = 0; k < n; ++k) {
        if (nulls && nulls[k * na + attr]) continue;  // a null key drops the event
        const int64_t kv = kg::key_of_raw(h->P.stream_types[stream][attr], vals[k * na + attr]);
        auto& v = h->inst[pi][kv];
        if (v.empty()) v.resize(pd.queries.size());
        touched[kv] = true;
        for (size_t j = 0; j < pd.queries.size(); ++j)
          step_instance(h, pd.queries[j], kv, v[j], stream, seq0 + k, ts[k], vals + k * na,
                        nulls ? nulls + k * na : nullptr);
      }
      for (auto& kvp : touched) {
        auto& v = h->inst[pi][kvp.first];
        for (size_t j = 0; j < pd.queries.size(); ++j) compact(h->shape[pd.queries[j]], v[j]);
      }
    }
    std::stable_sort(h->out.begin(), h->out.end(), [](const Rec& a, const Rec& b) {
      if (a.seq != b.seq) return a.seq < b.seq;
      if (a.rank != b.rank) return a.rank < b.rank;
      return a.idx < b.idx;
    });
    return 0;
  } catch (const std::exception& ex) {
    h->err = ex.what();
    return -1;
  }
}

int64_t slh_live(void* hp) {
  Host* h = (Host*)hp;
  int64_t n = 0;
  for (size_t pi = 0; pi < h->inst.size(); ++pi)
    for (auto& kv : h->inst[pi])
      for (size_t j = 0; j < kv.second.size(); ++j) {
        const Shape& sh = h->shape[h->P.parts[pi].queries[j]];
        for (size_t k = 0; k < kv.second[j].size(); k += sh.EW)
          if (!(kv.second[j][k] & EF_MARKER)) ++n;
      }
  return n;
}
int64_t slh_num_matches(void* hp) { return (int64_t)((Host*)hp)->out.size(); }
int64_t slh_match_words(void* hp) {
  int64_t w = 0;
  for (auto& r : ((Host*)hp)->out)
    for (auto& s : r.slots) w += 1 + (int64_t)s.size();
  return w;
}
int slh_get_matches(void* hp, int64_t* query, int64_t* key, int64_t* ts, int64_t* off, int64_t* words) {
  Host* h = (Host*)hp;
  int64_t w = 0;
  for (size_t i = 0; i < h->out.size(); ++i) {
    const Rec& r = h->out[i];
    query[i] = r.query;
    key[i] = r.key;
    ts[i] = r.ts;
    off[i] = w;
    for (auto& s : r.slots) {
      words[w++] = (int64_t)s.size();
      for (int64_t x : s) words[w++] = x;
    }
  }
  off[h->out.size()] = w;
  return 0;
}
void slh_clear(void* hp) { ((Host*)hp)->out.clear(); }
const char* slh_error(void* hp) { return ((Host*)hp)->err.c_str(); }
void slh_destroy(void* hp) { delete (Host*)hp; }

}  // extern "C"
