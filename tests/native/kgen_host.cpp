// kgen_host.cpp -- TEST INFRASTRUCTURE ONLY: the K_gen interpreter (siddhi_amd/csrc/kgen.h, the
// per-lane body of the device kernel) compiled for the host with one lane per instance, driven the
// way nfa_gen.hip drives it (instances own the whole batch; matches re-ordered by the output
// sort key), so the restatement can be cross-checked against the oracle and the reference KATs on
// a machine without a GPU. Never part of the product path (libsiddhi_hip.so does not link it).
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../../siddhi_amd/csrc/chm_order.h"
#include "../../siddhi_amd/csrc/java_fmt.h"
#include "../../siddhi_amd/csrc/gen_lower.h"

using namespace sdh::kg;

namespace {

struct Rec {
  int64_t seq, rank, idx;
  int64_t tts = 0;  // timer records (rank -1): the timer's time, ordered before idx
  int64_t fpos = -1, frank = 0;  // fan-out records: the key's map position, the query's rank in it
  int64_t query, key, ts;
  std::vector<std::vector<int64_t>> slots;
};

struct Inst {
  int qi;
  int64_t key;
  int64_t timer_idx = 0;  // fire ordinal of this instance's timer matches
  std::vector<int32_t> w32;
  std::vector<int64_t> w64;
  bool init = false;
};

struct Host {
  LProgram P;
  std::vector<GQuery> gq;  // per query
  std::vector<int> rank;
  std::vector<std::unique_ptr<Inst>> top;                       // unpartitioned instances
  std::vector<std::map<int64_t, std::vector<std::unique_ptr<Inst>>>> part;
  std::vector<std::vector<int64_t>> korder;  // per partition: keys in creation order
  std::vector<char> kkind;                   //   key values: 0 int / long, 1 bool, 3 float, 4 double
  std::vector<Rec> out;
  std::string err;
  int64_t chunk_len = 0;  // >0: unpartitioned instances with a bounded look-back run event chunks
                          // like the device (kg::seq_lookback; nfa_gen.hip)
  bool window = false;    // unpartitioned K_seq-class instances evaluate event windows (kg::seq_match)
  bool started = false;   // absent states: the runtime's start time, playback mode
  int64_t start_ts = 0;
  bool playback = false;
  // last events of each stream (window mode): ts, seq, raw attribute words, null flags
  struct Ev {
    int64_t ts, seq;
    std::vector<int64_t> v;
    std::vector<uint8_t> nl;
  };
  std::map<int, std::vector<Ev>> tail;
};

struct HostWin {  // kg::seq_match's window over Host::Ev records
  static constexpr bool kStagedConsts = false;
  int64_t lane_const(int) const { return 0; }
  const std::vector<Host::Ev>* ev;
  size_t s;
  const int32_t* cap;
  int64_t ts(int p) const { return (*ev)[s + p].ts; }
  int64_t raw(int p, int j, bool = false) const { return (*ev)[s + p].v[cap[j]]; }
  bool null(int p, int j, bool = false) const { return (*ev)[s + p].nl[cap[j]] != 0; }
};

Inst* make_inst(Host* h, int qi, int64_t key) {
  auto* in = new Inst;
  in->qi = qi;
  in->key = key;
  in->w32.assign(h->gq[qi].lay.n32, 0);
  in->w64.assign(h->gq[qi].lay.n64, 0);
  return in;
}

// run one event through one instance (what one lane does for one event): the absent states'
// timers due by the event fire first (nfa_gen.hip); event == false: only time passes, to `upto`
void run(Host* h, Inst* in, int stream, int64_t seq, int64_t ts, const int64_t* vals, const uint8_t* nulls,
         bool live = true, bool event = true, int64_t upto = 0, int64_t fpos = -1) {
  const GQuery& q = h->gq[in->qi];
  Ctx c{};
  c.bind(&q, &q);
  c.w32 = in->w32.data();
  c.w64 = in->w64.data();
  c.stride = 1;
  int32_t hot32[3 * GMAXS];
  int64_t hot64[1 + GMAXNU];
  c.h32 = hot32;
  c.h64 = hot64;
  c.hstride = 1;
  c.hs = GMAXS;
  c.load_hot();
  int64_t evv[GMAXNA];
  int32_t pins[4];
  c.ev_val = evv;
  c.pins = pins;
  c.npin = 0;
  c.n_ret = 0;
  c.err = GE_OK;
  if (!in->init) {
    c.seq = seq;
    c.ts = ts;
    c.stream = stream;
    c.init_instance();
    if (in->key == -1 && h->gq[in->qi].partition < 0) c.start_instance(h->start_ts);  // clones never start
    in->init = true;
  }
  c.seq = seq;
  c.ts = event ? ts : upto;
  c.stream = stream;
  c.ev_null = 0;
  for (int j = 0; event && j < q.n_cap[stream]; ++j) {
    const int a = q.cap_attr[stream][j];
    evv[j] = vals[a];
    if (nulls && nulls[a]) c.ev_null |= 1u << j;
  }
  int64_t idx = 0;
  auto emit = [&](const Ctx& cx, int se) {
    if (!live) return;  // look-back replay of an event chunk
    Rec r;
    r.seq = seq;
    if (cx.in_timer) {
      r.rank = -1;
      r.tts = cx.timer_ts;
      r.idx = in->timer_idx++;
    } else {
      r.rank = h->rank[(size_t)in->qi * h->P.stream_types.size() + stream];
      r.idx = idx++;
      if (fpos >= 0) {  // fan-out: (partition's first rank, key position, rank in the partition)
        const int ns = (int)h->P.stream_types.size();
        int base = r.rank;
        for (int pq : h->P.parts[h->P.q[in->qi].partition].queries) base = std::min(base, h->rank[(size_t)pq * ns + stream]);
        r.frank = r.rank - base;
        r.rank = base;
        r.fpos = fpos;
      }
    }
    r.query = in->qi;
    r.key = in->key;
    r.ts = cx.se_ts(se);
    for (int i = 0; i < cx.nS(); ++i) {
      std::vector<int64_t> ch;
      for (int n = cx.slot(se, i); n >= 0; n = cx.nd_next(n)) ch.push_back(cx.nd_seq(n));
      r.slots.push_back(ch);
    }
    h->out.push_back(r);
  };
  c.fire_timers(event ? ts : upto, h->playback, emit);
  if (event && c.err == GE_OK) c.receive(emit);
  c.store_hot();
  if (c.err == GE_CAPACITY)
    throw std::runtime_error("K_gen instance capacity exceeded (kinds " + std::to_string(c.capk) + ")");
  if (c.err == GE_REFERENCE) throw std::runtime_error("reference engine would throw here");
}

void sort_out(Host* h) {
  std::stable_sort(h->out.begin(), h->out.end(), [](const Rec& a, const Rec& b) {
    if (a.seq != b.seq) return a.seq < b.seq;
    if (a.rank != b.rank) return a.rank < b.rank;
    if (a.rank == -1 && a.tts != b.tts) return a.tts < b.tts;
    if (a.rank == -1 && a.query != b.query) return a.query < b.query;
    if (a.rank == -1 && a.key != b.key) return a.key < b.key;
    if (a.fpos != b.fpos) return a.fpos < b.fpos;
    if (a.frank != b.frank) return a.frank < b.frank;
    return a.idx < b.idx;
  });
}

}  // namespace

extern "C" {

// test hook: chm_order.h positions of n keys inserted in order
void kgh_chm_positions(const int32_t* hashes, int64_t n, int32_t* pos) {
  const std::vector<int32_t> p = sdh::ChmOrder().positions(std::vector<int32_t>(hashes, hashes + n));
  for (int64_t k = 0; k < n; ++k) pos[k] = p[(size_t)k];
}


void* kgh_create(const void* blob, size_t len, int R, int N, int LC) {
  try {
    auto* h = new Host;
    h->P = read_program(blob, len);
    Sizing sz;
    if (R > 0) sz.R = R;
    if (N > 0) sz.N = N;
    if (LC > 0) sz.LC = LC;
    for (int qi = 0; qi < (int)h->P.q.size(); ++qi) h->gq.push_back(lower_gen(h->P, qi, sz));
    h->rank = output_ranks(h->P);
    h->top.resize(h->P.q.size());
    for (int qi = 0; qi < (int)h->P.q.size(); ++qi)
      if (h->P.q[qi].partition < 0) h->top[qi].reset(make_inst(h, qi, -1));
    h->part.resize(h->P.parts.size());
    h->korder.resize(h->P.parts.size());
    h->kkind.resize(h->P.parts.size(), 0);
    return h;
  } catch (const std::exception&) {
    return nullptr;
  }
}

// events are delivered one at a time (per-event sends), like sdh_engine_push
int kgh_send(void* hp, int stream, int64_t n, int64_t seq0, const int64_t* ts, const int64_t* vals,
             const uint8_t* nulls) {
  Host* h = (Host*)hp;
  try {
    const size_t na = h->P.stream_types[stream].size();
    if (!h->started && n > 0) {
      h->started = true;
      h->start_ts = ts[0];
    }
    // every instance processes the whole batch (the device order), then matches are sorted
    std::vector<Host::Ev> win;  // this stream's tail ++ batch (window mode)
    if (h->window) {
      win = h->tail[stream];
      for (int64_t k = 0; k < n; ++k) {
        Host::Ev e{ts[k], seq0 + k, std::vector<int64_t>(vals + k * na, vals + (k + 1) * na),
                   std::vector<uint8_t>(na, 0)};
        if (nulls)
          for (size_t a = 0; a < na; ++a) e.nl[a] = nulls[k * na + a];
        win.push_back(e);
      }
    }
    const int64_t t0 = (int64_t)win.size() - n;  // window index of batch event 0
    for (auto& in : h->top) {
      if (!in) continue;
      const int S = h->window ? seq_window(h->gq[in->qi]) : -1;
      if (S > 0) {
        const GQuery& q = h->gq[in->qi];
        if (q.recv_n[stream] == 0) continue;
        for (int64_t k = 0; k < n; ++k) {  // the window ending at batch event k
          const int64_t s = t0 + k - (S - 1);
          if (s < 0) continue;  // fewer than S events seen so far
          HostWin w{&win, (size_t)s, q.cap_attr[stream]};
          if (!seq_match(&q, &q, q.within, w)) continue;
          Rec r;
          r.seq = seq0 + k;
          r.rank = h->rank[(size_t)in->qi * h->P.stream_types.size() + stream];
          r.idx = 0;
          r.query = in->qi;
          r.key = in->key;
          r.ts = ts[k];
          for (int i = 0; i < q.n_states; ++i) r.slots.push_back({win[s + i].seq});
          h->out.push_back(r);
        }
        continue;
      }
      const int look = seq_lookback(h->gq[in->qi]);
      const int64_t clen = h->chunk_len > 0 ? std::max<int64_t>(h->chunk_len, look) : n;
      if (look < 0 || h->gq[in->qi].recv_n[stream] == 0 || clen >= n) {
        for (int64_t k = 0; k < n; ++k)
          run(h, in.get(), stream, seq0 + k, ts[k], vals + k * na, nulls ? nulls + k * na : nullptr);
        continue;
      }
      // chunk 0 continues the instance; chunk c > 0 starts a fresh one and replays `look` events;
      // the last chunk's instance carries on (the device copies its arena back)
      for (int64_t e0 = 0; e0 < n; e0 += clen) {
        std::unique_ptr<Inst> fresh;
        Inst* cur = in.get();
        if (e0 > 0) {
          fresh.reset(make_inst(h, in->qi, in->key));
          cur = fresh.get();
        }
        const int64_t e1 = std::min(n, e0 + clen);
        for (int64_t k = e0 > 0 ? e0 - look : 0; k < e1; ++k)
          run(h, cur, stream, seq0 + k, ts[k], vals + k * na, nulls ? nulls + k * na : nullptr, k >= e0);
        if (e1 == n && fresh) in = std::move(fresh);
      }
    }
    // partitions: each event goes to its key's clones (created at the key's first event); every
    // other key's clones with absent states only see time pass (their timers due by the event fire)
    for (size_t pi = 0; pi < h->P.parts.size(); ++pi) {
      const LPart& pd = h->P.parts[pi];
      int attr = -1;
      for (const auto& key : pd.keys)
        if (key.stream == stream) attr = (int)key.code[0].imm;
      if (const LFanOut* fo = pd.fan(stream)) {  // every key's instances, in the map's order
        std::vector<int32_t> hs;
        const int kk = h->kkind[pi];
        for (int64_t kv : h->korder[pi])
          hs.push_back(sdh::java_hash_cat(fo->id_hash, kk == 3   ? sdh::jfmt::float_to_string((uint32_t)kv)
                                                       : kk == 4 ? sdh::jfmt::double_to_string((uint64_t)kv)
                                                                 : sdh::java_value_of(kk == 1, kv)));
        const std::vector<int32_t> pos = sdh::ChmOrder().positions(hs);
        for (int64_t k = 0; k < n; ++k)
          for (size_t j = 0; j < h->korder[pi].size(); ++j)
            for (auto& in : h->part[pi].at(h->korder[pi][j]))
              run(h, in.get(), stream, seq0 + k, ts[k], vals + k * na, nulls ? nulls + k * na : nullptr, true, true, 0,
                  pos[j]);
        continue;
      }
      for (int64_t k = 0; k < n; ++k) {
        bool has_key = attr >= 0 && !(nulls && nulls[k * na + attr]);  // a null key drops the event
        int64_t kv = 0;
        if (has_key) {
          kv = key_of_raw(h->P.stream_types[stream][attr], vals[k * na + attr]);
          if (h->part[pi].find(kv) == h->part[pi].end()) {
            std::vector<std::unique_ptr<Inst>> v;
            for (int pq : pd.queries) v.emplace_back(make_inst(h, pq, kv));
            h->part[pi].emplace(kv, std::move(v));
            h->korder[pi].push_back(kv);
            const int ty = h->P.stream_types[stream][attr];
            h->kkind[pi] = ty == T_BOOL ? 1 : ty == T_FLOAT ? 3 : ty == T_DOUBLE ? 4 : 0;
          }
        }
        for (auto& kvp : h->part[pi])
          for (auto& in : kvp.second) {
            if (has_key && kvp.first == kv)
              run(h, in.get(), stream, seq0 + k, ts[k], vals + k * na, nulls ? nulls + k * na : nullptr);
            else if (in->init && h->gq[in->qi].lay.TQ > 0)
              run(h, in.get(), stream, seq0 + k, ts[k], nullptr, nullptr, true, false, ts[k]);
          }
      }
    }
    if (h->window) {
      const size_t keep = std::min<size_t>(win.size(), GMAXS - 1);
      h->tail[stream].assign(win.end() - keep, win.end());
    }
    sort_out(h);
    return 0;
  } catch (const std::exception& ex) {
    h->err = ex.what();
    return -1;
  }
}

int64_t kgh_num_matches(void* hp) { return (int64_t)((Host*)hp)->out.size(); }
int64_t kgh_match_words(void* hp) {
  int64_t w = 0;
  for (auto& r : ((Host*)hp)->out)
    for (auto& s : r.slots) w += 1 + (int64_t)s.size();
  return w;
}
int kgh_get_matches(void* hp, int64_t* query, int64_t* key, int64_t* ts, int64_t* off, int64_t* words) {
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
void kgh_clear(void* hp) { ((Host*)hp)->out.clear(); }
void kgh_start(void* hp, int64_t t) {
  ((Host*)hp)->started = true;
  ((Host*)hp)->start_ts = t;
}
void kgh_set_playback(void* hp, int on) { ((Host*)hp)->playback = on != 0; }
// time passes to t with no event (sdh_engine_advance_time): timer records get trigger seq `seq`
int kgh_advance(void* hp, int64_t t, int64_t seq) {
  Host* h = (Host*)hp;
  try {
    if (!h->started) {
      h->started = true;
      h->start_ts = t;
    }
    for (auto& in : h->top)
      if (in && h->gq[in->qi].lay.TQ > 0) run(h, in.get(), 0, seq, t, nullptr, nullptr, true, false, t);
    for (auto& pm : h->part)
      for (auto& kvp : pm)
        for (auto& in : kvp.second)
          if (in->init && h->gq[in->qi].lay.TQ > 0) run(h, in.get(), 0, seq, t, nullptr, nullptr, true, false, t);
    sort_out(h);
    return 0;
  } catch (const std::exception& ex) {
    h->err = ex.what();
    return -1;
  }
}
void kgh_set_chunk(void* hp, int64_t len) { ((Host*)hp)->chunk_len = len; }
void kgh_set_window(void* hp, int on) { ((Host*)hp)->window = on != 0; }
const char* kgh_error(void* hp) { return ((Host*)hp)->err.c_str(); }
void kgh_destroy(void* hp) { delete (Host*)hp; }

}  // extern "C"

#ifdef KG_PROFILE
// access census by arena field (test infrastructure: sizes the device's arena traffic)
namespace sdh { namespace kg {
int64_t g_prof[16];
int g_prof_phase = 0;
void kg_prof_hit(const GLayout& L, int is64, int off) {
  if (g_prof_phase) { ++g_prof[15]; return; }
  int r;
  if (!is64) {
    const int b[] = {L.o_flags, L.o_pn, L.o_nn, L.o_plist, L.o_nlist, L.o_seslot, L.o_ndnext, L.o_ndnull, L.o_init};
    r = 0;
    for (int k = 0; k < 9; ++k) if (off >= b[k]) r = k;
    if (L.v32 && off >= L.o_ndval) r = 14;
  } else {
    const int b[] = {L.o_seused, L.o_ndused, L.o_sets, L.o_ndseq, L.o_ndts, L.o_ndval};
    r = 9;
    for (int k = 0; k < 6; ++k) if (off >= b[k]) r = 9 + k;
  }
  ++g_prof[r];
}
}}
extern "C" void kgh_prof(int64_t* out) {
  for (int k = 0; k < 16; ++k) { out[k] = sdh::kg::g_prof[k]; sdh::kg::g_prof[k] = 0; }
}
#endif

// test hook: Java 8 Float / Double.toString of raw bits (java_fmt.h), into out (cap bytes)
extern "C" int kgh_java_fmt(uint64_t bits, int is_double, char* out, int cap) {
  const std::string t = is_double ? sdh::jfmt::double_to_string(bits) : sdh::jfmt::float_to_string((uint32_t)bits);
  if ((int)t.size() >= cap) return -1;
  std::memcpy(out, t.c_str(), t.size() + 1);
  return (int)t.size();
}
