// spec.hip -- shape-compiled kernels: source generation and run-time compilation (see spec.h).
#include "knobs.h"
#include "spec.h"

#include "nfa_types.h"

#include <hip/hiprtc.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "build/spec_src.inc"  // k_spec_headers: the device headers (embed_src.py)

namespace sdh {
namespace spec {

namespace {

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

// tuning macros the generated kernels see (SDH_RING_CHUNK: device-record output reservations)
std::string tuning_defines() {
  std::string d;
  if (const char* v = sdh::knob("SDH_RING_CHUNK")) d += fmt("#define SDH_RING_CHUNK %d\n", atoi(v));
  return d;
}

// an integer knob from the environment, clamped (tuning A/Bs of the generated kernels)
int env_int(const char* env, int dflt, int lo, int hi) {
  const char* v = sdh::knob(env);
  const int n = v && *v ? atoi(v) : dflt;
  return n < lo ? lo : n > hi ? hi : n;
}

// register budget of a shape-compiled kernel: SDH_SEQ_WPE / SDH_PART_WPE = N asks for N resident
// waves per SIMD (amdgpu_waves_per_eu); unset or 0 leaves the compiler's choice
std::string wpe_attr(const char* env, int dflt) {
  const char* v = sdh::knob(env);
  const int n = v && *v ? atoi(v) : dflt;
  return n > 0 ? fmt("__attribute__((amdgpu_waves_per_eu(%d))) ", std::min(n, 8)) : std::string();
}


// hiprtc has no system headers: the fixed-width types and limits kgen.h / nfa_types.h use
const char* const kPrelude =
    "typedef __hip_internal::int8_t int8_t;\n"
    "typedef __hip_internal::uint8_t uint8_t;\n"
    "typedef __hip_internal::int16_t int16_t;\n"
    "typedef __hip_internal::uint16_t uint16_t;\n"
    "typedef __hip_internal::int32_t int32_t;\n"
    "typedef __hip_internal::uint32_t uint32_t;\n"
    "typedef __hip_internal::int64_t int64_t;\n"
    "typedef __hip_internal::uint64_t uint64_t;\n"
    "#define INT32_MIN (-2147483647 - 1)\n"
    "#define INT32_MAX 2147483647\n"
    "#define INT64_MIN (-9223372036854775807LL - 1)\n"
    "#define INT64_MAX 9223372036854775807LL\n";

// The lane's constants: one register each, loaded once per work item (ql->code[pc].imm)
struct Consts {
  std::vector<int> pcs;
  std::string use(int pc) {
    for (size_t i = 0; i < pcs.size(); ++i)
      if (pcs[i] == pc) return fmt("k.c[%zu]", i);
    pcs.push_back(pc);
    return fmt("k.c[%zu]", pcs.size() - 1);
  }
  std::string decl() const { return fmt("  struct K { int64_t c[%zu]; };\n", pcs.empty() ? (size_t)1 : pcs.size()); }
  std::string load() const {
    std::string s = "  __device__ static void load(K& k, const sdh::kg::GQuery* ql) {\n";
    if (pcs.empty()) s += "    k.c[0] = 0;\n";
    for (size_t i = 0; i < pcs.size(); ++i) s += fmt("    k.c[%zu] = ql->code[%d].imm;\n", i, pcs[i]);
    return s + "  }\n";
  }
  // from the group's lane-constant table column lc (kg::LaneConsts: slot LC_FIRST + the instruction's
  // rank among the shape's CONST instructions; one coalesced row per constant)
  std::string load_table(const kg::GQuery& g, const std::string& sig) const {
    int8_t rank[kg::GMAXCODE];
    int n = 0;
    kg::const_ranks(g, rank, &n);
    std::string s = "  __device__ static void load(K& k, const sdh::kg::GQuery* ql, " + sig + ", const int64_t* lc) {\n";
    if (pcs.empty()) s += "    k.c[0] = 0;\n";
    for (size_t i = 0; i < pcs.size(); ++i)
      s += fmt("    k.c[%zu] = lc[%d * 64];\n", i, kg::LC_FIRST + (int)rank[pcs[i]]);
    return s + "  }\n";
  }
};

// One filter (bytecode range [b, e) of g) as statements; returns the variable holding its kg::Val.
// attr(in) / stream_null(in) give the expressions for OP_ATTR (a kg::Val) and OP_STREAM_IS_NULL
// (a bool) -- what the interpreter's callbacks answer (kg::eval_code).
std::string emit_filter(const kg::GQuery& g, int b, int e, const std::string& pre, Consts& K,
                        const std::function<std::string(const kg::GInsn&)>& attr,
                        const std::function<std::string(const kg::GInsn&)>& stream_null, std::string& out) {
  std::vector<std::string> stk;
  auto pop = [&]() {
    std::string v = stk.empty() ? std::string("sdh::kg::Val{sdh::kg::T_BOOL, 1, 0}") : stk.back();
    if (!stk.empty()) stk.pop_back();
    return v;
  };
  for (int pc = b; pc < e; ++pc) {
    const kg::GInsn& in = g.code[pc];
    const std::string v = fmt("%s%d", pre.c_str(), pc);
    std::string rhs;
    switch (in.op) {
      case kg::OP_CONST: rhs = fmt("sdh::kg::sp_const<%d>(%s)", in.res, K.use(pc).c_str()); break;
      case kg::OP_ATTR: rhs = attr(in); break;
      case kg::OP_STREAM_IS_NULL: rhs = "sdh::kg::sp_bool(" + stream_null(in) + ")"; break;
      case kg::OP_IS_NULL: rhs = "sdh::kg::sp_is_null(" + pop() + ")"; break;
      case kg::OP_NOT: rhs = "sdh::kg::sp_not(" + pop() + ")"; break;
      case kg::OP_AND:
      case kg::OP_OR: {
        const std::string r = pop(), l = pop();
        rhs = fmt("sdh::kg::sp_%s(%s, %s)", in.op == kg::OP_AND ? "and" : "or", l.c_str(), r.c_str());
        break;
      }
      case kg::OP_CMP: {
        const std::string r = pop(), l = pop();
        rhs = fmt("sdh::kg::sp_cmp<%d, %d, %d>(%s, %s)", (int)in.imm, in.lt, in.rt, l.c_str(), r.c_str());
        break;
      }
      case kg::OP_ARITH: {
        const std::string r = pop(), l = pop();
        rhs = fmt("sdh::kg::sp_arith<%d, %d, %d, %d>(%s, %s)", (int)in.imm, in.res, in.lt, in.rt, l.c_str(), r.c_str());
        break;
      }
      default: rhs = "sdh::kg::Val{sdh::kg::T_BOOL, 1, 0}";
    }
    out += "    const sdh::kg::Val " + v + " = " + rhs + ";\n";
    stk.push_back(v);
  }
  if (stk.size() == 1) return stk[0];
  out += "    const sdh::kg::Val " + pre + "r = sdh::kg::Val{sdh::kg::T_BOOL, 1, 0};\n";
  return pre + "r";
}

std::string header() {
  return std::string(kPrelude) +
         "#include \"kgen.h\"\n#include \"nfa_types.h\"\n#include \"dev_common.h\"\n";
}

struct Loaded {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};

}  // namespace

// K_seq window test (kg::seq_match over a window of one-event slots): state i's filters see slots
// 0 .. i at chain index 0 / CURRENT, every other reference is null; a step i >= 1 whose event is
// more than `within` from the start event fails first (StreamPreStateProcessor.isExpired:102-113)
std::string seq_source(const kg::GQuery& g, int out_w) {
  Consts K;
  std::string body;
  for (int i = 0; i < g.n_states; ++i) {
    body += fmt("    // state %d\n", i);
    if (i >= 1 && g.within >= 0) body += fmt("    ok = ok & !w.exp(%d, within);\n", i);
    const kg::GState& st = g.st[i];
    for (int f = 0; f < st.n_filt; ++f) {
      auto here = [i](const kg::GInsn& in) { return in.a <= i && (in.b == 0 || in.b == -1); };
      const std::string r = emit_filter(
          g, st.fb[f], st.fe[f], fmt("s%df%d_", i, f), K,
          [&](const kg::GInsn& in) {
            if (!here(in)) return fmt("sdh::kg::Val{%d, 1, 0}", in.res);
            return fmt("sdh::kg::sp_attr<%d>(w.raw(%d, %d), w.null(%d, %d))", in.res, in.a, (int)in.imm, in.a, (int)in.imm);
          },
          [&](const kg::GInsn& in) { return std::string(here(in) ? "false" : "true"); }, body);
      body += "    ok = ok & sdh::kg::sp_true(" + r + ");\n";
    }
  }
  // branch-free: every state is evaluated (filters are pure and total -- /0 is null, no traps), so
  // seq_body can test several window starts at once with their LDS reads in flight together
  int na = 1;  // LDS row: ts, seq, null bits and the captured words
  for (int st = 0; st < kg::GMAXSTREAM; ++st) na = std::max(na, (int)g.n_cap[st]);
  std::string s = tuning_defines() + header() + "#include \"seq_body.h\"\n\nstruct SpecSeq {\n  static constexpr bool kBranchFree = true;\n";
  s += fmt("  static constexpr int kRow = %d, kOutW = %d;\n", 3 + std::min(na, kg::GMAXNA),
           env_int("SDH_KSEQ_OUTW", out_w > 0 ? out_w : 1024, 256, 4096) & ~15);  // (16-word LDS blocks)
  s += K.decl();
  s += K.load();
  s += "  template <class W>\n  __device__ static bool match(const K& k, const sdh::kg::GQuery*, const sdh::kg::GQuery*, "
       "int64_t within, const W& w) {\n    (void)k;\n    (void)within;\n    bool ok = true;\n";
  s += body;
  s += "    return ok;\n  }\n};\n\n";
  s += "extern \"C\" __global__ __launch_bounds__(64) " + wpe_attr("SDH_SEQ_WPE", 0) +
       "void sdh_seq_spec(sdh::SeqLaunch L) { sdh::seq_body<SpecSeq>(L); }\n";
  return s;
}

// K_part filters (part_body.h; the interpreted form is nfa_part.hip PartInterp): f1 / fa / fb / f2
// read the current event in their own state's slot only; the count chain's f3 reads e1 (slot 0),
// the chain's first (e2[0]) or last (e2[last] / e2) event (slot 1) and the current event (slot 2)
std::string part_source(const kg::GQuery& g, const PartLayout& lay) {
  Consts K;
  auto here = [](const kg::GInsn& in) { return in.b == 0 || in.b == -1; };
  auto ev_fn = [&](const char* name, int sid) {
    std::string body = fmt("  __device__ static bool %s(const K& k, const sdh::kg::GQuery*, const sdh::kg::GQuery*, "
                           "const sdh::PartLaunch&, const sdh::PartEv& ev) {\n    (void)k;\n    (void)ev;\n"
                           "    bool ok = true;\n",
                           name);
    if (sid >= 0) {
      const kg::GState& st = g.st[sid];
      for (int f = 0; f < st.n_filt; ++f) {
        const std::string r = emit_filter(
            g, st.fb[f], st.fe[f], fmt("%s%d_", name, f), K,
            [&](const kg::GInsn& in) {
              if (in.a != sid || !here(in)) return fmt("sdh::kg::Val{%d, 1, 0}", in.res);
              return fmt("sdh::kg::sp_attr<%d>(ev.word(%d), ev.null(%d))", in.res, (int)in.imm, (int)in.imm);
            },
            [&](const kg::GInsn& in) { return std::string(in.a == sid && here(in) ? "false" : "true"); }, body);
        body += "    ok = ok & sdh::kg::sp_true(" + r + ");\n";
      }
    } else {
      body += "    ok = false;\n";
    }
    return body + "    return ok;\n  }\n";
  };
  const bool logical = lay.kind != PK_COUNT;
  std::string fns = ev_fn("f1", 0);
  fns += ev_fn("fa", logical ? lay.sA : -1);
  fns += ev_fn("fb", logical ? lay.sB : -1);
  fns += ev_fn("f2", logical ? -1 : 1);
  fns += "  template <class En>\n  __device__ static bool f3(const K& k, const sdh::kg::GQuery*, const sdh::kg::GQuery*, "
         "const sdh::PartLaunch&, const sdh::PartEv& ev, const En& en) {\n    (void)k;\n    (void)ev;\n    (void)en;\n"
         "    bool ok = true;\n";
  if (!logical) {
    const kg::GState& st = g.st[2];
    for (int f = 0; f < st.n_filt; ++f) {
      const std::string r = emit_filter(
          g, st.fb[f], st.fe[f], fmt("f3%d_", f), K,
          [&](const kg::GInsn& in) {
            const int j = (int)in.imm;
            if (in.a == 2 || in.a == 0) {
              if (!here(in)) return fmt("sdh::kg::Val{%d, 1, 0}", in.res);
              if (in.a == 2) return fmt("sdh::kg::sp_attr<%d>(ev.word(%d), ev.null(%d))", in.res, j, j);
              return fmt("sdh::kg::sp_attr<%d>(en.e1(%d), en.e1_null(%d))", in.res, j, j);
            }
            const char* which = in.b == 0 ? "first" : "last";
            return fmt("sdh::kg::sp_attr<%d>(en.%s(%d), en.%s_null(%d))", in.res, which, j, which, j);
          },
          [&](const kg::GInsn&) { return std::string("false"); }, fns);
      fns += "    ok = ok & sdh::kg::sp_true(" + r + ");\n";
    }
  } else {
    fns += "    ok = false;\n";
  }
  fns += "    return ok;\n  }\n";
  std::string s = tuning_defines() + header() + "#include \"part_body.h\"\n\nstruct SpecPart {\n";
  int na = 1;  // captured words the tile staging holds
  for (int st = 0; st < kg::GMAXSTREAM; ++st) na = std::max(na, (int)g.n_cap[st]);
  s += "  static constexpr bool kHotRegs = true;  // count partials' hot words in registers (part_body.h)\n";
  s += fmt("  static constexpr int kRegEntries = %d, kEW = %d, kNA = %d, kOutW = %d;\n", lay.reg_entries, lay.ew,
           std::min(na, kg::GMAXNA), env_int("SDH_KPART_OUTW", lay.out_w > 0 ? lay.out_w : 1536, 256, 4096) & ~15);
  s += fmt("  __device__ static sdh::PartOffs offs(const sdh::PartLaunch&) { return sdh::PartOffs{%d, %d, %d, %d}; }\n",
           lay.cmax, lay.n_e1, lay.n_first, lay.n_last);
  s += K.decl();
  s += K.load_table(g, "const sdh::PartLaunch&");
  s += fns;
  s += "};\n\n";
  s += fmt("extern \"C\" __global__ __launch_bounds__(64) %svoid sdh_part_spec(sdh::PartLaunch L) {\n"
           "  sdh::part_body<%d, SpecPart>(L);\n}\n",
           wpe_attr("SDH_PART_WPE", 0).c_str(), lay.kind);
  return s;
}

// hiprtc: src -> code object for `arch` (e.g. "gfx950"); empty and *err on failure
std::vector<char> compile(const std::string& src_in, const std::string& arch, std::string* err) {
  // measurement builds: SDH_PART_PROF=1 compiles part_body's phase clocks in (engine prints them)
  const std::string src = sdh::knob("SDH_PART_PROF") ? "#define SDH_PART_PROF 1\n" + src_in : src_in;
  hiprtcProgram prog = nullptr;
  if (hiprtcCreateProgram(&prog, src.c_str(), "sdh_spec.hip", k_spec_n_headers, k_spec_headers,
                          k_spec_header_names) != HIPRTC_SUCCESS) {
    *err = "hiprtcCreateProgram failed";
    return {};
  }
  // the static kernels' floating-point contract: no contraction, IEEE denormals (Java semantics)
  const std::string a = "--offload-arch=" + arch;
  const char* opts[] = {a.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                        "-fno-gpu-flush-denormals-to-zero"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)(sizeof opts / sizeof opts[0]), opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    *err = "hiprtc: " + log.substr(0, 4000);
    return {};
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (const char* dir = sdh::knob("SDH_SPEC_DUMP")) {  // inspection: source + code object per kernel
    const size_t h = std::hash<std::string>{}(src);
    const std::string base = std::string(dir) + "/" + fmt("spec_%016zx", h);
    if (FILE* f = fopen((base + ".hip").c_str(), "w")) {
      fwrite(src.data(), 1, src.size(), f);
      fclose(f);
    }
    if (FILE* f = fopen((base + ".co").c_str(), "wb")) {
      fwrite(code.data(), 1, code.size(), f);
      fclose(f);
    }
  }
  return code;
}

hipFunction_t get_kernel(const std::string& src, const char* name, std::string* err) {
  static std::mutex mu;
  static std::map<std::pair<int, std::string>, Loaded> cache;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    *err = "no device";
    return nullptr;
  }
  std::lock_guard<std::mutex> lock(mu);
  const auto key = std::make_pair(dev, src + '\0' + name);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second.fn;
  hipDeviceProp_t prop{};
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    *err = "hipGetDeviceProperties failed";
    return nullptr;
  }
  std::string arch = prop.gcnArchName;
  const std::vector<char> code = compile(src, arch.substr(0, arch.find(':')), err);
  if (code.empty()) return nullptr;
  Loaded l;
  if (hipModuleLoadData(&l.mod, code.data()) != hipSuccess || hipModuleGetFunction(&l.fn, l.mod, name) != hipSuccess) {
    (void)hipGetLastError();
    *err = std::string("loading the compiled kernel ") + name + " failed";
    return nullptr;
  }
  cache[key] = l;
  return l.fn;
}

}  // namespace spec
}  // namespace sdh

// Build check without a device (tests/test_abi.py): the generated K_seq and K_part kernels of
// representative shapes (filterless 3-state windows / partials; every K_part kind, register tables
// on and off) compile for gfx950. Returns the number compiled, or -1 with the first log in `log`.
extern "C" int sdh_spec_selftest(char* log, size_t cap) {
  using namespace sdh;
  kg::GQuery g{};
  g.n_states = 3;
  g.within = 0;
  std::vector<std::string> srcs{spec::seq_source(g)};
  for (int kind = PK_OR; kind <= PK_COUNT; ++kind)
    for (int regs : {0, 4}) {
      const int ew = kind == PK_COUNT ? 3 + 5 + 1 + 1 + 1 : 3;
      srcs.push_back(spec::part_source(g, spec::PartLayout{kind, 1, 2, 5, 1, 1, 1, ew, regs}));
    }
  int ok = 0;
  for (const auto& src : srcs) {
    std::string err;
    if (spec::compile(src, "gfx950", &err).empty()) {
      if (log && cap) snprintf(log, cap, "%s", err.c_str());
      return -1;
    }
    ++ok;
  }
  return ok;
}
