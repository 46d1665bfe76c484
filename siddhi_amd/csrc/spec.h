// spec.h -- shape-compiled kernels (spec.hip).
//
// A wave runs 64 queries of one shape (kg::shape_of: the same program up to constants), so a
// shape's filters can be compiled once into straight-line code instead of being walked per event:
// spec.hip generates HIP source for the shape (one kg::sp_* call per bytecode instruction, types
// and operators as template arguments, the lane's constants loaded into registers once per work
// item), compiles it for the device with hiprtc when the engine is created, and the engine
// launches the generated kernel in place of the interpreted one. Kernel bodies are the same
// headers the static kernels instantiate (seq_body.h, part_body.h), embedded into the library at
// build time (embed_src.py).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "kgen.h"

namespace sdh {
namespace spec {

// K_seq (seq_body.h) for windows of shape g: source of kernel "sdh_seq_spec"
// out_w: words of the wave's LDS output buffer (0: the default for normal-mode output)
std::string seq_source(const kg::GQuery& g, int out_w = 0);

// K_part (part_body.h) of kind `kind` for shape g with the set's side / entry layout: source of
// kernel "sdh_part_spec"
struct PartLayout {
  int kind, sA, sB, cmax, n_e1, n_first, n_last;
  int ew;            // words per entry
  int reg_entries;   // entries of a lane's table kept in registers
  int out_w = 0;     // words of the wave's LDS output buffer (0: the default for normal-mode output)
};
std::string part_source(const kg::GQuery& g, const PartLayout& lay);

// hiprtc: src -> code object for `arch` (e.g. "gfx950"); empty and *err on failure
std::vector<char> compile(const std::string& src, const std::string& arch, std::string* err);

// Compile `src` for the current device and load it; returns kernel `name`. Cached per (device,
// source) for the life of the process. nullptr and *err on failure.
hipFunction_t get_kernel(const std::string& src, const char* name, std::string* err);

}  // namespace spec
}  // namespace sdh
