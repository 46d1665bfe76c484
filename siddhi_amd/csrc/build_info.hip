// build_info.hip -- provenance of the built library: the hash of the sources it was compiled from
// (src_hash.py, passed in by the Makefile), so a run can show that the .so it loaded matches its tree.
#ifndef SDH_SRC_HASH
#define SDH_SRC_HASH "unknown"
#endif

extern "C" const char* sdh_build_info(void) { return "src " SDH_SRC_HASH " gfx950"; }
