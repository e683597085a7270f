// jit.hpp — the scenario compiler (jit.cpp), internal to libtimewarp.so.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/timewarp.h"

namespace tw {

// Compile the event kernel (engine_dev.hpp's tw_run_kernel) for a program
// image: `inst` are template argument lists of tw_run_kernel without its last
// (JIT) argument, one kernel each; `defs` the -D options of the library's own
// build (so both kernels see the same configuration).  On TW_OK, `code` is a
// gfx950 code object and `names[i]` the symbol of kernel i.  Cached in process
// (and under $TW_JIT_CACHE when set); *compile_ms is 0 on a cache hit.
__attribute__((visibility("hidden"))) int jit_compile(const tw_insn* insns, uint32_t n_insns,
                                                      const std::vector<std::string>& inst,
                                                      const std::vector<std::string>& defs, std::string* code,
                                                      std::vector<std::string>* names, double* compile_ms);

}  // namespace tw
